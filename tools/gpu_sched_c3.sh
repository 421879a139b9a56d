# C3 matcher under other LLVM scheduler settings (build variants), interleaved, checksums
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/sched_c3; mkdir -p $O
for r in 1 2 3; do
  for v in base ilp memcl bias0 bias100; do
    L=""; [ $v != base ] && L=tools/variants/lib$v.so
    SOD_LIB_PATH=$L timeout -k 10 200 python3 tools/ab_i8.py 50000 1000 40 1 > $O/${v}_$r.log 2>&1 || { tail -5 $O/${v}_$r.log; exit 1; }
    echo "$v r$r $(tail -1 $O/${v}_$r.log)"
  done
done
