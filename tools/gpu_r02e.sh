set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02e; export TMPDIR=/tmp
: > gpurun_out/r02e/ab.log
for a in "10000 100 40 0" "500 1000 40 1" "2000 1000 40 1" "50000 1000 40 1" "20000 1000 40 1"; do
  for q in 8 4 2; do
    echo -n "QT=$q $a: " >> gpurun_out/r02e/ab.log
    SOD_MATCH_QT=$q timeout -k 10 120 python3 tools/ab_i8.py $a >> gpurun_out/r02e/ab.log 2>&1 || { tail -5 gpurun_out/r02e/ab.log; exit 1; }
  done
done
cat gpurun_out/r02e/ab.log
