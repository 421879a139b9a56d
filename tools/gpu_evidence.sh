# a round's closing evidence on one box: smoke, the default bench line (C3 + extras + CPU
# baselines), img1 / c2 lines, rocprofv3 kernel stats of the C3 bench, PMC passes of the
# matcher at c3 / c2 / img1.   usage: bash tools/gpu_evidence.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-evidence}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -c "import torch" > /dev/null 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench_c3.json
for CFG in img1 c2; do
  timeout -k 10 300 python3 bench.py --config $CFG --no-cpu-baseline --no-extras > $O/bench_$CFG.log 2>&1 || { tail -20 $O/bench_$CFG.log; exit 1; }
  grep '^{' $O/bench_$CFG.log > $O/bench_$CFG.json
done
echo benches done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o c3 --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-extras > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo rocprof done
for CFG in c3 c2 img1; do
  bash tools/gpu_pmc.sh $CFG i8 || exit 1
  mv gpurun_out/pmc_match_i8_kernel_$CFG $O/ || exit 1
  echo pmc $CFG done
done
