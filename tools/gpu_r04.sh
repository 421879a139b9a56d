# round-4 evidence: GPU parity suite, smoke, default bench line (C3 + extras), img1 / c2
# bench lines.  usage: tools/gpu_r04.sh TAG [notests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-r04}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
if [ "$2" != notests ]; then
# the first import of torch on a fresh box pages the image in (minutes): before the suite
timeout -k 10 400 python3 -u -c "import torch; print('torch', torch.__version__)" > $O/torch_warm.log 2>&1 || { tail -5 $O/torch_warm.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench_c3.json
for CFG in c2 img1; do
  timeout -k 10 200 python3 bench.py --config $CFG --no-cpu-baseline --no-extras > $O/bench_$CFG.log 2>&1 || { tail -20 $O/bench_$CFG.log; exit 1; }
  grep '^{' $O/bench_$CFG.log > $O/bench_$CFG.json
done
echo benches done
