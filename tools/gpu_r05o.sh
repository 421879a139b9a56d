# round-5 check: GPU suite, smoke, default bench line (C3 + main.py extras), img1 / c2 lines,
# rocprofv3 kernel stats of the C3 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-r05o}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -c "import torch; print('torch', torch.__version__)" > $O/torch_warm.log 2>&1 || { tail -5 $O/torch_warm.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench_c3.json
for CFG in img1 c2; do
  timeout -k 10 300 python3 bench.py --config $CFG --no-cpu-baseline > $O/bench_$CFG.log 2>&1 || { tail -20 $O/bench_$CFG.log; exit 1; }
  grep '^{' $O/bench_$CFG.log > $O/bench_$CFG.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o c3 --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-extras > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo done
