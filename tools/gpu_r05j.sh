# round-5 check: GPU parity suite, smoke, default bench line (C3 + main.py extras)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-r05j}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -c "import torch; print('torch', torch.__version__)" > $O/torch_warm.log 2>&1 || { tail -5 $O/torch_warm.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench_c3.json
echo bench done
