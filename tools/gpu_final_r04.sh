# round-4 evidence: GPU parity suite, smoke, default bench line (C3 + extras), rocprofv3
# kernel stats + timed-window matcher stats (C3), c2 / img1 bench lines, PMC passes of the
# matcher for C3, C2 and one query image.  usage: tools/gpu_final_r04.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-r04f}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
# the first import of torch on a fresh box pages the image in (minutes): before the suite
timeout -k 10 400 python3 -u -c "import torch; print('torch', torch.__version__)" > $O/torch_warm.log 2>&1 || { tail -5 $O/torch_warm.log; exit 1; }
SOD_DEBUG_SYNC=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_r03d.sh $T || exit 1
