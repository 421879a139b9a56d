# GPU suite then the one-image latency probes + timelines.  usage: TAG [configs]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-r04lat}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
# the first import of torch on a fresh box pages the image in (minutes): before the suite
timeout -k 10 400 python3 -u -c "import torch; print('torch', torch.__version__)" > $O/torch_warm.log 2>&1 || { tail -5 $O/torch_warm.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_latency.sh $T "${2:-img1 c2 c3}"
