# fused Hough/select tests, then the latency probes.  usage: TAG [configs]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-fused}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "fused or pipeline_golden or hough_affine" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/gpu_latency.sh $T "${2:-img1 c2 c3}"
