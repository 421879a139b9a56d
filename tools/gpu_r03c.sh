# round-3: GPU suite (+ guard counts) and the small-query kernel A/B.  usage: tools/gpu_r03c.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r03c}; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=20 > gpurun_out/$TAG/pytest.log 2>&1 || { tail -60 gpurun_out/$TAG/pytest.log; exit 1; }
tail -8 gpurun_out/$TAG/pytest.log
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "near_edge" -s -q > gpurun_out/$TAG/guard.log 2>&1 || { tail -30 gpurun_out/$TAG/guard.log; exit 1; }
grep -E "listed" gpurun_out/$TAG/guard.log
timeout -k 10 500 python3 -u tools/small_q.py > gpurun_out/$TAG/small_q.log 2> gpurun_out/$TAG/small_q.err || { tail -30 gpurun_out/$TAG/small_q.err; exit 1; }
head -3 gpurun_out/$TAG/small_q.log
