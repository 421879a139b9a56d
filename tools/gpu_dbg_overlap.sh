# the CU-split overlap test with sync diagnostics (SOD_DEBUG_SYNC), verbose, stdout unbuffered
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-dbgov}; mkdir -p $O; export TMPDIR=/tmp
SOD_DEBUG_SYNC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_api.py -m gpu -x -v -s -k "overlap_equals_serial or shared_db" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; echo "rc $?"
grep -n "sod:\|PASSED\|FAILED\|Timeout" $O/pytest.log | tail -30
