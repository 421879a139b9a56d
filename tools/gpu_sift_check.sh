# SIFT parity suite + the bench-like one-image / batch probe (3 rounds, default streams)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-siftchk}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sift.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  PROBE_UNSPLIT=1 PROBE_TAG="[default r$r]" timeout -k 10 120 python3 tools/sift_ctx_probe.py 10 >> $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
  tail -1 $O/probe.log
done
