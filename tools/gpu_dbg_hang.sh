# find a hang: smoke with a traceback dump, then the GPU suite verbosely with per-test timeouts
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-dbg}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 5 120 python3 -u -c "import faulthandler; faulthandler.dump_traceback_later(90, exit=True); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc $?"; tail -30 $O/smoke.log
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 60 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc $?"; tail -40 $O/pytest.log
