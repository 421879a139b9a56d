# the whole GPU suite once (the driver's round-end command), log under gpurun_out/<tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-suite}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import torch" > /dev/null 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
