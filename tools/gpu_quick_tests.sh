# a named subset of the GPU tests. usage: TAG "-k expression"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-qt}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import torch" > /dev/null 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "$2" --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
