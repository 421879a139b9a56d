# the GPU suite twice in a row (stability check of the CU-split stream switches)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-twice}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import torch" > /dev/null 2>&1
for i in 1 2; do
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_$i.log 2>&1 || { tail -30 $O/pytest_$i.log; exit 1; }
  tail -1 $O/pytest_$i.log
done
