# Main drop-in tests + the staged C3 probe (tools/main_c3_probe.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-maincheck}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import torch" > /dev/null 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -k "main or Main or posebin or affine or dropin" --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/main_c3_probe.py
