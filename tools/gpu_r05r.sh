# affine outlier-test rounding (option affine_fma) and the affine / pipeline parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "outlier or affine or pipeline or main or c3 or golden" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
