# SIFT parity (GPU suite, SIFT tests) with the tree's library, then single-image and batch
# timing of the variants in tools/variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/siftab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sift.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do for v in tools/variants/*.so; do
  echo "== $v" ; SOD_LIB_PATH=$PWD/$v timeout -k 10 120 python3 tools/sift_bench.py 800 1000 30 || exit 1
  SOD_LIB_PATH=$PWD/$v timeout -k 10 120 python3 tools/sift_batch_bench.py || exit 1
done; done
