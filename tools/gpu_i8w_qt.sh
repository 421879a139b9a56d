# 32x32x32 kernel (impl i8w) at 1 / 2 / 4 query tiles of 32 per wave (option match_qt):
# parity of the i8w tests at each, then matcher-only times against the ring kernel for one
# image (500 x 1M) and C2 (10k x 100k)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/i8w_qt; mkdir -p $O
for qt in 1 2; do
  SOD_MATCH_QT=$qt timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -q -k "i8w" --timeout 200 --timeout-method thread > $O/pytest_qt$qt.log 2>&1 || { tail -30 $O/pytest_qt$qt.log; exit 1; }
  tail -1 $O/pytest_qt$qt.log
done
for r in 1 2; do
  for a in "500 1000" "10000 100"; do
    timeout -k 10 200 python3 tools/ab_match.py $a i8 2>&1 | grep match
    for qt in 1 2 4; do
      SOD_MATCH_QT=$qt timeout -k 10 200 python3 tools/ab_match.py $a i8w 2>&1 | grep match | sed "s/^/qt$qt /"
    done
  done
done
