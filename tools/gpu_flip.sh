# parity of a variant build (VAR) on the GPU suite, then interleaved matcher A/B of all
# tools/variants/*.so at C3, 10k x 100k and 500 x 1M
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${OUT:-flip}; mkdir -p $O
SOD_LIB_PATH=$PWD/tools/variants/${VAR:-libsod_flip.so} timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYSEL:-} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.log
for i in 1 2; do
  for v in tools/variants/*.so; do
    for a in "50000 1000 40" "10000 100 40" "500 1000 40"; do
      SOD_LIB_PATH="$PWD/$v" timeout -k 10 120 python3 tools/ab_i8.py $a >> $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
    done
  done
done
cat $O/ab.log
