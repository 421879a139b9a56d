# GPU parity suite on the default library, then an interleaved matcher A/B against
# tools/variants/$VAR_libsod.so at several sizes (ab_i8.py: nq n_images launches reserve)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/libab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for a in "50000 1000 40 1" "10000 100 400 1" "2000 1000 100 0" "500 1000 200 0"; do
    for v in new ${VAR:-seed0}; do
      if [ $v = new ]; then unset SOD_LIB_PATH; else export SOD_LIB_PATH=$PWD/tools/variants/${v}_libsod.so; fi
      echo -n "$v " ; timeout -k 10 120 python3 tools/ab_i8.py $a || exit 1
    done
  done
done
