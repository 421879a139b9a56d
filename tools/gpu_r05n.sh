# streamed matcher: preloaded refill, 4 early bodies; seed over 3 windows; stamps + hits
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05n; mkdir -p $O; export ROUNDS=2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "streamed" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 150 python -u tools/ab_small.py img1,c2,q5k > $O/default.log 2>&1 || { tail -20 $O/default.log; exit 1; }
cat $O/default.log
for v in snopre sseed3; do
  SOD_LIB_PATH=tools/variants/lib$v.so timeout -k 10 150 python -u tools/ab_small.py img1,c2,q5k > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  cat $O/$v.log
done
for v in sstamp sseed3st; do
  SOD_LIB_PATH=tools/variants/lib$v.so timeout -k 10 120 python -u tools/ab_small.py img1 > $O/${v}_img1.log 2>&1 || { tail -20 $O/${v}_img1.log; exit 1; }
done
echo done
