# streamed matcher, top-2 list exchange: parity tests, A/B vs the ring kernel, stamps + hits
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05l; mkdir -p $O; export ROUNDS=2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "streamed or query_tiles or matcher_vs_oracle or edges" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u -m pytest tests/test_postprocess.py tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -v -k "postprocess or fused_pipeline or query_batch or main" --timeout 150 --timeout-method thread > $O/pytest_results.log 2>&1 || { tail -30 $O/pytest_results.log; exit 1; }
tail -1 $O/pytest_results.log
timeout -k 10 200 python -u tools/run_profile.py > $O/run_profile.log 2>&1 || { tail -30 $O/run_profile.log; exit 1; }
head -12 $O/run_profile.log
timeout -k 10 150 python -u tools/ab_small.py img1,c2,q5k,q2k > $O/default.log 2>&1 || { tail -20 $O/default.log; exit 1; }
cat $O/default.log
for v in se1 se4; do
  SOD_LIB_PATH=tools/variants/lib$v.so timeout -k 10 150 python -u tools/ab_small.py img1,c2,q5k > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
done
for c in img1 c2; do
  SOD_LIB_PATH=tools/variants/libsstamp.so timeout -k 10 120 python -u tools/ab_small.py $c > $O/sstamp_$c.log 2>&1 || { tail -20 $O/sstamp_$c.log; exit 1; }
done
SOD_LIB_PATH=tools/variants/libsnoslowst.so timeout -k 10 120 python -u tools/ab_small.py img1 > $O/snoslowst_img1.log 2>&1
r=$?; [ $r -le 1 ] || exit $r
echo done
