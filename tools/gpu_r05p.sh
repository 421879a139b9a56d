# round-5: changed GPU tests (results fetch, post-processing, streamed-kernel configs), then
# PMC passes of the ring matcher for C3 and one query image
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05p; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_postprocess.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_api.py -m gpu -x -v -k "post or fused_pipeline or query_batch or main or streamed or one_query or c2_full or toggle" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 bench.py --config img1 --no-cpu-baseline > $O/bench_img1.log 2>&1 || { tail -20 $O/bench_img1.log; exit 1; }
grep '^{' $O/bench_img1.log > $O/bench_img1.json
for CFG in c3 img1; do
  bash tools/gpu_pmc.sh $CFG i8 || exit 1
done
echo pmc done
