# GPU round check: parity tests, benches, rocprofv3 kernel stats of the C3 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 2 > gpurun_out/bench_c3.log 2>&1 || exit $?
# multi-process plumbing of the bench (2 ranks on this box's one GPU, host-staged exchange)
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --comm host --config c3 \
  > gpurun_out/bench_c3_2rank_host.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o c3 --output-format csv -- python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-extras --contexts 1 > gpurun_out/prof_c3.log 2>&1 || exit $?
exit $rc
