# GPU round check: parity tests, short benches, rocprofv3 kernel stats of the C3 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 2 > gpurun_out/bench_c3.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o c3 --output-format csv -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || exit $?
exit $rc
