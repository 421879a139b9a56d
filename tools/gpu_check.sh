set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
nproc > gpurun_out/nproc.txt
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config tiny --steps 3 --warmup 1 > gpurun_out/bench_tiny.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 2 > gpurun_out/bench_c3.log 2>&1 || exit $?
exit $rc
