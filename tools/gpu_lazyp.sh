set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
AB_IMPLS=i8 AB_VARIANT_IMPL=i8 bash tools/gpu_ab.sh || exit $?
AB_IMPLS=i8 AB_VARIANT_IMPL=i8 bash -c 'for i in 1 2; do for v in "" tools/variants/libsod_eagerp.so; do SOD_LIB_PATH=$v timeout -k 10 200 python tools/ab_match.py 50000 1000 i8 || exit 1; done; done' >> gpurun_out/ab.log 2>&1
cat gpurun_out/ab.log | grep match
