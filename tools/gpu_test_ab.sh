# GPU parity tests, then an interleaved A/B of the default build against tools/variants/*.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
AB_IMPLS=${AB_IMPLS:-i8} AB_VARIANT_IMPL=${AB_VARIANT_IMPL:-i8} bash tools/gpu_ab.sh || exit $?
grep match gpurun_out/ab.log
