# GPU parity suite, then an interleaved matcher A/B of tools/variants/*.so over sizes
# AB_SIZES="nq nimg launches reserve;..." (default: C3, C2, one 500-query image, 2k queries)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02d; export TMPDIR=/tmp
if [ -z "$AB_NOTEST" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02d/pytest.log 2>&1 || { tail -40 gpurun_out/r02d/pytest.log; exit 1; }
tail -2 gpurun_out/r02d/pytest.log
fi
: > gpurun_out/r02d/ab.log
IFS=';' read -ra SIZES <<< "${AB_SIZES:-50000 1000 40 1;10000 100 40 0;500 1000 40 1;2000 1000 40 1}"
for i in $(seq ${AB_ROUNDS:-2}); do
for a in "${SIZES[@]}"; do
  for v in tools/variants/*.so; do
    SOD_LIB_PATH="$PWD/$v" timeout -k 10 120 python3 tools/ab_i8.py $a >> gpurun_out/r02d/ab.log 2>&1 || { tail -5 gpurun_out/r02d/ab.log; exit 1; }
  done
done
done
cat gpurun_out/r02d/ab.log
