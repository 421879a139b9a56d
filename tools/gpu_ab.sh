# A/B the matcher variants in tools/variants/*.so against the main build (same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python tools/ab_match.py > gpurun_out/ab.log 2>&1 || exit $?
for v in tools/variants/*.so; do
  SOD_LIB_PATH="$v" timeout -k 10 200 python tools/ab_match.py >> gpurun_out/ab.log 2>&1 || exit $?
done
timeout -k 10 200 python tools/ab_match.py >> gpurun_out/ab.log 2>&1 || exit $?
