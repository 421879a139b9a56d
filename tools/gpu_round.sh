# tests + bench + kernel trace + A/B of matcher variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh || exit $?
bash tools/gpu_ab.sh || exit $?
