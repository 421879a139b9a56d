set -o pipefail
cd "$GRAFT_REPO_ROOT"
AB_ROUNDS=2 OUT=xev bash tools/gpu_ab_sizes.sh || exit 1
bash tools/gpu_pmc_fetch_ab.sh || exit 1
