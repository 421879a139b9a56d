# round-5 closing evidence: suite, smoke, bench lines (c3 with extras, img1, c2), rocprofv3
# kernel stats of the C3 bench, PMC passes of the ring matcher for C3, one image and C2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r05o.sh r05v || exit 1
for CFG in c3 img1 c2; do
  bash tools/gpu_pmc.sh $CFG i8 || exit 1
done
echo pmc done
