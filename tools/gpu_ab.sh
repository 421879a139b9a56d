# A/B of matcher implementations / variant builds on the same box (interleaved)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab.log
for i in 1 2; do
  for impl in ${AB_IMPLS:-bf16 i8 i8w}; do
    timeout -k 10 200 python tools/ab_match.py 50000 1000 $impl >> gpurun_out/ab.log 2>&1 || exit $?
  done
  for v in tools/variants/*.so; do
    [ -e "$v" ] || continue
    SOD_LIB_PATH="$v" timeout -k 10 200 python tools/ab_match.py 50000 1000 ${AB_VARIANT_IMPL:-i8w} >> gpurun_out/ab.log 2>&1 || exit $?
  done
done
