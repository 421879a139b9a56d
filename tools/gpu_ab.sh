# A/B of matcher implementations / variant builds on the same box (interleaved)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab.log
for i in 1 2; do
  timeout -k 10 200 python tools/ab_match.py 50000 1000 bf16 >> gpurun_out/ab.log 2>&1 || exit $?
  timeout -k 10 200 python tools/ab_match.py 50000 1000 i8 >> gpurun_out/ab.log 2>&1 || exit $?
  for v in tools/variants/*.so; do
    [ -e "$v" ] || continue
    SOD_LIB_PATH="$v" timeout -k 10 200 python tools/ab_match.py >> gpurun_out/ab.log 2>&1 || exit $?
  done
done
