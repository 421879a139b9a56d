# interleaved steady-state A/B of the matcher variants in tools/variants/*.so (+ the tree's
# libsod.so), AB_ROUNDS rounds; args to ab_i8.py from AB_ARGS
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/ab_i8.log
for i in $(seq ${AB_ROUNDS:-3}); do
  for v in tools/variants/*.so; do
    SOD_LIB_PATH="$PWD/$v" timeout -k 10 120 python3 tools/ab_i8.py ${AB_ARGS:-} >> gpurun_out/ab_i8.log 2>&1 || { tail -5 gpurun_out/ab_i8.log; exit 1; }
  done
done
cat gpurun_out/ab_i8.log
