set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/small.log
for a in "10000 100 40 0" "10000 100 40 1" "2000 1000 40 1" "500 1000 40 1" "50000 1000 40 1"; do
  SOD_LIB_PATH="$PWD/tools/variants/libsod_a_base.so" timeout -k 10 120 python3 tools/ab_i8.py $a >> gpurun_out/small.log 2>&1 || { tail -5 gpurun_out/small.log; exit 1; }
done
cat gpurun_out/small.log
