set -o pipefail
export ROUNDS=2
timeout -k 10 120 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05e_default.log 2>&1 &&
for v in scount ss2 ss2c snox se0 se3; do
  SOD_LIB_PATH=tools/variants/lib$v.so timeout -k 10 120 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05e_$v.log 2>&1 || exit 1
done
