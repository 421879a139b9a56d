set -o pipefail
export ROUNDS=1
timeout -k 10 120 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05g_default.log 2>&1 &&
SOD_LIB_PATH=tools/variants/libsd8.so timeout -k 10 120 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05g_d8.log 2>&1 &&
for v in sstamp sstampnp sstampnx; do
  for c in img1 c2; do
    SOD_LIB_PATH=tools/variants/lib$v.so timeout -k 10 120 python -u tools/ab_small.py $c > gpurun_out/r05g_${v}_$c.log 2>&1 || exit 1
  done
done
