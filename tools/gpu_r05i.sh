set -o pipefail
export ROUNDS=1
timeout -k 10 120 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05i_default.log 2>&1 &&
for v in sx2 sl32 sl8 scount; do
  SOD_LIB_PATH=tools/variants/lib$v.so timeout -k 10 120 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05i_$v.log 2>&1 || exit 1
done &&
for v in sstamp sstampx2; do
  for c in img1 c2; do
    SOD_LIB_PATH=tools/variants/lib$v.so timeout -k 10 120 python -u tools/ab_small.py $c > gpurun_out/r05i_${v}_$c.log 2>&1 || exit 1
  done
done
