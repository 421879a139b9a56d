set -o pipefail
export ROUNDS=1
for v in sstamp sstamp2 sstampnx; do
  for c in img1 c2; do
    SOD_LIB_PATH=tools/variants/lib$v.so timeout -k 10 120 python -u tools/ab_small.py $c > gpurun_out/r05f_${v}_$c.log 2>&1 || exit 1
  done
done
