# streamed matcher diagnostics: finer body-0 stamps, no global publish, no slow path
set -o pipefail
export ROUNDS=1
for v in sstamp snopubst; do
  for c in img1 c2; do
    SOD_LIB_PATH=tools/variants/lib$v.so timeout -k 10 120 python -u tools/ab_small.py $c > gpurun_out/r05k_${v}_$c.log 2>&1 || exit 1
  done
done &&
SOD_LIB_PATH=tools/variants/libsnopub.so timeout -k 10 120 python -u tools/ab_small.py img1,c2,q5k > gpurun_out/r05k_snopub.log 2>&1 &&
for c in img1 c2; do
  SOD_LIB_PATH=tools/variants/libsnoslowst.so timeout -k 10 120 python -u tools/ab_small.py $c > gpurun_out/r05k_snoslowst_$c.log 2>&1
  r=$?; [ $r -le 1 ] || exit $r
done
