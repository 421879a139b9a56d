# interleaved matcher A/B of tools/variants/*.so at C3, 10k x 100k and 500 x 1M (AB_ROUNDS rounds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${OUT:-absz}; mkdir -p $O; : > $O/ab.log
for i in $(seq ${AB_ROUNDS:-2}); do
  for v in tools/variants/*.so; do
    for a in ${AB_SIZES:-"50000,1000,40" "10000,100,40" "500,1000,40"}; do
      SOD_LIB_PATH="$PWD/$v" timeout -k 10 120 python3 tools/ab_i8.py ${a//,/ } >> $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
    done
  done
done
sort -s -k1,1 $O/ab.log | awk '{print $1, $3, $4, $11, $14}'
