# interleaved matcher A/B of environment settings on one library (AB_ENVS: "NAME=V,NAME=V ..."
# groups separated by spaces, "-" = none) at AB_SIZES
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${OUT:-abenv}; mkdir -p $O; : > $O/ab.log
for i in $(seq ${AB_ROUNDS:-2}); do
  for e in ${AB_ENVS:--}; do
    for a in ${AB_SIZES:-"50000,1000,40" "10000,100,40" "500,1000,40"}; do
      echo -n "$e " >> $O/ab.log
      env $( [ "$e" = "-" ] || echo ${e//,/ } ) timeout -k 10 120 python3 tools/ab_i8.py ${a//,/ } >> $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
    done
  done
done
awk '{print $1, $2, $4, $5}' $O/ab.log | sort -s -k1,1
