# slow-path statistics of the counting builds, then interleaved C3 matcher A/B of tools/variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${OUT:-flip2}; mkdir -p $O; : > $O/count.log; : > $O/ab.log
for v in tools/variants_count/*.so; do
  for a in "50000 1000" "10000 100"; do
    echo "== $v $a" >> $O/count.log
    SOD_LIB_PATH="$PWD/$v" timeout -k 10 120 python3 tools/ab_match.py $a i8 >> $O/count.log 2>&1 || { tail -5 $O/count.log; exit 1; }
  done
done
for i in 1 2; do
  for v in tools/variants/*.so; do
    SOD_LIB_PATH="$PWD/$v" timeout -k 10 120 python3 tools/ab_i8.py ${AB_ARGS:-50000 1000 40} >> $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
  done
done
cat $O/count.log $O/ab.log
