# streamed matcher diagnostics after the list exchange: early-body variants, stamps + hits
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05m; mkdir -p $O; export ROUNDS=2
for v in se1 se4; do
  SOD_LIB_PATH=tools/variants/lib$v.so timeout -k 10 150 python -u tools/ab_small.py img1,c2,q5k > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  cat $O/$v.log
done
for c in img1 c2; do
  SOD_LIB_PATH=tools/variants/libsstamp.so timeout -k 10 120 python -u tools/ab_small.py $c > $O/sstamp_$c.log 2>&1 || { tail -20 $O/sstamp_$c.log; exit 1; }
done
SOD_LIB_PATH=tools/variants/libsnoslowst.so timeout -k 10 120 python -u tools/ab_small.py img1 > $O/snoslowst_img1.log 2>&1
r=$?; [ $r -le 1 ] || exit $r
echo done
