# round-3 matcher diagnostics on small query sets: in-kernel stamps (work-group timeline) and
# slow-path counts for one query image (QT 2 and 4), C2 and C3.  usage: tools/gpu_r03e.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-r03e}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
S=$PWD/tools/variants/libsod_stamp.so; C=$PWD/tools/variants/libsod_count.so
for qt in 2 4; do
  SOD_MATCH_QT=$qt SOD_LIB_PATH=$S timeout -k 10 120 python3 tools/ab_match.py 500 1000 i8 > $O/stamp_img1_qt$qt.log 2>&1 || { tail -5 $O/stamp_img1_qt$qt.log; exit 1; }
  cp gpurun_out/stamps_i8.npy $O/stamps_img1_qt$qt.npy
done
SOD_LIB_PATH=$S timeout -k 10 120 python3 tools/ab_match.py 10000 100 i8 > $O/stamp_c2.log 2>&1 || { tail -5 $O/stamp_c2.log; exit 1; }
cp gpurun_out/stamps_i8.npy $O/stamps_c2.npy
for cfg in "500 1000" "10000 100" "50000 1000"; do
  set -- $cfg
  SOD_LIB_PATH=$C timeout -k 10 150 python3 tools/ab_match.py $1 $2 i8 > $O/count_$1.log 2>&1 || { tail -5 $O/count_$1.log; exit 1; }
done
grep -h "" $O/*.log | grep -v "^$" | cut -c1-220
CONFIGS=img500x1M,c2,q2kx1M timeout -k 10 400 python3 -u tools/small_q.py > $O/small_q_qt.log 2> $O/small_q_qt.err || { tail -20 $O/small_q_qt.err; exit 1; }
head -3 $O/small_q_qt.log | cut -c1-400
