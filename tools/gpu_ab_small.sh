# small-query-set matcher A/B: the tree's library against tools/abvar/*.so variants, with
# SOD_MATCH_QT choices, interleaved rounds (tools/ab_i8.py, back-to-back launches).
# usage: tools/gpu_ab_small.sh TAG "nq nimg launches reserve" "LIB:QT" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-absmall}; shift; ARGS=$1; shift; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
  for spec in "$@"; do
    lib=${spec%%:*}; qt=${spec##*:}
    [ "$lib" = tree ] && lib=$PWD/sift-based-od_amd/libsod.so || lib=$PWD/tools/abvar/$lib
    env SOD_LIB_PATH=$lib ${qt:+SOD_MATCH_QT=$qt} timeout -k 10 120 python3 tools/ab_i8.py $ARGS >> $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
    echo "[$spec r$r] $(tail -1 $O/ab.log)"
  done
done
