# interleaved A/B of libsod builds (tools/variants/libsod_<v>.so; "base" = the in-tree
# library) on the small-query configs of tools/small_q.py, one process per build and round.
# usage: tools/gpu_ab_small.sh TAG v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=$1; shift; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then unset SOD_LIB_PATH; else export SOD_LIB_PATH=$PWD/tools/variants/libsod_$v.so; fi
    VAR=SOD_AB_NONE MODES=0 timeout -k 10 300 python3 -u tools/small_q.py > $O/ab_${v}_$r.log 2> $O/ab_${v}_$r.err || { tail -20 $O/ab_${v}_$r.err; exit 1; }
    echo "$v r$r $(tail -1 $O/ab_${v}_$r.log)"
  done
done
