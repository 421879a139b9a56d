# SIFT on one 1000 x 800 image (tools/sift_prof.py): rocprofv3 kernel trace, every kernel's
# average time per image and the critical path of one image (first kernel start -> last
# kernel end, the busy union and the idle gaps).  usage: tools/gpu_sift_timeline.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-sifttl}; O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O -o tl --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sift_prof.py 30 > $O/tl.log 2>&1) || { tail -5 $O/tl.log; exit 1; }
cat $O/tl.log
python3 tools/sift_timeline.py $O/tl_kernel_trace.csv 30 > $O/timeline.txt && cat $O/timeline.txt
