set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06l; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_suite.sh r06l || exit 1
timeout -k 10 200 python3 tools/run_timeline.py > $O/rt.log 2>&1 || exit 1
cat $O/rt.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o rt --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/run_timeline.py > $GRAFT_REPO_ROOT/$O/rt_prof.log 2>&1
