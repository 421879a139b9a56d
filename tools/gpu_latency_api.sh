# one-image latency: HIP API + kernel timeline of tools/latency_probe.py.  usage: TAG [cfg]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-latapi}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
CFG=${2:-img1}
timeout -k 10 150 rocprofv3 --kernel-trace --hip-runtime-trace -d "$GRAFT_REPO_ROOT/$O/tr" -o lat --output-format csv -- python3 tools/latency_probe.py $CFG 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/latency_api_timeline.py $O/tr > $O/api_timeline.txt
tail -80 $O/api_timeline.txt
