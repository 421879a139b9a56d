# one-image latency probe + kernel timeline.  usage: tools/gpu_latency.sh TAG [configs]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-lat}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for CFG in ${2:-img1 c2}; do
  timeout -k 10 120 python3 tools/latency_probe.py $CFG 30 > $O/lat_$CFG.log 2>&1 || { tail -20 $O/lat_$CFG.log; exit 1; }
  tail -1 $O/lat_$CFG.log
  timeout -k 10 150 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/tr_$CFG" -o lat --output-format csv -- python3 tools/latency_probe.py $CFG 5 > $O/prof_$CFG.log 2>&1 || { tail -20 $O/prof_$CFG.log; exit 1; }
  python3 tools/latency_timeline.py $(ls $O/tr_$CFG/*/lat_kernel_trace.csv 2>/dev/null || ls $O/tr_$CFG/lat_kernel_trace.csv) > $O/timeline_$CFG.txt
  cat $O/timeline_$CFG.txt | tail -25
done
