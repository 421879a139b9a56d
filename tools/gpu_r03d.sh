# round-3 evidence: default bench line, rocprofv3 kernel stats + timed-window matcher stats
# (C3), PMC passes of the matcher for C3, C2 and one query image.  usage: tools/gpu_r03d.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-r03d}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench_c3.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O" -o c3 --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-extras > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/kernel_window_stats.py $O/c3_kernel_trace.csv match_i8_kernel 10 20 $O/c3_match_window.json > /dev/null
grep '^{' $O/prof.log > $O/prof_bench.json
echo profiled
for CFG in c2 img1; do
  timeout -k 10 200 python3 bench.py --config $CFG --no-cpu-baseline --no-extras > $O/bench_$CFG.log 2>&1 || { tail -20 $O/bench_$CFG.log; exit 1; }
  grep '^{' $O/bench_$CFG.log > $O/bench_$CFG.json
done
echo benches
for CFG in c3 c2 img1; do
  bash tools/gpu_pmc.sh $CFG i8 || exit 1
done
echo pmc done
