# rocprofv3 kernel stats + timed-window matcher stats for the c2 and img1 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-profsmall}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import torch" > /dev/null 2>&1
for CFG in c2 img1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O" -o $CFG --output-format csv -- python3 bench.py --config $CFG --no-cpu-baseline --no-extras > $O/prof_$CFG.log 2>&1 || { tail -20 $O/prof_$CFG.log; exit 1; }
  grep '^{' $O/prof_$CFG.log > $O/prof_bench_$CFG.json
  python3 -c "import json; d=json.load(open('$O/prof_bench_$CFG.json')); print('$CFG steps', d['steps'], 'warmup', d['warmup'], 'match', d['stage_ms']['match_kernel'])"
done
echo done
