# bench lines on one box: TAG then configs (default "c3 img1 c2"); C3 without the extras
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-bench}; shift; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
CFGS=${*:-c3 img1 c2}
timeout -k 10 400 python3 -u -c "import torch" > /dev/null 2>&1
for CFG in $CFGS; do
  timeout -k 10 300 python3 bench.py --config $CFG --no-cpu-baseline --no-extras > $O/bench_$CFG.log 2>&1 || { tail -20 $O/bench_$CFG.log; exit 1; }
  grep '^{' $O/bench_$CFG.log > $O/bench_$CFG.json
  python3 -c "
import json; d=json.load(open('$O/bench_$CFG.json'))
print('$CFG', 'step %.4f ms' % d['ms_per_step'], 'matcher %.4f ms' % d['stage_ms']['match_kernel'], 'frac %.3f' % d['roofline']['frac'],
      'host %.4f blocked %.4f cpu %.4f' % (d['host_enqueue_ms_per_step'], d['host_blocked_ms_per_step'], d['host_cpu_enqueue_ms_per_step']))"
done
