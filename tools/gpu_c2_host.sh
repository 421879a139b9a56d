# C2 step time vs the host time spent enqueueing a step (is the C2 pipeline launch-bound?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/c2h; mkdir -p $O
for args in "" "--cu-reserve 0 --contexts 2" "--cu-reserve 0 --contexts 1 --overlap 0"; do
  timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-extras $args > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep '^{' $O/b.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('%-40s' % '$args', 'step', round(d['ms_per_step'],4), 'host', round(d['host_enqueue_ms_per_step'],4), 'match', round(d['stage_ms']['match_kernel'],4), {k: round(v,3) for k,v in d['stage_ms'].items() if v})"
done
