# bench step time vs warmup length (clock ramp): C3 and C2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/wu; mkdir -p $O
for args in "--warmup 10" "--warmup 40" "--config c2 --warmup 10" "--config c2 --warmup 500 --steps 200" "--warmup 10" "--warmup 40"; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras $args > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep '^{' $O/b.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('%-40s' % '$args', 'step', round(d['ms_per_step'],4), 'match', round(d['stage_ms']['match_kernel'],4), 'frac', round(d['roofline']['frac'],4))"
done
