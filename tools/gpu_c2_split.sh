# C2 step time: two contexts (default) vs the CU split with 1 or 2 reserved CUs per XCD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/c2s; mkdir -p $O
for args in "" "--cu-reserve 1" "--cu-reserve 2" "--contexts 1 --overlap 1"; do
  timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-extras $args > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep '^{' $O/b.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('%-28s' % '$args', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4), d['config']['cu_reserve_per_xcd'], d['config']['query_streams'], {k: round(v,3) for k,v in d['stage_ms'].items() if v})"
done
