# GPU suite + C2 / C3 bench lines (tail changes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/tc; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in c2 c2 c3; do
  timeout -k 10 200 python3 bench.py --config $cfg --no-cpu-baseline --no-extras > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep '^{' $O/b.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', round(d['ms_per_step'],4), round(d['stage_ms']['match_kernel'],4), {k: round(v,3) for k,v in d['stage_ms'].items() if v})"
done
