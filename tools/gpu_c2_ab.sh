# C2 step: A/B of an environment assignment given as $1 (bench default otherwise)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/c2ab; mkdir -p $O
for v in "" "$1" "" "$1"; do
  env $v timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-extras > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep '^{' $O/b.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('%-20s' % '$v', 'step', round(d['ms_per_step'],4), 'host', round(d['host_enqueue_ms_per_step'],4))"
done
