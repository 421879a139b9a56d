# round 2: GPU parity suite after the ABI fixes, then the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02a; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02a/pytest.log 2>&1 || { tail -40 gpurun_out/r02a/pytest.log; exit 1; }
tail -2 gpurun_out/r02a/pytest.log
timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/r02a/bench.log 2>&1 || { tail -20 gpurun_out/r02a/bench.log; exit 1; }
grep '^{' gpurun_out/r02a/bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stage_ms'], d['roofline']['frac'])"
