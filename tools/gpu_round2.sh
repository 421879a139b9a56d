# full GPU parity suite, default bench, kernel trace of the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r2; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/pytest.log 2>&1 || { tail -30 gpurun_out/r2/pytest.log; exit 1; }
tail -2 gpurun_out/r2/pytest.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extras > gpurun_out/r2/bench.log 2>&1 || { tail -20 gpurun_out/r2/bench.log; exit 1; }
grep '^{' gpurun_out/r2/bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stage_ms'], d['roofline']['frac'])"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r2" -o tr --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/r2/tr.log 2>&1 || exit 1
