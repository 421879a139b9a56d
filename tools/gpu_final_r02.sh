# round-2 evidence: GPU parity suite, smoke(), default bench line, rocprofv3 kernel stats +
# trace of the default bench (timed-window matcher stats), C2 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r02f; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02f/pytest.log 2>&1 || { tail -30 gpurun_out/r02f/pytest.log; exit 1; }
tail -1 gpurun_out/r02f/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02f/smoke.log 2>&1 || { tail -20 gpurun_out/r02f/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python3 bench.py > gpurun_out/r02f/bench.log 2>&1 || { tail -20 gpurun_out/r02f/bench.log; exit 1; }
grep '^{' gpurun_out/r02f/bench.log > gpurun_out/r02f/bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r02f/bench.json')); print(d['value'], d['ms_per_step'], d['stage_ms']['match_kernel'], d['roofline']['frac'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r02f" -o c3 --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/r02f/prof.log 2>&1 || exit 1
python3 tools/kernel_window_stats.py gpurun_out/r02f/c3_kernel_trace.csv match_i8_kernel 10 20 gpurun_out/r02f/c3_match_window.json > /dev/null
grep '^{' gpurun_out/r02f/prof.log > gpurun_out/r02f/prof_bench.json
python3 -c "
import json; w=json.load(open('gpurun_out/r02f/c3_match_window.json')); d=json.load(open('gpurun_out/r02f/prof_bench.json')); print('rocprof window', w['avg_ms'], 'events', d['stage_ms']['match_kernel'])"
timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-extras > gpurun_out/r02f/c2.log 2>&1 || exit 1
grep '^{' gpurun_out/r02f/c2.log | cut -c1-200
