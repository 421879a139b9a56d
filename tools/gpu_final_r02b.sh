# round-2 evidence (second session): GPU parity suite, smoke(), default bench line, rocprofv3 kernel stats + timed-window matcher stats, C2 bench line, matcher PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/${OUT:-r02x}; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${OUT:-r02x}/pytest.log 2>&1 || { tail -30 gpurun_out/${OUT:-r02x}/pytest.log; exit 1; }
tail -1 gpurun_out/${OUT:-r02x}/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${OUT:-r02x}/smoke.log 2>&1 || { tail -20 gpurun_out/${OUT:-r02x}/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python3 bench.py > gpurun_out/${OUT:-r02x}/bench.log 2>&1 || { tail -20 gpurun_out/${OUT:-r02x}/bench.log; exit 1; }
grep '^{' gpurun_out/${OUT:-r02x}/bench.log > gpurun_out/${OUT:-r02x}/bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/${OUT:-r02x}/bench.json')); print(d['value'], d['ms_per_step'], d['stage_ms']['match_kernel'], d['roofline']['frac'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${OUT:-r02x}" -o c3 --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/${OUT:-r02x}/prof.log 2>&1 || exit 1
python3 tools/kernel_window_stats.py gpurun_out/${OUT:-r02x}/c3_kernel_trace.csv match_i8_kernel 10 20 gpurun_out/${OUT:-r02x}/c3_match_window.json > /dev/null
grep '^{' gpurun_out/${OUT:-r02x}/prof.log > gpurun_out/${OUT:-r02x}/prof_bench.json
python3 -c "
import json; w=json.load(open('gpurun_out/${OUT:-r02x}/c3_match_window.json')); d=json.load(open('gpurun_out/${OUT:-r02x}/prof_bench.json')); print('rocprof window', w['avg_ms'], 'events', d['stage_ms']['match_kernel'])"
timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-extras > gpurun_out/${OUT:-r02x}/c2.log 2>&1 || exit 1
grep '^{' gpurun_out/${OUT:-r02x}/c2.log | cut -c1-200
bash tools/gpu_pmc.sh c3 i8 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_match_i8_kernel_c3 gpurun_out/${OUT:-r02x}/pmc_match_i8_kernel_c3.json $(python3 -c "import json; print(json.load(open('gpurun_out/${OUT:-r02x}/c3_match_window.json'))['avg_ms'])") match_i8_kernel | grep -E "hbm_bytes|clock|mfma_busy"
