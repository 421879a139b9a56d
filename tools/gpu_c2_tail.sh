# C2 tail work: GPU parity suite, C2 step (default split), C2 kernel stats under rocprofv3, C3 step
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/c2t; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 bench.py --config c2 --no-cpu-baseline --no-extras > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
grep '^{' $O/b.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('C2 step', round(d['ms_per_step'],4), 'host', round(d['host_enqueue_ms_per_step'],4), {k: round(v,3) for k,v in d['stage_ms'].items() if v})"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O" -o tr --output-format csv -- python3 bench.py --config c2 --steps 30 --warmup 10 --no-cpu-baseline --no-extras > $O/tr.log 2>&1 || exit 1
python3 - <<'PY'
import csv, re
rows = list(csv.DictReader(open("gpurun_out/c2t/tr_kernel_stats.csv")))
for r in rows[:24]:
    n = r["Name"]
    m = re.search(r"::([A-Za-z0-9_<>]+)\(", n)
    print("%-36s %5s %9.1f us" % (m.group(1) if m else n[:36], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
grep '^{' $O/c3.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('C3 step', round(d['ms_per_step'],4), 'host', round(d['host_enqueue_ms_per_step'],4), {k: round(v,3) for k,v in d['stage_ms'].items() if v})"
