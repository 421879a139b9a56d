# the tail stages on the whole chip (no CU split, one context): bench stage times + kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/tail; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --cu-reserve 0 --overlap 0 --contexts 1 --steps 10 --warmup 3 --no-extras --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stage_ms'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O" -o tr --output-format csv -- python3 bench.py --cu-reserve 0 --overlap 0 --contexts 1 --steps 10 --warmup 3 --no-extras --no-cpu-baseline > $O/tr.log 2>&1 || exit 1
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/tail/tr_kernel_stats.csv")))
for r in rows[:25]:
    print("%-40s %5s %10.1f us" % (r["Name"].split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
