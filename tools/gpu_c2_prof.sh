set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/c2p; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O" -o tr --output-format csv -- python3 bench.py --config c2 --steps 30 --warmup 10 --no-cpu-baseline --no-extras > $O/tr.log 2>&1 || exit 1
grep '^{' $O/tr.log | cut -c1-300
python3 - <<'PY'
import csv, re
rows = list(csv.DictReader(open("gpurun_out/c2p/tr_kernel_stats.csv")))
for r in rows[:24]:
    n = r["Name"]
    m = re.search(r"::([A-Za-z0-9_<>]+)\(", n)
    print("%-36s %5s %9.1f us" % (m.group(1) if m else n[:36], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
