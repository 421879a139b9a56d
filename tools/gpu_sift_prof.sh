set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/siftprof; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O" -o sp --output-format csv -- python3 tools/sift_bench.py 800 1000 20 > $O/sp.log 2>&1 || exit 1
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/siftprof/sp_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:16]:
    n = r["Name"]
    n = n.split("(")[0].split("::")[-1] if "::" in n.split("(")[0] else n.split("(")[0]
    if not n.strip(): n = r["Name"][:60]
    print("%-40s %5s %9.1f us %5.1f %%" % (n[-40:], r["Calls"], float(r["AverageNs"]) / 1e3, 100 * float(r["TotalDurationNs"]) / tot))
PY
