# instruction-cache behaviour of the matcher (SQC counters, one pass) on C3 launches
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT="$GRAFT_REPO_ROOT/gpurun_out/icache"; mkdir -p "$OUT"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --kernel-include-regex match_i8_kernel -d "$OUT/ic" -o pmc --output-format csv -- python3 tools/ab_i8.py 50000 1000 8 1 > "$OUT/ic.log" 2>&1 || { tail -5 "$OUT/ic.log"; exit 1; }
python3 - <<'PY'
import csv, glob, collections
v = collections.defaultdict(list)
for f in glob.glob("gpurun_out/icache/ic/*/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "match_i8_kernel" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: sum(x) / len(x) for k, x in v.items()})
PY
