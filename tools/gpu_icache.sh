# instruction-cache behaviour of the matcher (SQ/SQC counters, one pass per config):
# C3, C2 (10k x 100k) and one query image (500 x 1M).  usage: tools/gpu_icache.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=${1:-icache}; OUT="$GRAFT_REPO_ROOT/gpurun_out/$T"; mkdir -p "$OUT"
for c in "50000 1000" "10000 100" "500 1000"; do
  n=${c// /x}
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-include-regex match_i8_kernel -d "$OUT/ic_$n" -o pmc --output-format csv -- python3 tools/ab_i8.py $c 8 > "$OUT/ic_$n.log" 2>&1 || { tail -5 "$OUT/ic_$n.log"; exit 1; }
  python3 - "$OUT/ic_$n" "$n" <<'PY'
import csv, glob, collections, sys
v = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "match_i8_kernel" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: round(sum(x) / len(x)) for k, x in sorted(v.items())})
PY
done
