# SQ counters of the int8 matcher for the default build and each tools/variants/*.so
# (tools/ab_match.py workload, one counter group per rocprofv3 run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
K=match_i8_kernel
for v in default tools/variants/*.so; do
  name=$(basename $v .so)
  OUT="$GRAFT_REPO_ROOT/gpurun_out/pmcab_$name"
  mkdir -p "$OUT"
  if [ "$v" = default ]; then unset SOD_LIB_PATH; else export SOD_LIB_PATH="$v"; fi
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU --kernel-include-regex "$K" -d "$OUT/sq" -o pmc --output-format csv -- python3 tools/ab_match.py 50000 1000 i8 > "$OUT/sq.log" 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "$K" -d "$OUT/sq2" -o pmc --output-format csv -- python3 tools/ab_match.py 50000 1000 i8 > "$OUT/sq2.log" 2>&1 || exit $?
done
unset SOD_LIB_PATH
python3 - <<'PY'
import csv, glob, os, collections
for d in sorted(glob.glob("gpurun_out/pmcab_*")):
    acc = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    # per launch: counters are summed over dimensions per dispatch row; average over dispatches
    per = {}
    for k, v in acc.items():
        per[k] = sum(v)
    print(os.path.basename(d), {k: "%.4g" % v for k, v in sorted(per.items())})
PY
