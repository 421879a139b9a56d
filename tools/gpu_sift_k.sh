# descriptor_kernel / small_octaves_kernel times of SIFT variants (tools/variants/libsod_<v>.so;
# "base" = the in-tree library), one rocprofv3 kernel trace each.  usage: tools/gpu_sift_k.sh TAG v...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=$1; shift; O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for v in base "$@"; do
  if [ $v = base ]; then unset SOD_LIB_PATH; else export SOD_LIB_PATH=$GRAFT_REPO_ROOT/tools/variants/libsod_$v.so; fi
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O -o $v --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sift_prof.py 50 > $O/$v.log 2>&1) || { tail -5 $O/$v.log; exit 1; }
  python3 - $O/${v}_kernel_stats.csv $v <<'PY'
import csv, re, sys
rows = {}
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"::(\w+?)(<[^>]*>)?\(", r["Name"])
    rows[m.group(1) if m else r["Name"]] = r
n = int(rows["descriptor_kernel"]["Calls"])
tot = sum(float(r["TotalDurationNs"]) for r in rows.values()) / n / 1000
print(sys.argv[2], "per image %.1f us" % tot, " ".join("%s %.1f" % (k, float(rows[k]["AverageNs"]) / 1000)
      for k in ("descriptor_kernel", "small_octaves_kernel", "orient_kernel", "rank_kernel", "extrema_all_kernel", "sort_dedup_kernel") if k in rows))
PY
done
