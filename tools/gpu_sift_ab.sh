# SIFT kernel timings of libsod.so and each tools/variants/*.so (rocprofv3 kernel stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/sift_ab
: > gpurun_out/sift_ab/summary.txt
for v in sift-based-od_amd/libsod.so tools/variants/*.so; do
  [ -e "$v" ] || continue
  n=$(basename "$v" .so)
  SOD_LIB_PATH="$PWD/$v" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sift_ab/$n -o k --output-format csv -- python3 tools/sift_bench.py ${SIFT_H:-800} ${SIFT_W:-1000} 5 > gpurun_out/sift_ab/$n.log 2>&1 || exit $?
  echo "== $n: $(grep '^sift' gpurun_out/sift_ab/$n.log)" >> gpurun_out/sift_ab/summary.txt
  python3 - "$n" >> gpurun_out/sift_ab/summary.txt <<'PY'
import csv, glob, sys
f = glob.glob("gpurun_out/sift_ab/%s/**/k_kernel_stats.csv" % sys.argv[1], recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print("  %-34s calls %4s avg %8.2f us total/img %8.1f us" % (r["Name"].split("::")[-1][:34], r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 6e3))
PY
done
