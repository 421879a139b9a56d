"""Where one Main.run goes, from the host's HIP calls and the device's kernels on one clock.

    rocprofv3 --kernel-trace --hip-runtime-trace -d OUT -o rt --output-format csv -- \\
        python3 tools/run_api_timeline.py run            # 300 Main.run of one 500-keypoint image
    python3 tools/run_api_timeline.py analyze OUT        # medians over the last 200 runs

Each run (found by its matcher kernel) is split at: the run's first HIP call, the matcher's
launch call, the matcher's start and end on the device, the end of the last kernel, and the
end of the last HIP call before the next run's first one (the results wait).  The host time
between one run's last HIP call and the next run's first is Python (the results arrays,
final_pose, the loop, the enqueue's Python side)."""
import csv
import glob
import os
import re
import sys

import numpy as np


def run():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import sod_pkg
    sod_pkg.load()
    from sift_based_od_amd import Main, SiftDatabase, _lib, synthetic
    db = synthetic.make_database(1000, 1000, seed=0, workers=8)
    qs = synthetic.make_queries(500, seed=7, db_seed=0, kp_per_image=1000, n_objects=1)
    c = _lib.Context(0)
    c.set_impl("i8")
    m = Main(c)
    m.set_database(SiftDatabase(db.des, db.kp, db.img, db.centroid, db.size))
    m.get_query_features(qs.des, qs.kp, qs.shape)
    for _ in range(300):
        m.run((32, 32, 8, 12))
    c.synchronize()


def _rows(out, pattern):
    paths = glob.glob(os.path.join(out, "**", pattern), recursive=True)
    if not paths:
        raise SystemExit("no %s under %s" % (pattern, out))
    return list(csv.DictReader(open(paths[0])))


def analyze(out):
    kern = _rows(out, "*kernel_trace.csv")
    api = _rows(out, "*hip_api_trace.csv")
    kern = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                    int(r["Correlation_Id"])) for r in kern))
    api = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"],
                   int(r["Correlation_Id"])) for r in api))
    api_by_corr = {a[3]: a for a in api}
    starts = np.array([a[0] for a in api])
    kstarts = np.array([k[0] for k in kern])
    runs = [(k, api_by_corr[k[3]]) for k in kern
            if "match_i8_kernel" in k[2] and k[3] in api_by_corr]
    # a run's results wait is its stream queries: the last query before the next matcher
    # launch call ends it, and the next call starts the next run's enqueue (Python between)
    split = []
    for i in range(len(runs) - 1):
        lo, hi = np.searchsorted(starts, runs[i][1][0]), np.searchsorted(starts, runs[i + 1][1][0])
        calls = api[lo:hi + 1]
        j = max(j for j, a in enumerate(calls) if a[2] == "hipStreamQuery")
        split.append((calls[j][1], calls[j + 1][0], hi - lo))
    ph = {k: [] for k in ("enqueue_start_to_matcher_launch", "matcher_launch_to_start",
                          "matcher_kernel", "matcher_end_to_last_kernel_end",
                          "last_kernel_end_to_wait_end", "run_enqueue_start_to_wait_end",
                          "python_after_wait", "hip_calls_per_run", "kernels_per_run")}
    for i in range(1, len(runs) - 1):
        (mk, la), first, (wait_end, next_first, ncalls) = runs[i], split[i - 1][1], split[i]
        ks = kern[np.searchsorted(kstarts, mk[0]):np.searchsorted(kstarts, runs[i + 1][0][0])]
        last_k_end = max(k[1] for k in ks)
        ph["enqueue_start_to_matcher_launch"].append(la[0] - first)
        ph["matcher_launch_to_start"].append(mk[0] - la[0])
        ph["matcher_kernel"].append(mk[1] - mk[0])
        ph["matcher_end_to_last_kernel_end"].append(last_k_end - mk[1])
        ph["last_kernel_end_to_wait_end"].append(wait_end - last_k_end)
        ph["run_enqueue_start_to_wait_end"].append(wait_end - first)
        ph["python_after_wait"].append(next_first - wait_end)
        ph["hip_calls_per_run"].append(ncalls * 1000)
        ph["kernels_per_run"].append(len(ks) * 1000)
    for k, v in ph.items():
        v = np.array(v[-200:], float) / 1e3
        if "per_run" in k:
            print("  %-34s median %5.0f" % (k, np.median(v)))
        else:
            print("  %-34s median %7.1f us  min %7.1f" % (k, np.median(v), v.min()))
    # the HIP calls of one run in order, with their start offsets (the last analysed run)
    i = len(runs) - 2
    first, wait_end = split[i - 1][1], split[i][0]
    lo, hi = np.searchsorted(starts, first), np.searchsorted(starts, wait_end)
    prev = None
    names = []
    for a in api[lo:hi + 1]:
        if a[2] == "hipGetLastError":   # (after every launch and every busy query)
            continue
        if prev is not None and a[2] == prev[0]:
            prev[1] += 1
            continue
        prev = [a[2], 1, (a[0] - first) / 1e3]
        names.append(prev)
    print("  calls of one run (start offset us, repeats):")
    for n, c, t in names:
        print("    %8.1f  %s%s" % (t, n, " x%d" % c if c > 1 else ""))
    for k in kern[np.searchsorted(kstarts, runs[i][0][0]):np.searchsorted(kstarts, runs[i + 1][0][0])]:
        name = re.findall(r"([A-Za-z_][A-Za-z0-9_]*)\s*(?:<[^(]*>)?\s*\(",
                          k[2].replace("(anonymous namespace)::", "").replace("void ", ""))
        print("    kernel %8.1f .. %8.1f  %s" % ((k[0] - first) / 1e3, (k[1] - first) / 1e3,
                                                 name[0] if name else k[2][:40]))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        analyze(sys.argv[2])
