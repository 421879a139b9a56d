"""Merge a rocprofv3 HIP-API trace and kernel trace (same clock) of tools/latency_probe.py:
the last step's API calls and kernels in time order, relative to the last matcher launch's
hipExtLaunchKernel... call.  python tools/latency_api_timeline.py DIR"""
import csv
import glob
import re
import sys


def load(pattern):
    f = glob.glob(pattern, recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d = sys.argv[1]
    ker = load(d + "/**/*kernel_trace.csv")
    api = load(d + "/**/*hip_api_trace.csv")
    ev = []
    for r in ker:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        mm = re.search(r"([A-Za-z_][A-Za-z0-9_]*)\s*(<[^(]*>)?\s*\(", k)
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + (mm.group(1) if mm else k)))
    for r in api:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A " + r["Function"]))
    ev.sort()
    ms = [e for e in ev if e[2].startswith("K match_i8_kernel")]
    t_m = ms[-1][0]
    # the last hipStreamSynchronize / hipDeviceSynchronize before the last matcher start
    syncs = [e for e in ev if e[2].startswith("A ") and "Synchronize" in e[2] and e[1] < t_m]
    t0 = syncs[-1][1] if syncs else t_m
    for s, e, n in ev:
        if s >= t0 - 1000 and s <= t_m + 400000:
            print("%9.1f %8.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, n[:60]))


if __name__ == "__main__":
    main()
