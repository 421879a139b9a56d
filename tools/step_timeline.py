"""Kernel timeline of one pipelined step from a rocprofv3 kernel trace: every kernel that
starts between matcher launch i and launch i+2, with start offset and duration.

    python tools/step_timeline.py TRACE.csv [i] [matcher_kernel_name]
"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    i = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    name = sys.argv[3] if len(sys.argv) > 3 else "match_i8_kernel"
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    m = [r for r in rows if name in r["Kernel_Name"]]
    t0, t1 = int(m[i]["Start_Timestamp"]), int(m[i + 2]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s < t1:
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            mm = re.search(r"([A-Za-z_][A-Za-z0-9_]*)\s*(<[^(]*>)?\s*\(", k)
            n = mm.group(1) + (mm.group(2) or "") if mm else k
            print("%-40s start %9.1f us  dur %8.1f us" % (n[:40], (s - t0) / 1e3, (e - s) / 1e3))


if __name__ == "__main__":
    main()
