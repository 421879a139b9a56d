"""Kernel timeline of the last latency step of tools/latency_probe.py from a rocprofv3 kernel
trace: every kernel from the last matcher launch on, start offset, duration and the gap to the
previous kernel's end.   python tools/latency_timeline.py TRACE.csv [matcher_kernel_name]"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    name = sys.argv[2] if len(sys.argv) > 2 else "match_i8_kernel"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    m = [i for i, r in enumerate(rows) if name in r["Kernel_Name"]]
    for which in (m[-2], m[-1]):
        t0 = int(rows[which]["Start_Timestamp"])
        end = which + 1
        while end < len(rows) and name not in rows[end]["Kernel_Name"]:
            end += 1
        prev = None
        last = t0
        for r in rows[which:end]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            mm = re.search(r"([A-Za-z_][A-Za-z0-9_]*)\s*(<[^(]*>)?\s*\(", k)
            n = mm.group(1) + (mm.group(2) or "") if mm else k
            print("%-36s start %8.1f us  dur %7.1f us  gap %6.1f us" % (
                n[:36], (s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0))
            prev = e
            last = max(last, e)
        print("span %.1f us\n" % ((last - t0) / 1e3))


if __name__ == "__main__":
    main()
