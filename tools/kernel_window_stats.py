"""Per-kernel statistics of a window of launches from a rocprofv3 kernel trace.

bench.py launches the matcher W times (warmup), K times (timed region), then a few isolated
launches for the per-stage timings; rocprofv3 --stats averages all of them.  This picks the
timed-region launches (launch indices W .. W+K-1 of the kernel, in start order) so the
rocprof average can be compared with bench.py's live HIP-event average.

    python tools/kernel_window_stats.py TRACE.csv match_i8_kernel 10 20 [out.json]
"""
import csv
import json
import sys


def main():
    path, name, skip, count = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    win = rows[skip:skip + count]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in win]
    starts = [int(r["Start_Timestamp"]) for r in win]
    ends = [int(r["End_Timestamp"]) for r in win]
    out = {"trace": path, "kernel": name, "launches_total": len(rows), "window_first": skip,
           "window_count": len(win), "avg_ms": sum(dur) / len(dur), "min_ms": min(dur),
           "max_ms": max(dur),
           "start_to_start_ms": (starts[-1] - starts[0]) / 1e6 / max(1, len(win) - 1),
           "gap_end_to_next_start_us": sum((starts[i + 1] - ends[i]) / 1e3
                                           for i in range(len(win) - 1)) / max(1, len(win) - 1)}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 5:
        with open(sys.argv[5], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
