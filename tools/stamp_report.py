"""Work-group timeline of one matcher launch from a SOD_I8_STAMP build (tools/ab_match.py
saves gpurun_out/stamps_<impl>.npy: per work-group s_memtime / s_memrealtime at start and
end, HW_ID, XCC_ID).  Prints the start skew, the duration spread, the end spread, the
in-kernel clock and the per-XCD medians.

    python tools/stamp_report.py gpurun_out/stamps_i8.npy
"""
import sys

import numpy as np


def main():
    st = np.load(sys.argv[1]).astype(np.int64)
    t0, r0, t1, r1, xcc = st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 5] & 0xF
    us = lambda r: r / 100.0                      # s_memrealtime ticks at 100 MHz
    start = us(r0 - r0.min())
    end = us(r1 - r0.min())
    dur = us(r1 - r0)
    clk = (t1 - t0) / np.maximum(r1 - r0, 1) * 0.1   # GHz
    print("work-groups %d  kernel span %.1f us" % (len(st), end.max()))
    for name, v in (("start", start), ("duration", dur), ("end", end)):
        q = np.percentile(v, [0, 10, 50, 90, 100])
        print("%-9s us  min %.1f  p10 %.1f  median %.1f  p90 %.1f  max %.1f" % (name, *q))
    print("clock GHz median %.3f" % np.median(clk))
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        print("  xcc %d: n %3d  start med %.1f  dur med %.1f  end max %.1f" % (
            x, m.sum(), np.median(start[m]), np.median(dur[m]), end[m].max()))


if __name__ == "__main__":
    main()
