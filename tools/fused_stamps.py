"""Phase times of hough_small_kernel from a SOD_SEL_STAMP build (s_memrealtime, 100 MHz):
run the one-image latency steps, then print the median per phase.
    SOD_LIB_PATH=tools/stampvar/libsod.so python tools/fused_stamps.py [img1]"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.argv = [sys.argv[0]] + (sys.argv[1:] or ["img1"]) + ["40"]
sys.path.insert(0, HERE)
import latency_probe  # noqa: E402

latency_probe.main()
from sift_based_od_amd import _lib  # noqa: E402

buf = (C.c_ulonglong * (64 * 8))()
assert _lib.lib().sod_debug_fusedstamps(buf) == 0
a = np.array(buf, dtype=np.uint64).reshape(64, 8)
a = a[a[:, 0] > 0]
names = ["init", "pose+hash", "voting list", "vote eval", "emit", "offsets", "members"]
d = np.diff(a[:, :7].astype(np.int64), axis=1) / 100.0   # us
for i, n in enumerate(names[1:]):
    print("%-12s median %7.2f us" % (n, float(np.median(d[:, i]))))
print("total        median %7.2f us" % float(np.median(d.sum(1))))
print("emit: scan %.2f us, emission %.2f us" % (float(np.median((a[:, 7].astype(np.int64) - a[:, 3].astype(np.int64)) / 100.0)),
                                             float(np.median((a[:, 4].astype(np.int64) - a[:, 7].astype(np.int64)) / 100.0))))
