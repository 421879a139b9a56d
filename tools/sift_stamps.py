"""Diagnostic: phase times of the small-octave chain kernel (SOD_SIFT_STAMP build).
    SOD_LIB_PATH=tools/variants/libsiftstamp.so python tools/sift_stamps.py"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

img = synthetic.textured_image(800, 1000, seed=1)
ctx = _lib.Context(0)
for _ in range(3):
    ctx.sift_detect(img)
buf = (ctypes.c_ulonglong * 256)()
_lib.lib().sod_debug_sift_stamps(buf)
st = np.array(buf[:], np.int64)
n = int(np.argmax(st[1:] == 0)) + 1 if np.any(st[1:] == 0) else 256
d = np.diff(st[:n]) / 100.0   # 100 MHz ticks -> us
print("phases:", n - 1, "total %.1f us" % ((st[n - 1] - st[0]) / 100.0))
print(" ".join("%.1f" % x for x in d))
