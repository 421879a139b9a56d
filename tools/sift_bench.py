"""SIFT-on-device timing: wall time per detectAndCompute of one image
(upload, whole device pipeline, keypoints + descriptors back) and the oracle's CPU time.
    python tools/sift_bench.py [h w] [reps]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

h = int(sys.argv[1]) if len(sys.argv) > 1 else 800
w = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
img = synthetic.textured_image(h, w, seed=1)
ctx = _lib.Context(0)
r = ctx.sift_detect(img)
ts = []
for _ in range(reps):
    t = time.perf_counter()
    r = ctx.sift_detect(img)
    ts.append(time.perf_counter() - t)
ts = np.array(ts) * 1e3
print("sift %dx%d: %d keypoints, %.3f ms/image (min %.3f)" % (h, w, len(r["x"]), ts.mean(), ts.min()),
      flush=True)
if "--cpu" in sys.argv:
    from oracle import sift as osift
    t = time.perf_counter()
    osift.detect_and_compute(img)
    print("oracle (C, 1 thread): %.1f ms/image" % ((time.perf_counter() - t) * 1e3))
