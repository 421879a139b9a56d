"""SIFT on one synthetic 1000 x 800 texture (as bench.py's extras), repeated: for
rocprofv3 --kernel-trace --stats.  python tools/sift_prof.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
lane_order = int(sys.argv[2]) if len(sys.argv) > 2 else -1   # -1: the context's probe decides
img = synthetic.textured_image(800, 1000, seed=2000)
c = _lib.Context(0)
if lane_order >= 0:
    c.sift_set_lane_order(lane_order)
for _ in range(5):
    c.sift_detect(img)
c.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    r = c.sift_detect(img)
print("keypoints %d, %.3f ms per image" % (len(r["x"]), 1000 * (time.perf_counter() - t0) / reps))
