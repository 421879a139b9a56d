"""SIFT one-image time in a bench-like process: a context split for the matcher
(sod_set_cu_reserve, overlap) plus a second context running SIFT, as bench.py's extras.
    python tools/sift_ctx_probe.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
img = synthetic.textured_image(800, 1000, seed=2000)
a = _lib.Context(0)
if os.environ.get("PROBE_SPLIT", "1") == "1":
    a.set_overlap(True)
    a.set_cu_reserve(1)
    if os.environ.get("PROBE_UNSPLIT", "0") == "1":   # bench.py undoes the split before extras
        a.set_cu_reserve(0)
c = _lib.Context(0) if os.environ.get("PROBE_SECOND", "1") == "1" else a
c.sift_detect(img)
c.sift_detect(img)
c.synchronize()
out = []
for r in (reps, reps, 200):
    t0 = time.perf_counter()
    for _ in range(r):
        c.sift_detect(img)
    out.append("%.3f" % (1000 * (time.perf_counter() - t0) / r))
imgs = [synthetic.textured_image(800, 1000, seed=2000 + k) for k in range(16)]
c.sift_detect_batch(imgs, results=False)
c.synchronize()
bt = []
for _ in range(5):
    t0 = time.perf_counter()
    c.sift_detect_batch(imgs, results=False)
    c.synchronize()
    bt.append(1000 * (time.perf_counter() - t0))
bt.sort()
print(os.environ.get("PROBE_TAG", ""), "ms per image (reps %d, %d, 200):" % (reps, reps), " ".join(out),
      "| batch of 16: %.3f ms (median of 5)" % bt[2])
