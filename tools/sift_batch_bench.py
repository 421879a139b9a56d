"""SIFT batch throughput (sod_sift_detect_batch) vs one image at a time, and the host-side
enqueue cost.  python tools/sift_batch_bench.py [n_images] [h w]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
h = int(sys.argv[2]) if len(sys.argv) > 2 else 800
w = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
imgs = [synthetic.textured_image(h, w, seed=2000 + k) for k in range(n)]
ctx = _lib.Context(0)
ctx.sift_detect_batch(imgs, results=False)
for rep in range(2):
    t = time.perf_counter()
    counts = ctx.sift_detect_batch(imgs, results=False)
    tb = (time.perf_counter() - t) * 1e3
    t = time.perf_counter()
    for im in imgs:
        ctx.sift_detect_batch([im], results=False)
    ts = (time.perf_counter() - t) * 1e3
    print("%s: %d images %dx%d, %d keypoints: batch %.2f ms (%.3f ms/image, %.0f images/s); "
          "one at a time %.3f ms/image" % (os.path.basename(_lib.LIB_PATH), n, w, h, counts.sum(), tb,
                                          tb / n, n / tb * 1e3, ts / n), flush=True)
