"""Probe: consecutive query images on two contexts (two streams) so one image's
Hough / select / affine tail overlaps the next image's matcher."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

db = synthetic.make_database(1000, 1000, seed=0)
qs = synthetic.make_queries(50000, seed=1, db_seed=0, kp_per_image=1000)
ctxs = []
for _ in range(2):
    c = _lib.Context(0)
    c.set_keypoints(db.kp, db.img, db.centroid, db.size)
    c.upload_db(db.des)
    c.upload_queries(qs.des, qs.kp)
    ctxs.append(c)
bins = (32, 32, 8, 12)


def run(nctx, steps):
    for c in ctxs:
        c.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        ctxs[i % nctx].pipeline(qs.shape, bins)
    for c in ctxs:
        c.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


for nctx in (1, 2, 1, 2):
    run(nctx, 10)
    print("contexts %d: %.3f ms per image" % (nctx, run(nctx, 30)), flush=True)
