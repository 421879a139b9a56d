"""B small query images (C1-like, 500 keypoints each) against the 1M-row
DB -- one matcher pass for the whole batch vs one full pipeline per image."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, run_query_batch, synthetic  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
nq = int(sys.argv[2]) if len(sys.argv) > 2 else 500
db = synthetic.make_database(1000, 1000, seed=0)
imgs = []
for k in range(B):
    qs = synthetic.make_queries(nq, seed=100 + k, db_seed=0, kp_per_image=1000)
    imgs.append((qs.des, qs.kp, qs.shape))
ctx = _lib.Context(0)
ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
ctx.upload_db(db.des)


def per_image():
    for des, kp, shape in imgs:
        ctx.upload_queries(des, kp)
        ctx.pipeline(shape, (32, 32, 8, 12))


def batched():
    run_query_batch(ctx, imgs, bins=(32, 32, 8, 12), results=False, fused=False)


def fused():
    run_query_batch(ctx, imgs, bins=(32, 32, 8, 12), results=False, fused=True)


def match_only():
    des = np.concatenate([d for d, _, _ in imgs])
    ctx.upload_queries(des)
    ctx.match()


for name, fn in (("per-image pipeline", per_image), ("batched, windowed stages", batched),
                 ("batched, fused stages", fused), ("batched matcher alone", match_only)):
    fn()
    ctx.synchronize()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        fn()
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / reps
    pairs = B * nq * len(db)
    print("%-24s %d images x %d queries: %8.2f ms per batch, %.3g pairs/s, %.1f images/s" % (
        name, B, nq, dt * 1e3, pairs / dt, B / dt), flush=True)
