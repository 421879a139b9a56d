"""Valid-bin size statistics of the bench workload (diagnostic for the select stage)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
nq, nimg, kpi, bins = {"c3": (50000, 1000, 1000, (32, 32, 8, 12))}[cfg]
db = synthetic.make_database(nimg, kpi, seed=0)
qs = synthetic.make_queries(nq, seed=1, db_seed=0, kp_per_image=kpi)
ctx = _lib.Context(0)
ctx.set_impl("i8")
ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
ctx.upload_db(db.des)
ctx.upload_queries(qs.des, qs.kp)
ctx.pipeline(qs.shape, bins, ratio=0.75, vote_threshold=5, affine_threshold=4,
             x_factor=128.0, y_factor=128.0, run_affine=True)
ctx.synchronize()
v = ctx.valid_result()
sz = np.diff(v["offsets"])
print("V", len(sz), "M", int(sz.sum()), "max", int(sz.max()), "p50/p90/p99",
      np.percentile(sz, [50, 90, 99]).tolist())
print("top sizes", np.sort(sz)[-10:].tolist())
keys, votes = ctx.all_bins()
print("all bins", len(keys), "votes", int(votes.sum()), "max votes", int(votes.max()))
for i in range(5):
    ctx.pipeline(qs.shape, bins, ratio=0.75, vote_threshold=5, affine_threshold=4,
                 x_factor=128.0, y_factor=128.0, run_affine=True)
    ctx.synchronize()
    print("stage_ms", [round(x, 4) for x in ctx.stage_ms()])
