"""C2 pipeline step time only (no matcher-event readback), for A/B runs of launch variants
selected by environment switches in the library.  Usage: python tools/ab_c2_step.py [steps]"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402
from sift_based_od_amd.database import Keypoints

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
db = synthetic.make_database(100, 1000, seed=0)
qs = synthetic.make_queries(10000, seed=1, db_seed=0, kp_per_image=1000)
ctx = _lib.Context(0)
ctx.set_impl("i8")
ctx.set_keypoints(Keypoints(db.kp.x, db.kp.y, db.kp.angle, db.kp.octave), db.img, db.centroid, db.size)
ctx.upload_db(db.des)
ctx.upload_queries(qs.des, qs.kp)
ctx.set_overlap(True)
ctx.set_cu_reserve(1)
ctx.set_stage_timing(False)
bins = (15, 15, 15, 15)
step = lambda: ctx.pipeline(qs.shape, bins, ratio=0.75, vote_threshold=5, affine_threshold=4,
                            x_factor=128.0, y_factor=128.0, run_affine=False)
for _ in range(10):
    step()
ctx.synchronize()
res = []
for rep in range(reps):
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.synchronize()
    res.append(1000.0 * (time.perf_counter() - t0) / steps)
print("%-24s step ms %s" % (os.environ.get("SOD_AB", "-"), " ".join("%.4f" % r for r in res)))
