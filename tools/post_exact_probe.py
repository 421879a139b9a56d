"""C3 post-processing with the survivors' exact x / y means (sod_set_post_exact) vs the
device means, and the exact-means call alone."""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

db = synthetic.make_database(1000, 1000, seed=0)
qs = synthetic.make_queries(50000, seed=1, db_seed=0, kp_per_image=1000)
c = _lib.Context(0)
c.set_keypoints(db.kp, db.img, db.centroid, db.size)
c.upload_db(db.des)
c.upload_queries(qs.des, qs.kp)
c.pipeline(qs.shape, (32, 32, 8, 12), vote_threshold=5, x_factor=128.0, y_factor=128.0)
c.synchronize()
a = c.affine_result()
v = c.valid_result()
surv = np.nonzero(a["survived"])[0]
n = np.diff(v["offsets"])[surv]
print("survivors", len(surv), "members", int(n.sum()), "max", int(n.max()), flush=True)


def t(fn, reps=10):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) * 1e3 / reps


print("exact_means(survivors) %.3f ms" % t(lambda: c.exact_means(surv)))
print("postprocess exact %.3f ms" % t(lambda: c.postprocess()))
c.set_post_exact(False)
print("postprocess device means %.3f ms" % t(lambda: c.postprocess()))
c.close()
