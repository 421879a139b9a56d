"""C3 selection shape: member counts of the valid bins (the PoseBin means chain is as long
as the largest bin)."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402
from sift_based_od_amd.database import Keypoints  # noqa: E402

db = synthetic.make_database(1000, 1000, seed=0)
qs = synthetic.make_queries(50000, seed=1, db_seed=0, kp_per_image=1000)
c = _lib.Context(0)
c.set_keypoints(db.kp, db.img, db.centroid, db.size)
c.upload_db(db.des)
c.upload_queries(qs.des, qs.kp)
c.pipeline(qs.shape, (32, 32, 8, 12), vote_threshold=5, x_factor=128.0, y_factor=128.0)
r = c.valid_result()
n = np.diff(r["offsets"])
print("bins", len(n), "members", int(n.sum()), "max", int(n.max()), "top", np.sort(n)[-8:].tolist(),
      "p50", int(np.median(n)))
c.close()
