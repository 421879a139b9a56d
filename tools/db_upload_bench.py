"""DB upload time, raw descriptors (H2D + validation + pack kernel) vs
the packed image (one H2D copy), for a 1M-row shard."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

nimg = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
db = synthetic.make_database(nimg, 1000, seed=0)
ctx = _lib.Context(0)
ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
ctx.upload_db(db.des)
img = ctx.export_packed()
for name, fn in (("raw uint8 upload + pack", lambda: ctx.upload_db(db.des)),
                 ("packed image import", lambda: ctx.import_packed(img))):
    ts = []
    for i in range(6):
        ctx.synchronize()
        t0 = time.perf_counter()
        fn()
        ctx.synchronize()
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts[1:]) * 1e3
    print("%-26s %8.2f ms (min %.2f)  %d rows, %.1f MB" % (
        name, ts.mean(), ts.min(), len(db), (db.des.nbytes if "raw" in name else img.nbytes) / 1e6),
        flush=True)
