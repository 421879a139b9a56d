"""Matcher A/B in steady state: back-to-back launches (the way the bench runs them), timed
per launch with the matcher's own HIP event ring (sod_match_times).
    SOD_LIB_PATH=tools/variants/libX.so python tools/ab_i8.py [nq] [n_images] [launches] [reserve]
Prints mean/median kernel ms, the int8 peak fraction and a result checksum."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

nq = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
nimg = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
nl = int(sys.argv[3]) if len(sys.argv) > 3 else 40
reserve = int(sys.argv[4]) if len(sys.argv) > 4 else 1
rng = np.random.default_rng(0)
db = synthetic.sift_like_descriptors(np.random.default_rng(7), nimg * 1000)
q = synthetic.sift_like_descriptors(rng, nq)
q[: nq // 5] = np.clip(db[rng.integers(0, len(db), nq // 5)].astype(int) +
                       rng.integers(-3, 4, (nq // 5, 128)), 0, 255).astype(np.uint8)
ctx = _lib.Context(0)
ctx.upload_db(db)
ctx.upload_queries(q)
if reserve:
    ctx.set_cu_reserve(reserve)
else:
    ctx.set_overlap(True)
for _ in range(10):
    ctx.match()
ctx.synchronize()
for _ in range(nl):
    ctx.match()
ctx.synchronize()
ts = ctx.match_times(min(nl, 64))
tops = 256.0 * nq * len(db) / (ts.mean() / 1e3) / 1e12
ctx.ratio(0.75)
idx1, d1, d2, good = ctx.match_result()
print("%-28s match %.4f ms (median %.4f, min %.4f)  %.0f TOP/s  frac %.4f  checksum %d %.1f %d" % (
    os.path.basename(_lib.LIB_PATH), ts.mean(), np.median(ts), ts.min(), tops, tops / 5000.0,
    int(idx1.astype(np.int64).sum()), float(d1.astype(np.float64).sum()), int(good.sum())),
    flush=True)
