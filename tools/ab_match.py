"""Matcher-only timing for A/B of kernel variants (one process per library build):
    SOD_LIB_PATH=tools/variants/libX.so python tools/ab_match.py [nq] [n_images]
Prints the mean/min matcher kernel time (HIP events) and the bf16 MFMA fraction."""
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
impl = sys.argv[3] if len(sys.argv) > 3 else "bf16"
rng = np.random.default_rng(0)
db = np.concatenate([synthetic.sift_like_descriptors(np.random.default_rng([0, i]), 1000)
                     for i in range(nimg)])
q = synthetic.sift_like_descriptors(rng, nq)
q[: nq // 5] = np.clip(db[rng.integers(0, len(db), nq // 5)].astype(int) +
                       rng.integers(-3, 4, (nq // 5, 128)), 0, 255).astype(np.uint8)
ctx = _lib.Context(0)
ctx.set_impl(impl)
ctx.upload_db(db)
ctx.upload_queries(q)
ts = []
for i in range(12):
    ctx.match()
    ctx.synchronize()
    if i >= 2:
        ts.append(ctx.last_match_ms())
ts = np.array(ts)
tf = 256.0 * nq * len(db) / (ts.mean() / 1e3) / 1e12
peak = 2500.0 if impl == "bf16" else 5000.0   # dense bf16 / int8 MFMA peaks
print("%s [%s]: match %.3f ms (min %.3f)  %.0f T(FL)OP/s  frac %.3f  %.3g pairs/s" % (
    os.path.basename(_lib.LIB_PATH), impl, ts.mean(), ts.min(), tf, tf / peak,
    nq * len(db) / (ts.mean() / 1e3)), flush=True)
ctx.ratio(0.75)
idx1, d1, d2, good = ctx.match_result()
print("checksum", int(idx1.astype(np.int64).sum()), float(d1.astype(np.float64).sum()), flush=True)
