"""Phase times of select_small_kernel (SOD_SEL_STAMP build, tools/variants/libsod_selst.so):
one query image x 1M rows, pipelined steps as bench.py img1; prints the median us per phase.
    SOD_LIB_PATH=tools/variants/libsod_selst.so python tools/sel_stamps.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

nq = int(sys.argv[1]) if len(sys.argv) > 1 else 500
db = synthetic.make_database(1000, 1000, seed=0, workers=16)
qs = synthetic.make_queries(nq, seed=1, db_seed=0, kp_per_image=1000)
ctx = _lib.Context(0)
ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
ctx.upload_db(db.des)
ctx.upload_queries(qs.des, qs.kp)
ctx.set_cu_reserve(1)
ctx.set_stage_timing(False)
for _ in range(300):
    ctx.pipeline(qs.shape, (32, 32, 8, 12))
ctx.synchronize()
st = np.zeros((64, 5), np.uint64)
assert ctx._L.sod_debug_selstamps(st.ctypes.data_as(C.c_void_p)) == 0
d = np.diff(st[:, :4].astype(np.int64), axis=1) / 100.0   # 100 MHz ticks -> us
print("valid bins %d; phase us (median of 64): select %.2f, offsets %.2f, members %.2f; total %.2f"
      % (int(np.median(st[:, 4])), *np.median(d, axis=0), np.median(d.sum(axis=1))))
