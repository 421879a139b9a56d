"""Host cost of one pipeline step (sod_pipeline_enqueue) with the device idle -- the CPU time
of the launches themselves, no waiting on earlier steps -- against the device time of a
step run back to back.  python tools/enqueue_cost.py [config ...] (img500x1M, c2)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

CONFIGS = {"img500x1M": (500, 1000, (32, 32, 8, 12)), "c2": (10000, 100, (15, 15, 15, 15))}


def main():
    for name in sys.argv[1:] or ["img500x1M", "c2"]:
        nq, nimg, bins = CONFIGS[name]
        db = synthetic.make_database(nimg, 1000, seed=0, workers=16)
        qs = synthetic.make_queries(nq, seed=1, db_seed=0, kp_per_image=1000)
        ctx = _lib.Context(0)
        ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
        ctx.upload_db(db.des)
        ctx.upload_queries(qs.des, qs.kp)
        ctx.set_overlap(True)
        ctx.set_stage_timing(False)   # as bench.py's timed steps
        for _ in range(200):
            ctx.pipeline(qs.shape, bins)
        ctx.synchronize()
        idle = []
        for _ in range(200):
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.pipeline(qs.shape, bins)
            idle.append(time.perf_counter() - t0)
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            ctx.pipeline(qs.shape, bins)
        ctx.synchronize()
        b2b = (time.perf_counter() - t0) / 200
        print("%s: enqueue with the device idle %.1f us (median; p90 %.1f), back-to-back step %.1f us"
              % (name, 1e6 * np.median(idle), 1e6 * np.percentile(idle, 90), 1e6 * b2b), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
