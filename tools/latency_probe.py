"""One query image alone, start to finish (bench.py's single_image_latency_ms): host clock
between two device syncs around one pipeline step, tail on the whole chip, matcher on its own
stream (the bench's context after its CU split is undone).  Prints the median latency and the
host enqueue time; run under rocprofv3 --kernel-trace for the kernel timeline
(tools/latency_timeline.py).
    python tools/latency_probe.py [img1|c2|c3] [steps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

CONFIGS = {"img1": (500, 1000, (32, 32, 8, 12)), "c2": (10000, 100, (15, 15, 15, 15)),
           "c3": (50000, 1000, (32, 32, 8, 12))}


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "img1"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    nq, nimg, bins = CONFIGS[name]
    db = synthetic.make_database(nimg, 1000, seed=0, workers=16)
    qs = synthetic.make_queries(nq, seed=1, db_seed=0, kp_per_image=1000)
    ctx = _lib.Context(0)
    ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
    ctx.upload_db(db.des)
    ctx.upload_queries(qs.des, qs.kp)
    ctx.set_overlap(True)
    ctx.set_stage_timing(False)
    if os.environ.get("SOD_LAT_MATCH_TIMING", "0") != "1":
        ctx.set_match_timing(False)
    for _ in range(300 if nq < 20000 else 20):      # clock ramp
        ctx.pipeline(qs.shape, bins)
    ctx.synchronize()
    lat, host = [], []
    for _ in range(steps):
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.pipeline(qs.shape, bins)
        t1 = time.perf_counter()
        ctx.synchronize()
        t2 = time.perf_counter()
        lat.append((t2 - t0) * 1e3)
        host.append((t1 - t0) * 1e3)
        time.sleep(0.002)
    v = ctx.valid_result()
    print("%s latency median %.4f ms (min %.4f) host enqueue %.4f ms, %d valid bins"
          % (name, float(np.median(lat)), float(np.min(lat)), float(np.median(host)),
             len(v["keys"])))


if __name__ == "__main__":
    main()
