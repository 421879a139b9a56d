"""Where Main.run's host time goes for one query image (500 keypoints) against the 1M-row DB
(bench.py main_path_extras IMG1): per-call wall clock inside Main.run's sequence and a
cProfile of 30 runs.     python tools/run_profile.py [n_images_in_db] [queries]"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import Main, SiftDatabase, _lib, synthetic  # noqa: E402
from sift_based_od_amd.postprocessing import final_pose_from_arrays  # noqa: E402


def main():
    nimg = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    nq = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    db = synthetic.make_database(nimg, 1000, seed=0, workers=8)
    qs = synthetic.make_queries(nq, seed=7, db_seed=0, kp_per_image=1000, n_objects=1)
    bins = (32, 32, 8, 12)
    c = _lib.Context(0)
    c.set_impl("i8")
    m = Main(c)
    m.set_database(SiftDatabase(db.des, db.kp, db.img, db.centroid, db.size))
    m.get_query_features(qs.des, qs.kp, qs.shape)
    for _ in range(10):
        m.run(bins)
    c.synchronize()

    steps = [
        ("pipeline enqueue", lambda: c.pipeline(m.rgb_query.shape, bins, 0.75, 5, 4, 128.0 * 4,
                                                128.0 * 4, True)),
        ("synchronize", c.synchronize),
        ("match_result", c.match_result),
        ("valid_result", c.valid_result),
        ("affine_result", c.affine_result),
        ("postprocess", c.postprocess),
    ]
    acc = {k: [] for k, _ in steps}
    acc["final_pose"] = []
    for _ in range(30):
        for k, fn in steps:
            t0 = time.perf_counter()
            r = fn()
            acc[k].append((time.perf_counter() - t0) * 1e3)
            if k == "postprocess":
                t0 = time.perf_counter()
                final_pose_from_arrays(r)
                acc["final_pose"].append((time.perf_counter() - t0) * 1e3)
    tot = 0.0
    for k, v in acc.items():
        med = float(np.median(v))
        tot += med
        print("  %-18s %.4f ms (min %.4f)" % (k, med, min(v)))
    print("  sum of medians     %.4f ms" % tot)
    runs = []
    for _ in range(30):
        t0 = time.perf_counter()
        m.run(bins)
        runs.append((time.perf_counter() - t0) * 1e3)
    print("  Main.run           %.4f ms (min %.4f)" % (np.median(runs), min(runs)))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(30):
        m.run(bins)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
