"""Main.run for one query image (500 keypoints) against the 1M-row DB, split into its host
phases (median of 200 runs): the pipeline enqueue (ctypes call + C++ enqueue), the results
fetch (wait for the device + the staging read + numpy arrays), final_pose_from_arrays and
the rest of Main.run; the device step alone (enqueue -> synchronize, no read) beside it.
    python tools/run_timeline.py [n_images_in_db] [queries]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import Main, SiftDatabase, _lib, synthetic  # noqa: E402
from sift_based_od_amd.pipeline import POS_FACTOR  # noqa: E402
from sift_based_od_amd.postprocessing import final_pose_from_arrays  # noqa: E402


def spin(sec):
    # wait with the CPU busy (a sleep lets the core idle and cools its caches: the reads after
    # it would measure the wake-up, not the read)
    t = time.perf_counter() + sec
    while time.perf_counter() < t:
        pass


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
    for _ in range(50):
        m.run(bins)
    c.synchronize()
    parts = ("match", "valid", "affine", "post")
    ph = {k: [] for k in ("enqueue", "fetch", "final_pose", "run_total", "device_step",
                          "fetch_after_sync", "fetch_c_only", "fetch_c_match", "fetch_c_again",
                          "sync_idle", "sync_first", "enqueue_after_idle")}
    for _ in range(200):
        t0 = time.perf_counter()
        c.pipeline(m.rgb_query.shape, bins, 0.75, 5, 4, POS_FACTOR * 4.0, POS_FACTOR * 4.0, True,
                   stage=parts)
        t1 = time.perf_counter()
        r = c.results(parts=parts)
        t2 = time.perf_counter()
        final_pose_from_arrays(r["post"])
        t3 = time.perf_counter()
        ph["enqueue"].append(t1 - t0)
        ph["fetch"].append(t2 - t1)
        ph["final_pose"].append(t3 - t2)
        t0 = time.perf_counter()
        m.run(bins)
        ph["run_total"].append(time.perf_counter() - t0)
        c.synchronize()
        t0 = time.perf_counter()
        c.pipeline(m.rgb_query.shape, bins, 0.75, 5, 4, POS_FACTOR * 4.0, POS_FACTOR * 4.0, True)
        c.synchronize()
        ph["device_step"].append(time.perf_counter() - t0)
        # the read alone, the device idle (a busy wait, not synchronize: any API call makes the
        # staged results stale): host work of sod_results_fetch + the Python arrays
        c.pipeline(m.rgb_query.shape, bins, 0.75, 5, 4, POS_FACTOR * 4.0, POS_FACTOR * 4.0, True,
                   stage=parts)
        spin(0.002)
        t0 = time.perf_counter()
        c.results(parts=parts)
        ph["fetch_after_sync"].append(time.perf_counter() - t0)
        c.pipeline(m.rgb_query.shape, bins, 0.75, 5, 4, POS_FACTOR * 4.0, POS_FACTOR * 4.0, True,
                   stage=parts)
        spin(0.002)
        rs = _lib.Results()
        mask = sum(c.RES[p] for p in parts)
        t0 = time.perf_counter()
        c._L.sod_results_fetch(c._h, mask, _lib.C.byref(rs))
        ph["fetch_c_only"].append(time.perf_counter() - t0)
        # the same read of the matches alone (no key decode, no post-processing walk), then an
        # idle sod_synchronize (set_dev + three stream queries)
        c.pipeline(m.rgb_query.shape, bins, 0.75, 5, 4, POS_FACTOR * 4.0, POS_FACTOR * 4.0, True,
                   stage=parts)
        spin(0.002)
        t0 = time.perf_counter()
        c._L.sod_results_fetch(c._h, 1, _lib.C.byref(rs))
        ph["fetch_c_match"].append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        c._L.sod_results_fetch(c._h, 1, _lib.C.byref(rs))
        ph["fetch_c_again"].append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        c._L.sod_synchronize(c._h)
        ph["sync_idle"].append(time.perf_counter() - t0)
        # the first stream query after a finished pipeline, and an enqueue that follows a
        # finished pipeline with no query in between
        c.pipeline(m.rgb_query.shape, bins, 0.75, 5, 4, POS_FACTOR * 4.0, POS_FACTOR * 4.0, True,
                   stage=parts)
        spin(0.002)
        t0 = time.perf_counter()
        c._L.sod_synchronize(c._h)
        ph["sync_first"].append(time.perf_counter() - t0)
        c.pipeline(m.rgb_query.shape, bins, 0.75, 5, 4, POS_FACTOR * 4.0, POS_FACTOR * 4.0, True,
                   stage=parts)
        spin(0.002)
        t0 = time.perf_counter()
        c.pipeline(m.rgb_query.shape, bins, 0.75, 5, 4, POS_FACTOR * 4.0, POS_FACTOR * 4.0, True,
                   stage=parts)
        ph["enqueue_after_idle"].append(time.perf_counter() - t0)
        c.synchronize()
    # the Python side of the read, piece by piece (the device idle, results staged)
    rs = _lib.Results()
    mask = sum(c.RES[p] for p in parts)
    c._L.sod_results_fetch(c._h, mask, _lib.C.byref(rs))
    r = dict(zip(_lib._RES_DTYPE.names, np.frombuffer(rs, _lib._RES_DTYPE)[0].tolist()))
    lo = min(r[k] for k in ("idx1", "d1", "d2", "good") if r[k])
    nbytes = 9 * r["nq"] + 4096
    pinned = np.empty(nbytes, np.uint8)
    plain = np.ones(nbytes, np.uint8)
    for name, fn in (("memmove_pinned_10KB", lambda: _lib.C.memmove(pinned.ctypes.data, lo, nbytes)),
                     ("memmove_plain_10KB", lambda: _lib.C.memmove(pinned.ctypes.data, plain.ctypes.data, nbytes))):
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ph[name] = ts
    for k, v in ph.items():
        print("  %-12s median %.4f ms  min %.4f ms" % (k, 1e3 * float(np.median(v)), 1e3 * min(v)))


if __name__ == "__main__":
    main()
