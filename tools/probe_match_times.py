"""Which call leaves a sticky HIP error behind after sod_match_times?  (debug probe)"""
import sys, ctypes
sys.path.insert(0, ".")
import sod_pkg
sod_pkg.load()
from sift_based_od_amd import _lib, synthetic

hip = ctypes.CDLL("libamdhip64.so")
db = synthetic.make_database(30, 1000, seed=51)
qs = synthetic.make_queries(int(sys.argv[1]) if len(sys.argv) > 1 else 5000, seed=52, db_seed=51, kp_per_image=1000)


def run(reserve, overlap, n_read, launches, late=False):
    with _lib.Context(0) as c:
        if late:
            c.set_keypoints(db.kp, db.img, db.centroid, db.size)
            c.upload_db(db.des)
            c.upload_queries(qs.des, qs.kp)
        if reserve:
            c.set_cu_reserve(reserve)
        elif overlap:
            c.set_overlap(True)
        if not late:
            c.set_keypoints(db.kp, db.img, db.centroid, db.size)
            c.upload_db(db.des)
            c.upload_queries(qs.des, qs.kp)
        for _ in range(launches):
            c.pipeline(qs.shape, (32, 32, 8, 12))
        c.synchronize()
        e0 = hip.hipGetLastError()
        t = c.match_times(n_read)
        e1 = hip.hipGetLastError()
        try:
            c.pipeline(qs.shape, (32, 32, 8, 12))
            c.synchronize()
            ok = "ok"
        except Exception as ex:  # noqa: BLE001
            ok = repr(ex)
        print(f"late={late} reserve={reserve} overlap={overlap} n_read={n_read} launches={launches}: "
              f"err_before={e0} err_after_times={e1} next={ok} t={t[:2]}", flush=True)


for args in [(1, False, 3, 3, True), (1, False, 30, 40, True), (0, True, 3, 3, True)]:
    run(*args)
