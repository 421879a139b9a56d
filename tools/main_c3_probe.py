"""Where main.py-shaped get_valid_bins spends its time at C3 (pipeline.Main, staged calls):
select enqueue, the device selection's download (guard resolve included) and the PoseBin
objects, each timed on the host after a device sync."""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import Main, SiftDatabase, _lib, synthetic  # noqa: E402
from sift_based_od_amd.hough import posebins_from_device  # noqa: E402

db = synthetic.make_database(1000, 1000, seed=0)
qs = synthetic.make_queries(50000, seed=1, db_seed=0, kp_per_image=1000)
bins = (32, 32, 8, 12)
c = _lib.Context(0)
m = Main(c)
m.set_database(SiftDatabase(db.des, db.kp, db.img, db.centroid, db.size))
m.get_query_features(qs.des, qs.kp, qs.shape)
for rep in range(3):   # run_matcher's parts
    t = {}
    t0 = time.perf_counter(); c.match(); c.synchronize(); t["match+sync"] = time.perf_counter() - t0
    t0 = time.perf_counter(); c.ratio(0.75); c.synchronize(); t["ratio+sync"] = time.perf_counter() - t0
    t0 = time.perf_counter(); c.float_order(); c.synchronize(); t["float_order"] = time.perf_counter() - t0
    t0 = time.perf_counter(); r = c.match_result(); t["match_result"] = time.perf_counter() - t0
    t0 = time.perf_counter(); r = c.results(parts=("match",)); t["results(match)"] = time.perf_counter() - t0
    print("matcher parts", {k: round(v * 1e3, 3) for k, v in t.items()}, flush=True)
for rep in range(4):
    t = {}
    t0 = time.perf_counter(); m.run_matcher(); t["run_matcher"] = time.perf_counter() - t0
    t0 = time.perf_counter(); m.apply_hough_transform(bins); c.synchronize(); t["hough+sync"] = time.perf_counter() - t0
    t0 = time.perf_counter(); c.select(5); c.synchronize(); t["select+sync"] = time.perf_counter() - t0
    t0 = time.perf_counter(); res = c.valid_result(); t["valid_result"] = time.perf_counter() - t0
    t0 = time.perf_counter(); res = c.results(parts=("valid",))["valid"]; t["results(valid)"] = time.perf_counter() - t0
    t0 = time.perf_counter(); vb = posebins_from_device(res, m._pair, m._size_of, 1); t["posebins"] = time.perf_counter() - t0
    t0 = time.perf_counter(); m.valid_bins = []; m.get_valid_bins(5); t["get_valid_bins"] = time.perf_counter() - t0
    t0 = time.perf_counter(); m.apply_affine_parameters(4); t["affine"] = time.perf_counter() - t0
    t0 = time.perf_counter(); m.post_process(); t["post_process"] = time.perf_counter() - t0
    m.valid_bins = []
    print("rep", rep, {k: round(v * 1e3, 3) for k, v in t.items()}, len(vb), flush=True)
c.close()
