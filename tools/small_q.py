"""A/B of matcher launch settings on small query sets (one query image x 1M rows, C2 10k x
100k, 2k x 1M) in ONE process on one box, interleaved: the environment variable VAR
(default SOD_MATCH_QT) takes each value of MODES in turn; results must be bit-identical.
Prints per config and mode: pipeline ms/step (back-to-back steps, overlap on), matcher kernel
ms (launch-recorded events), merge ms (stage events, isolated steps).  (Round 3 measured a
register-streamed kernel this way -- no LDS ring, DB rows loaded per wave into registers,
8 / 16 query tiles per wave: 0.128 / 0.155 ms vs 0.067 for one query image; removed.)"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

CONFIGS = {"img500x1M": (500, 1000, (32, 32, 8, 12)), "c2": (10000, 100, (15, 15, 15, 15)),
           "q2kx1M": (2000, 1000, (32, 32, 8, 12))}
VAR = os.environ.get("VAR", "SOD_MATCH_QT")
MODES = [m for m in os.environ.get("MODES", "2,4,8").split(",")]
WARM, STEPS, ROUNDS = 300, 200, 2


def run(ctx, qs, bins, steps):
    for _ in range(steps):
        ctx.pipeline(qs.shape, bins)
    ctx.synchronize()


def main():
    out = {}
    for name in os.environ.get("CONFIGS", "img500x1M,c2,q2kx1M").split(","):
        nq, nimg, bins = CONFIGS[name]
        db = synthetic.make_database(nimg, 1000, seed=0, workers=16)
        qs = synthetic.make_queries(nq, seed=1, db_seed=0, kp_per_image=1000)
        ctx = _lib.Context(0)
        ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
        ctx.upload_db(db.des)
        ctx.upload_queries(qs.des, qs.kp)
        ctx.set_overlap(True)
        ref = None
        res = {m: {"step": [], "kernel": [], "merge": []} for m in MODES}
        for r in range(ROUNDS):
            for m in MODES:
                os.environ[VAR] = m
                ctx.set_stage_timing(False)
                run(ctx, qs, bins, WARM if r == 0 else 50)
                t0 = time.perf_counter()
                run(ctx, qs, bins, STEPS)
                res[m]["step"].append((time.perf_counter() - t0) * 1000.0 / STEPS)
                res[m]["kernel"].append(float(np.mean(ctx.match_times(64))))
                ctx.set_stage_timing(True)
                st = []
                for _ in range(5):
                    ctx.pipeline(qs.shape, bins)
                    ctx.synchronize()
                    st.append(ctx.stage_ms())
                res[m]["merge"].append(float(np.mean([x[1] for x in st])))
                got = ctx.match_result()
                if os.environ.get("SMALLQ_NOCHECK"):   # timing-only builds (SOD_I8_EXP)
                    pass
                elif ref is None:
                    ref = [np.asarray(a).copy() for a in got]
                else:
                    for a, b in zip(ref, got):
                        assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8)), (name, m)
        peak = 5.0e15
        for m in MODES:
            k = float(np.median(res[m]["kernel"]))
            res[m] = {"step_ms": float(np.median(res[m]["step"])), "kernel_ms": k,
                      "merge_ms": float(np.median(res[m]["merge"])),
                      "kernel_frac_i8": 256.0 * nq * len(db.des) / (k * 1e-3) / peak}
        out[name] = res
        print(name, json.dumps(res), flush=True)
        ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
