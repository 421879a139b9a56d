"""Small-query-set matcher: the register-streamed kernel (match_s.hip) against the LDS-ring
kernel (match_i8.hip) in ONE process on one box, interleaved rounds, same inputs.
    python tools/ab_small.py [configs]      (configs: comma list of the names below)
Checks the two kernels' results bit for bit (idx1, d1, d2, good after the 0.75 ratio) and
prints per kernel the steady-state launch time (matcher's own HIP event ring, back-to-back
launches) and the int8 peak fraction."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

CONFIGS = {  # name: (queries, DB rows)
    "img1": (500, 1_000_000), "c2": (10_000, 100_000), "q2k": (2000, 1_000_000),
    "odd": (400, 77_777), "tiny": (700, 1000), "q384": (384, 250_000), "q5k": (5000, 1_000_000),
}
WARM, LAUNCH, ROUNDS = 20, 64, int(os.environ.get("ROUNDS", "3"))
RESERVE = int(os.environ.get("RESERVE", "0"))


def counts(ctx, reset):
    import ctypes as C
    if not hasattr(ctx._L, "sod_debug_scounts"):   # diagnostic build only
        return None
    c = np.zeros(8, np.uint64)
    ctx.synchronize()
    ctx._L.sod_debug_scounts(c.ctypes.data_as(C.c_void_p), 1 if reset else 0)
    return c


def run(ctx, kernel, n):
    ctx.set_match_kernel(kernel)
    for _ in range(WARM):
        ctx.match()
    ctx.synchronize()
    for _ in range(n):
        ctx.match()
    ctx.synchronize()
    ts = ctx.match_times(min(n, 64))
    ctx.ratio(0.75)
    return ts, ctx.match_result()


def main():
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else list(CONFIGS)
    bad = 0
    for name in names:
        nq, ndb = CONFIGS[name]
        rng = np.random.default_rng(0)
        db = synthetic.sift_like_descriptors(np.random.default_rng(7), ndb)
        q = synthetic.sift_like_descriptors(rng, nq)
        k = nq // 5
        q[:k] = np.clip(db[rng.integers(0, ndb, k)].astype(int) + rng.integers(-3, 4, (k, 128)),
                        0, 255).astype(np.uint8)
        q[k:k + 4] = db[:4]   # exact duplicates of DB rows (distance 0)
        ctx = _lib.Context(0)
        ctx.upload_db(db)
        ctx.upload_queries(q)
        if RESERVE:
            ctx.set_cu_reserve(RESERVE)
        times = {"ring": [], "streamed": []}
        res = {}
        for r in range(ROUNDS):
            for kern in ("ring", "streamed"):
                counts(ctx, True)
                ts, out = run(ctx, kern, LAUNCH)
                c = counts(ctx, True)
                if c is not None and kern == "streamed" and r == 0:
                    nl = WARM + LAUNCH
                    print("  %s counts per launch: windows %.0f, hit windows %.0f (%.2f %%), hit tiles "
                          "%.0f (%.2f per hit window)" % (name, c[0] / nl, c[1] / nl,
                                                          100.0 * c[1] / max(1, c[0]), c[2] / nl,
                                                          c[2] / max(1, c[1])), flush=True)
                times[kern].append(float(np.median(ts)))
                if kern not in res:
                    res[kern] = out
                else:
                    for a, b in zip(res[kern], out):
                        if not np.array_equal(a, b):
                            print("  %s: %s results differ between rounds" % (name, kern))
                            bad += 1
        if hasattr(ctx._L, "sod_debug_sstamps"):   # diagnostic build: per-wave timeline
            import ctypes as C
            hits = np.zeros((4096, 9), np.uint32)
            ctx._L.sod_debug_shits(hits.ctypes.data_as(C.c_void_p), 1)
            run(ctx, "streamed", 8)
            ctx.synchronize()
            ctx._L.sod_debug_shits(hits.ctypes.data_as(C.c_void_p), 1)
            nl = WARM + 8
            hw = hits[hits.sum(axis=1) > 0].astype(np.float64) / nl
            print("  %s hit tiles per wave and launch, bodies 0..7 and the rest: %s (total %.1f)" % (
                name, " ".join("%.2f" % v for v in hw.mean(axis=0)), hw.sum(axis=1).mean()))
            st = np.zeros((4096, 28), np.uint64)
            ctx._L.sod_debug_sstamps(st.ctypes.data_as(C.c_void_p))
            st = st.astype(np.int64)   # (one config per process: rows of other grids stay)
            st = st[st[:, 25] > 0]
            clk = (st[:, 25] - st[:, 0]) / ((st[:, 27] - st[:, 26]) / 100.0)   # MHz
            rel = st[:, :26] - st[:, :1]   # each wave against its own start (XCD clocks differ)
            print("  %s stamps over %d waves (cycles after the wave's start: median [p10 p90]); "
                  "clock %.0f MHz" % (name, len(st), np.median(clk)))
            labels = ["start", "frags", "s.scan", "s.push", "s.bar", "s.apply", "s.load", "s.pull",
                      "w0", "sl0", "x0", "w1", "sl1", "x1", "w2", "sl2", "x2"] + \
                ["body%d" % b for b in range(1, 9)] + ["end"]
            for i, lab in enumerate(labels):
                if not lab:
                    continue
                ok = st[:, i] > 0
                col = rel[ok, i]
                if len(col):
                    print("    %-7s %8.0f [%8.0f %8.0f]" % (lab, np.median(col), np.percentile(col, 10),
                                                            np.percentile(col, 90)), flush=True)
        same = all(np.array_equal(a, b) for a, b in zip(res["ring"], res["streamed"]))
        if not same:
            bad += 1
            i1r, d1r, d2r, gr = res["ring"]
            i1s, d1s, d2s, gs = res["streamed"]
            diff = np.nonzero((i1r != i1s) | (d1r != d1s) | (d2r != d2s))[0]
            print("  %s: MISMATCH at %d queries, e.g. %s" % (name, len(diff), diff[:8]))
            for qq in diff[:4]:
                print("    q%d ring (%d %r %r) streamed (%d %r %r)" % (
                    qq, i1r[qq], d1r[qq], d2r[qq], i1s[qq], d1s[qq], d2s[qq]))
        line = "%-5s %6d x %8d  same=%s" % (name, nq, ndb, same)
        for kern in ("ring", "streamed"):
            ms = min(times[kern])
            frac = 256.0 * nq * ndb / (ms / 1e3) / 5e15
            line += "  %s %.4f ms (%.1f %%)" % (kern, ms, 100 * frac)
        print(line, flush=True)
        del ctx
    print("FAIL" if bad else "OK")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
