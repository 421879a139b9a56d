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
if len(sys.argv) > 4 and int(sys.argv[4]):   # CU split (sod_set_cu_reserve) for the matcher
    ctx.set_cu_reserve(int(sys.argv[4]))
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
if hasattr(ctx._L, "sod_debug_stamps"):   # diagnostic build: in-kernel clock
    import ctypes as C
    st = np.zeros((4096, 8), np.uint64)
    ctx._L.sod_debug_stamps(st.ctypes.data_as(C.c_void_p), 4096)
    nb = int((st[:, 3] > st[:, 1]).sum())
    st = st[:nb]
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(REPO, "gpurun_out", "stamps_%s.npy" % impl), st)
    ghz = (st[:, 2] - st[:, 0]) / (st[:, 3] - st[:, 1]) * 0.1
    dur = (st[:, 3] - st[:, 1]) / 100.0   # us (100 MHz realtime)
    print("in-kernel clock: median %.3f GHz (min %.3f max %.3f) over %d work-groups; "
          "WG duration us: min %.0f median %.0f max %.0f; start skew %.1f us, span %.0f us" % (
              np.median(ghz), ghz.min(), ghz.max(), len(st), dur.min(), np.median(dur),
              dur.max(), (st[:, 1].max() - st[:, 1].min()) / 100.0,
              (st[:, 3].max() - st[:, 1].min()) / 100.0), flush=True)
    # per-WG placement: HW_ID (gfx9: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13])
    hw = st[:, 4].astype(np.int64)
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    sh = (hw >> 12) & 1
    xcc = st[:, 5].astype(np.int64) & 0xF
    place = (xcc * 8 + se) * 32 + sh * 16 + cu
    uniq, inv, cnt = np.unique(place, return_inverse=True, return_counts=True)
    shared = cnt[inv] > 1
    print("WGs alone on a CU: %d, duration median %.0f us; sharing: %d, median %.0f us" % (
        (~shared).sum(), np.median(dur[~shared]) if (~shared).any() else 0,
        shared.sum(), np.median(dur[shared])), flush=True)
    for x in range(8):
        m = xcc == x
        if m.any():
            print("  xcc %d: %d WGs, duration median %.0f max %.0f us" % (
                x, m.sum(), np.median(dur[m]), dur[m].max()), flush=True)
    order = np.argsort(-dur)[:8]
    print("  slowest WGs (block, us, xcc, cu-slot):", [(int(b), int(dur[b]), int(xcc[b]),
                                                     int(place[b])) for b in order], flush=True)
if hasattr(ctx._L, "sod_debug_times"):   # diagnostic build: slow-path cycles per wave
    import ctypes as C
    tm = np.zeros((32768, 4), np.uint64)
    ctx._L.sod_debug_times(tm.ctypes.data_as(C.c_void_p), 1)
    ctx.match()
    ctx.synchronize()
    ctx._L.sod_debug_times(tm.ctypes.data_as(C.c_void_p), 0)
    cyc, n, tot = tm[:, 0].astype(np.float64), tm[:, 1].astype(np.float64), tm[:, 2].astype(np.float64)
    if os.environ.get("TIME2"):   # SOD_I8_TIME2 build: stage waits / seed / prologue per wave
        live = tot > 0
        med = lambda a: float(np.median(a[live]))  # noqa: E731
        print("per wave (median cycles): unit %.0f, stage-top waits %.0f (%.1f %%), seed %.0f, "
              "start to first barrier %.0f" % (med(tot), med(cyc), 100.0 * cyc[live].sum() / tot[live].sum(),
                                               med(n), med(tm[:, 3].astype(np.float64))), flush=True)
        cyc = np.zeros(1)
    print("slow path: %.0f cycles per entry, %.2f entries per wave, %.1f %% of the waves' cycles "
          "(work unit median %.0f cycles)" % (cyc.sum() / max(n.sum(), 1), n.sum() / max((tot > 0).sum(), 1),
                                             100.0 * cyc.sum() / max(tot.sum(), 1), np.median(tot[tot > 0])),
          flush=True)
if hasattr(ctx._L, "sod_debug_counts"):   # diagnostic build: slow-path statistics
    import ctypes as C
    cnt = np.zeros(8, np.uint64)
    ctx._L.sod_debug_counts(cnt.ctypes.data_as(C.c_void_p), 1)
    ctx.match()
    ctx.synchronize()
    ctx._L.sod_debug_counts(cnt.ctypes.data_as(C.c_void_p), 0)
    print("slow-path entries / wave-subtile %.4f, hit tiles / wave-subtile %.4f (%d wave-subtiles); "
          "first 64 subtiles of a chunk: %.1f %% of entries, %.1f %% of hit tiles" % (
              cnt[0] / cnt[2], cnt[1] / cnt[2], cnt[2], 100.0 * cnt[3] / max(cnt[0], 1),
              100.0 * cnt[4] / max(cnt[1], 1)), flush=True)
    if cnt[7]:   # s_memtime cycles inside the slow path (timer + atomics included)
        print("slow path: %.0f cycles per entry (s_memtime)" % (cnt[7] / max(cnt[0], 1)), flush=True)
    if cnt[5]:   # flipped kernel: (query, row-slot) groups with a passing lane, passing lanes
        print("passing slots / wave-subtile %.4f, passing lanes / slot %.2f" % (
            cnt[5] / cnt[2], cnt[6] / cnt[5]), flush=True)
ctx.ratio(0.75)
idx1, d1, d2, good = ctx.match_result()
print("checksum", int(idx1.astype(np.int64).sum()), float(d1.astype(np.float64).sum()), flush=True)
