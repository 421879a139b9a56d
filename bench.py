"""Benchmark of the sift-based-OD hot path on MI355X (driver contract: DESIGN.md § 6).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one pass of the whole hot path over one synthetic query image:
BF k=2 matching of Nq queries against this rank's DB shard (int8 MFMA, exact) -> RCCL all-gather
+ global top-2 merge -> ratio test -> Hough pose + LDS-privatised vote histogram (own
shard) -> RCCL all-reduce of bin counts / first touch -> valid-bin selection, members,
PoseBin means -> per-bin affine LSQ + outlier rejection to a fixed point.

Workload (weak scaling): every rank holds a 1M-row DB shard (1000 model
images x 1000 keypoints), so N GPUs search an N*1M-row DB (N=8: config C4/C5, 50k x 8M);
the query image has 50k keypoints (1000x800), bins 32x32x8x12, thresholds 5/4.

value = descriptor pairs / s over the whole job = N * Nq * Nshard / step time (max over
ranks).  Hough votes/s and per-stage times are reported beside it, the matcher kernel's
achieved MFMA rate against the dense peak of its type in "roofline", and the CPU
restatement (oracle, numpy/OpenBLAS on the host cores) on a bounded slice in
"cpu_baseline".
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import _lib, synthetic  # noqa: E402

METRIC = "descriptor-pair distances/sec + Hough votes/sec per query; 1/2/4/8 GPU"
OPS_PER_PAIR = 2 * 128          # one multiply + one add per dimension
# matcher implementations: kernel name, arithmetic type, dense MFMA peak of that type on
# MI355X (MI355X_MICROARCH.md "Matrix cores": bf16 ~2.5 PF, int8 2x bf16 per clock)
IMPLS = {
    "i8": ("match_i8_kernel", "i8", 5000.0, "TOP/s"),
    "i8w": ("match_i8w_kernel", "i8", 5000.0, "TOP/s"),
    "bf16": ("match_kernel", "bf16", 2500.0, "TFLOP/s"),
}

CONFIGS = {
    # name: (queries, images per rank, keypoints per image, bins, run_affine)
    "c3": (50000, 1000, 1000, (32, 32, 8, 12), True),
    "c2": (10000, 100, 1000, (15, 15, 15, 15), False),
    "c5": (50000, 1000, 1000, (32, 32, 8, 12), True),
    # C4 / C5's whole 8M-row DB on ONE GPU (1.1 GB of int8 rows): the matcher's fraction at
    # the per-job DB size of the 8-GPU configs (not a scaling number)
    "c4x1": (50000, 8000, 1000, (32, 32, 8, 12), True),
    # main.py's own use (main.py:36-86): ONE query image (~500 keypoints) against the DB
    "img1": (500, 1000, 1000, (32, 32, 8, 12), True),
    "tiny": (2000, 20, 1000, (15, 15, 15, 15), True),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # defaults per config: ~100 ms of warmup (the clock ramps over the first ~60 ms of
    # back-to-back launches: C2 0.163 ms per step after 10 warmup steps, 0.142 after 500;
    # C3 equal after 10 or 40) and a timed region of >= 30 ms (the last query's tail is 1/K
    # of a step)
    p.add_argument("--steps", type=int, default=None, help="default 50 (C2: 200)")
    p.add_argument("--warmup", type=int, default=None, help="default 10 (C2: 500)")
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the SURVEY 8(f) side measurements (query batching, packed DB upload)")
    p.add_argument("--cpu-queries", type=int, default=4096)
    # events on a dispatch delay the stream's next kernel (~3 us per one-image step measured:
    # 0.0733 ms per step with every launch timed, 0.0714 every 4th, 0.0704 none; r04 strideab1)
    p.add_argument("--matcher-streams", type=int, default=1, choices=[1, 2],
                   help="2: one matcher stream per partial-result slot (launches overlap; "
                        "their events then span the overlap)")
    p.add_argument("--match-timing-stride", type=int, default=4,
                   help="HIP begin/end events on every S-th matcher launch of the timed region")
    p.add_argument("--contexts", type=int, default=0,
                   help="query streams over the one resident DB (sod_db_share): consecutive "
                        "query images alternate between them, so one image's Hough/select/"
                        "affine tail overlaps the next image's matcher.  Default: 2 on one "
                        "GPU, 1 with several ranks")
    p.add_argument("--overlap", type=int, default=-1, choices=[-1, 0, 1],
                   help="matcher kernel on a stream of its own, overlapping the previous query "
                        "image's Hough/select/affine stages inside ONE context (collectives "
                        "stay on the context stream).  Default: on with several ranks")
    p.add_argument("--cu-reserve", type=int, default=-1,
                   help="CUs per XCD kept off the matcher for the other stages and the RCCL "
                        "exchanges (sod_set_cu_reserve; implies --overlap 1).  Default: 3 "
                        "below 5e5 DB rows per GPU (C2), else 1 "
                        "(0 with --contexts > 1 or --overlap 0)")
    p.add_argument("--impl", default="i8", choices=sorted(IMPLS),
                   help="matcher kernel: int8 MFMA 16x16x64 (default, fastest), int8 32x32x32 "
                        "or bf16 MFMA; all bit-exact")
    p.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                   help="multi-rank exchange: RCCL on the device (default) or staged "
                        "through host memory over gloo (for >1 rank per GPU)")
    a = p.parse_args()
    short = a.config in ("c2", "tiny", "img1")
    if a.steps is None:
        a.steps = 200 if short else 50
    if a.warmup is None:
        a.warmup = 500 if short else 10
    if a.overlap == 0 and a.cu_reserve > 0:
        p.error("--cu-reserve > 0 runs the matcher on a stream of its own: it needs --overlap 1")
    return a


class Dist:
    """Rendezvous, barriers, the RCCL unique-id broadcast and the max over ranks through
    sharded.FileStore (the ranks of one node share a directory; standard library only).
    The data path uses RCCL inside libsod."""

    def __init__(self, n):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != n:
            if n != 1 or self.world != 1:
                raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (n, self.world))
        self.store = None
        if self.world > 1:
            from sift_based_od_amd.sharded import FileStore
            self.store = FileStore(self.world, self.rank)

    def barrier(self):
        if self.store:
            self.store.barrier()

    def bcast_bytes(self, b):
        return self.store.broadcast_bytes(b) if self.store else b

    def max(self, x):
        return self.store.max(x) if self.store else x

    def sum(self, x):
        return self.store.sum(x) if self.store else x

    def gather_json(self, obj):
        """Every rank's JSON-able ``obj``, in rank order (rank 0 reports them)."""
        if not self.store:
            return [obj]
        return [json.loads(b.decode()) for b in self.store.allgather_bytes(json.dumps(obj).encode())]

    def close(self):
        if self.store:
            self.store.close()


def cpu_baseline(queries, db_des, nq_sample):
    """Oracle (numpy/OpenBLAS sgemm, exact) on a bounded slice: nq_sample queries against
    the full shard.  Returns pairs/s."""
    sys.path.insert(0, REPO)
    from oracle import oracle as orc
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.environ.get("OPENBLAS_NUM_THREADS")
                  or os.cpu_count())
    try:
        from threadpoolctl import threadpool_info
        nt = [i.get("num_threads") for i in threadpool_info() if i.get("internal_api") == "openblas"]
        if nt:
            threads = int(nt[0])
    except Exception:
        pass
    q = queries[:nq_sample]
    dbf = np.ascontiguousarray(db_des, dtype=np.float32)
    t0 = time.perf_counter()
    orc.knn2_match(q, dbf, chunk=64)
    dt = time.perf_counter() - t0
    return {"value": len(q) * len(db_des) / dt, "unit": "pairs/s", "cores": threads,
            "kind": "port",
            "sample": "oracle knn2 (numpy/OpenBLAS f32 GEMM + exact top-2) of %d queries x %d DB "
                      "rows on the host, %.1f s" % (len(q), len(db_des), dt)}


def cpu_hough_baseline(qs, kp_all, img, cent, size, idx1, good, bins):
    """The oracle's Python restatement of main.py:89-119 (single thread, like the
    reference) on the same good matches: votes/s."""
    from oracle import oracle as orc
    matches = [(int(q), int(idx1[q])) for q in np.nonzero(good)[0]]
    dbkp = {"x": kp_all[0], "y": kp_all[1], "angle": kp_all[2], "octave": kp_all[3], "img": img}
    qkp = {"x": qs.kp.x, "y": qs.kp.y, "angle": qs.kp.angle, "octave": qs.kp.octave}
    t0 = time.perf_counter()
    table = orc.hough_vote(matches, qkp, dbkp, {"centroid": cent, "size": size}, bins, qs.shape)
    dt = time.perf_counter() - t0
    votes = sum(b.votes for b in table.values())
    return {"value": votes / dt, "unit": "votes/s", "cores": 1, "kind": "port",
            "sample": "oracle Hough vote loop (Python, main.py:89-119) over %d good matches, "
                      "%d votes, %.1f s" % (len(matches), votes, dt)}


def cpu_post_baseline(ctx, post):
    """The oracle's restatement of PostProcessing.py (pure Python, like the reference) on
    the same surviving bins' PoseBin means."""
    from oracle import oracle as orc
    means = ctx.valid_result()["means"][post["bin_index"]]
    t0 = time.perf_counter()
    reps = 0
    while True:
        orc.post_process(means)
        reps += 1
        if time.perf_counter() - t0 > 0.5:
            break
    dt = (time.perf_counter() - t0) / reps
    return {"value": dt * 1000.0, "unit": "ms", "cores": 1, "kind": "port",
            "sample": "oracle PostProcessing (Python, PostProcessing.py:4-112) on the %d "
                      "surviving bins, mean of %d runs" % (len(means), reps)}


def extras(c, ctx, shard, bins, n_images=64, per_image=500):
    """SURVEY 8(f) rows 2-3 on the same resident DB (outside the timed region):
    * query batching: n_images small query images (per_image keypoints) in one matcher pass
      with the fused per-image stages, vs one pipeline per image;
    * DB upload: the packed image (one copy) vs raw descriptors (+ validation and packing)."""
    from sift_based_od_amd import run_query_batch
    imgs = []
    for k in range(n_images):
        q = synthetic.make_queries(per_image, seed=1000 + k, db_seed=0, kp_per_image=1000)
        imgs.append((q.des, q.kp, q.shape))

    def timed(fn, reps=3):
        fn()
        c.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        c.synchronize()
        return (time.perf_counter() - t0) / reps * 1000.0

    def one_by_one():
        for d, k, shp in imgs:
            c.upload_queries(d, k)
            c.pipeline(shp, bins)

    t_single = timed(one_by_one)
    t_fused = timed(lambda: run_query_batch(c, imgs, bins=bins, results=False, fused=True))
    packed = ctx.export_packed()
    t_raw = timed(lambda: c.upload_db(shard))
    t_packed = timed(lambda: c.import_packed(packed))
    if c is not ctx:
        c.share_db(ctx)     # back to the shared resident DB
    sift = sift_extras(c, bins)
    return {"sift": sift,
            "query_batch": {"images": n_images, "queries_per_image": per_image,
                            "per_image_pipeline_ms": t_single, "fused_batch_ms": t_fused,
                            "images_per_s": n_images / (t_fused / 1000.0),
                            "speedup": t_single / t_fused},
            "db_upload_ms": {"raw_descriptors": t_raw, "packed_image": t_packed,
                             "rows": len(shard)}}


def sift_extras(c, bins, n_batch=16, h=800, w=1000):
    """SURVEY 8(f) row 4 (outside the timed region): SIFT detect + describe on the device
    for 1000 x 800 query images (the C3 query shape) -- one image (latency, keypoints and
    descriptors back on the host), a batch of 16 (four in flight, features left on the
    device), and 16 query images end to end (SIFT -> one matcher pass over the resident
    DB -> fused Hough / affine / post-processing)."""
    from sift_based_od_amd import sift_query_batch
    imgs = [synthetic.textured_image(h, w, seed=2000 + k) for k in range(n_batch)]

    def timed(fn, reps=5):
        fn()
        c.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        c.synchronize()
        return (time.perf_counter() - t0) / reps * 1000.0

    n_kp = len(c.sift_detect(imgs[0])["x"])
    t_one = timed(lambda: c.sift_detect(imgs[0]), reps=10)
    counts = c.sift_detect_batch(imgs, results=False)
    t_batch = timed(lambda: c.sift_detect_batch(imgs, results=False))
    t_e2e = timed(lambda: sift_query_batch(c, imgs, bins=bins, results=False), reps=3)
    return {"image": [h, w], "keypoints_per_image": n_kp,
            "single_image_ms": t_one,
            "batch_images": n_batch, "batch_ms": t_batch,
            "batch_images_per_s": n_batch / (t_batch / 1000.0),
            "batch_keypoints": int(counts.sum()),
            "image_to_pose_batch_ms": t_e2e,
            "image_to_pose_images_per_s": n_batch / (t_e2e / 1000.0)}


def main_path_extras(dev, impl, c3_data, names=("C1", "C2", "C3", "IMG1")):
    """main.py's stage-by-stage driver (pipeline.Main:
    run_matcher -> apply_hough_transform -> get_valid_bins -> apply_affine_parameters ->
    post_process, the calls main.py:182-186 makes, PoseBin objects materialised lazily) timed
    beside the one-enqueue ``Main.run`` on the same inputs: host wall clock per call, from
    the enqueue to matches, valid bins, affine results, post-processing and ``final_pose``
    on the host (every result read back, any boundary-guard resolve included) -- the
    per-image time main.py sees.  C3 and IMG1 (one query image of 500 keypoints, main.py's
    regime) use the bench's 1M-row DB; ``fused_run_ms`` is the median of 100 runs (C3: 20)
    after half as many warm-up runs."""
    from sift_based_od_amd import Main, SiftDatabase
    out = {}
    cases = {
        "C1": lambda: (synthetic.make_database(1, 500, seed=0),
                       synthetic.make_queries(500, seed=1, db_seed=0, kp_per_image=500,
                                              n_objects=1), 15),
        "C2": lambda: (synthetic.make_database(100, 1000, seed=0),
                       synthetic.make_queries(10000, seed=1, db_seed=0, kp_per_image=1000), 15),
        "C3": lambda: c3_data,
        "IMG1": lambda: (c3_data[0], synthetic.make_queries(500, seed=7, db_seed=0,
                                                            kp_per_image=1000, n_objects=1),
                         c3_data[2]),
    }
    for name in names:
        make = cases[name]
        db, qs, bins = make()
        c = _lib.Context(dev)
        c.set_impl(impl)
        m = Main(c)
        m.set_database(SiftDatabase(db.des, db.kp, db.img, db.centroid, db.size))
        m.get_query_features(qs.des, qs.kp, qs.shape)
        stages = {}

        def staged():
            t = {}
            for k, fn in (("run_matcher", m.run_matcher),
                          ("apply_hough_transform", lambda: m.apply_hough_transform(bins)),
                          ("get_valid_bins", lambda: m.get_valid_bins(5)),
                          ("apply_affine_parameters", lambda: m.apply_affine_parameters(4)),
                          ("post_process", m.post_process)):
                t0 = time.perf_counter()
                fn()
                t[k] = (time.perf_counter() - t0) * 1000.0
            c.synchronize()
            m.valid_bins = []      # main.py builds a new Main per image
            return t
        staged()                   # warm-up (code objects, buffers)
        reps = 3
        for _ in range(reps):
            for k, v in staged().items():
                stages[k] = stages.get(k, 0.0) + v / reps
        # warm (clock ramp, buffers), then the median of 100 runs (20 at C3's ~4 ms)
        nrun = 20 if name == "C3" else 100
        for _ in range(nrun // 2):
            m.run(bins)
        runs = []
        for _ in range(nrun):
            t0 = time.perf_counter()
            m.run(bins)
            runs.append((time.perf_counter() - t0) * 1000.0)
        out[name] = {"queries": len(qs.des), "db_rows": len(db.des), "bins": bins,
                     "stage_ms": stages, "staged_total_ms": sum(stages.values()),
                     "fused_run_ms": float(np.median(runs)), "fused_run_ms_min": float(min(runs)),
                     "fused_run_includes": "enqueue -> matches, valid bins, affine, post-"
                                           "processing and final_pose on the host",
                     "affine_path": m.affine_path, "trig_exact": c.trig_exact(),
                     "final_poses": len(m.final_pose) if m.final_pose is not None else None,
                     "surviving_bins": len(m.valid_bins) if m.valid_bins else None}
        c.close()
    return out


def cpu_sift_baseline(h=800, w=1000):
    """oracle/sift_oracle.c (C, one thread) on the same 1000 x 800 image."""
    from oracle import sift as osift
    img = synthetic.textured_image(h, w, seed=2000)
    t0 = time.perf_counter()
    r = osift.detect_and_compute(img)
    dt = time.perf_counter() - t0
    return {"value": dt * 1000.0, "unit": "ms/image", "cores": 1, "kind": "port",
            "sample": "oracle SIFT detect+describe (C restatement of OpenCV's algorithm, "
                      "1 thread) of one %dx%d image, %d keypoints, %.2f s" % (w, h, len(r["x"]), dt)}


def pmc_traffic(kernel, config):
    """The newest committed PMC summary of the same kernel and workload
    (profiles/*_pmc_<kernel>_<config>.json, from tools/gpu_pmc.sh + tools/pmc_summary.py):
    HBM bytes per launch, MFMA-busy fraction, clock."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_%s_%s.json" % (kernel, config)))):
        best = f
    if not best:
        return None, None
    d = json.load(open(best))
    return d, os.path.relpath(best, REPO)


def _progress(rank, msg):
    # progress on stderr (stdout carries only the JSON line): a long run that prints nothing
    # reads as hung to a supervisor
    print("bench rank %d: %s" % (rank, msg), file=sys.stderr, flush=True)


def main():
    a = parse()
    D = Dist(a.gpus)
    nq, nimg, kpi, bins, run_affine = CONFIGS[a.config]
    world, rank = D.world, D.rank

    # ---- data: rank r holds DB images [r*nimg, (r+1)*nimg) of one seeded DB -------------
    t0 = time.time()
    # keypoints + image table of the WHOLE DB are replicated; descriptors
    # are generated for this rank's shard only
    parts = []
    shard = None
    for r in range(world):
        if r == rank:
            db = synthetic.make_database(nimg, kpi, seed=0, first_image=r * nimg)
            shard = db.des
            parts.append((db.kp, db.img, db.centroid, db.size))
        else:
            parts.append(synthetic.make_database(nimg, kpi, seed=0, first_image=r * nimg,
                                                 descriptors=False))
    x = np.concatenate([p[0].x for p in parts])
    y = np.concatenate([p[0].y for p in parts])
    ang = np.concatenate([p[0].angle for p in parts])
    octv = np.concatenate([p[0].octave for p in parts])
    img = np.concatenate([p[1] + r * nimg for r, p in enumerate(parts)])
    cent = np.concatenate([p[2] for p in parts])
    size = np.concatenate([p[3] for p in parts])
    qs = synthetic.make_queries(nq, seed=1, db_seed=0, kp_per_image=kpi)
    gen_s = time.time() - t0
    _progress(rank, "%s data generated (%.1f s)" % (a.config, gen_s))

    dev = D.local
    if world > 1:
        dev = D.local % max(1, _lib.device_count())   # >1 rank per GPU only with --comm host
    ctx = _lib.Context(dev)
    ctx.set_impl(a.impl)
    kernel, dtype, peak, peak_unit = IMPLS[a.impl]
    from sift_based_od_amd.database import Keypoints
    ctx.set_keypoints(Keypoints(x, y, ang, octv), img, cent, size)
    n_shard = shard.shape[0]
    ctx.upload_db(shard, row_offset=rank * n_shard)
    ctx.upload_queries(qs.des, qs.kp)
    from sift_based_od_amd.sharded import FileHostComm, RcclComm, run_sharded
    # auto: split the chip for the int8 matcher (tail on reserved CUs beside the next image's
    # matcher).  The tail's dependent kernel chain grows with the queries, the matcher with
    # queries x DB rows, so a small DB shard needs more tail CUs: 3 per XCD below 5e5 rows
    # (C2: 0.125 vs 0.134 ms per step at 1 per XCD, 0.168 with two unsplit contexts), else 1
    # (C3 / C5: ~3.8 ms against a ~0.7 ms tail on 8 CUs; one query image: 0.092 vs 0.106 ms
    # with two unsplit contexts).  2 per XCD leaves C2's 240-work-group grid no spare CU
    # (0.21 ms: a second dispatch round).  profiles/r03t_tail_ab.log
    reserve = a.cu_reserve if a.cu_reserve >= 0 else (
        0 if a.contexts > 1 or a.overlap == 0
        or a.impl != "i8" else (3 if shard.shape[0] < 500000 else 1))
    overlap = a.overlap if a.overlap >= 0 else (1 if world > 1 or reserve else 0)
    ctx.set_overlap(bool(overlap))
    if reserve:
        ctx.set_cu_reserve(reserve)
        overlap = 1                 # the split runs the matcher on its own stream
    if a.matcher_streams != 1:
        ctx.set_matcher_streams(a.matcher_streams)
    comm = None
    if world > 1 and a.comm == "rccl":
        # created under the split: sod_comm_init gives the communicator maxCTAs = the
        # reserved CU count (8 * reserve), so every block of an RCCL kernel is resident at once
        comm = RcclComm(ctx, world, rank, D.bcast_bytes)
    elif world > 1:
        comm = FileHostComm(D.store)
    own = (rank * n_shard, (rank + 1) * n_shard)
    ncontexts = a.contexts if a.contexts > 0 else (2 if world == 1 and not overlap else 1)
    ctxs = [ctx]
    for _ in range(ncontexts - 1):
        c = _lib.Context(dev)
        c.set_impl(a.impl)
        c.share_db(ctx)
        c.upload_queries(qs.des, qs.kp)
        ctxs.append(c)
    turn = [0]

    def step():
        c = ctxs[turn[0] % ncontexts]
        turn[0] += 1
        if comm is None or comm.kind == "rccl":
            # one enqueue: match, all-gather, ratio, vote, all-reduce, select, affine
            c.pipeline(qs.shape, bins, ratio=0.75, vote_threshold=5, affine_threshold=4,
                       x_factor=128.0, y_factor=128.0, run_affine=run_affine)
        else:
            run_sharded(c, comm, own, qs.shape, bins, 0.75, 5, 4, 128.0, 128.0, run_affine)

    def sync_all():
        for c in ctxs:
            c.synchronize()

    stride = max(1, a.match_timing_stride)
    for c in ctxs:
        c.set_stage_timing(False)   # stage events are marker packets on the tail's path
    _progress(rank, "DB resident, %d warmup steps" % a.warmup)
    for _ in range(a.warmup):
        step()
    sync_all()
    _progress(rank, "timing %d steps" % a.steps)

    # ---- timed region ----------------------------------------------------------------
    stage = []
    D.barrier()
    sync_all()
    for c in ctxs:
        c.set_match_timing(stride)  # counted from the first timed launch
        c.host_wait_ms(reset=True)
    t0 = time.perf_counter()
    host = 0.0                      # host time spent enqueueing (the calls return unsynced)
    for _ in range(a.steps):
        h0 = time.perf_counter()
        step()
        host += time.perf_counter() - h0
    sync_all()
    D.barrier()
    t1 = time.perf_counter()
    el = D.max(t1 - t0)
    ms_per_step = 1000.0 * el / a.steps
    # the enqueue calls' host time split: blocked on the device (slot wait) vs host work
    blocked_ms = sum(c.host_wait_ms(reset=True) for c in ctxs)

    # ---- matcher kernel time inside the timed region: begin/end HIP events recorded around
    # every launch on the matcher's own stream (sod_match_times), read back afterwards ----
    live = []
    for k, c in enumerate(ctxs):
        n_k = len(range(k, a.steps, ncontexts))      # timed launches of context k
        n_rec = len(range(0, n_k, stride))           # ... that recorded events
        if n_rec:
            live.extend(c.match_times(min(n_rec, 64)).tolist())
        c.set_match_timing(True)
    match_ms = float(np.mean(live))

    # ---- per-stage timing (HIP events on the ctx stream), separate untimed steps --------
    match_iso = []
    ctx.set_stage_timing(True)
    for _ in range(max(3, min(a.steps, 10))):
        turn[0] = 0            # always the first context (its events are read below)
        step()
        ctx.synchronize()
        match_iso.append(ctx.last_match_ms())
        stage.append(ctx.stage_ms())
    match_iso = float(np.mean(match_iso))
    stage = np.mean(np.array(stage), axis=0)
    stage_full = None
    if reserve:
        ctx.set_cu_reserve(0)      # post-processing and extras below on the whole chip
        # warm the whole-chip configuration as the timed run was warmed: after the idle gaps
        # of the isolated steps the matcher's clock ramps again (rocprofv3, r03zh: whole-chip
        # C3 launches 4.52, 4.35, 4.21 ... 3.78 ms over the first ten)
        for _ in range(a.warmup):
            turn[0] = 0
            step()
        ctx.synchronize()
        # the same stages on the whole chip (the timed run keeps them on the reserved CUs,
        # beside the next query's matcher)
        full = []
        for _ in range(5):
            turn[0] = 0
            step()
            ctx.synchronize()
            full.append(ctx.stage_ms())
        stage_full = np.mean(np.array(full), axis=0)
    # one step alone on the device: host clock from the enqueue to the device sync after the
    # last stage, tail on the whole chip (the timed steps above overlap each image's tail with
    # the next image's matcher).  Device-only: no result is read back and post-processing is
    # not in it -- main.py's per-image wall time is extras.main_path.*.fused_run_ms
    # (no timing events on the matcher launch either: with the split undone and the streams
    # idle the matcher runs on the context stream, where an event on its dispatch would delay
    # the merge ~5 us)
    _progress(rank, "stage timing and latency")
    lat = []
    ctx.set_stage_timing(False)
    ctx.set_match_timing(False)
    for _ in range(max(5, min(a.steps, 20))):
        turn[0] = 0
        ctx.synchronize()
        t0 = time.perf_counter()
        step()
        ctx.synchronize()
        lat.append((time.perf_counter() - t0) * 1000.0)
    ctx.set_match_timing(True)
    ctx.set_stage_timing(True)
    latency_ms = float(np.median(lat))

    # post-processing (main.py:159-168) over the surviving bins: timed
    # separately (it ends in a host DFS, so it is not inside the stream-ordered step)
    post_ms = None
    post = None
    if run_affine:
        post = ctx.postprocess()          # first call loads the kernel's code object
        # each timed call follows a fresh step (a second read of unchanged results would
        # reuse the staging its predecessor left: not the per-image cost)
        pt = []
        for _ in range(5):
            turn[0] = 0
            step()
            ctx.synchronize()
            t0 = time.perf_counter()
            post = ctx.postprocess()
            pt.append(time.perf_counter() - t0)
        post_ms = 1000.0 * float(np.mean(pt))
    V, M = ctx.valid_counts()
    keys, votes = ctx.all_bins()
    n_votes = int(votes.sum())
    aff = ctx.affine_result() if run_affine else None
    idx1, d1, d2, good = ctx.match_result()
    # self-verifying multi-rank record: the communicator as RCCL reports
    # it on every rank, and how many of the merged global winners (good matches) each shard
    # contributed -- every rank holds the same merged result, so each counts all shards and
    # its own count must agree with the others'
    cinfo = comm.info() if comm is not None else None
    real = (idx1 >= 0) & (idx1 < world * n_shard)       # (a DB row, not a sentinel)
    winners = np.bincount((idx1[real] // n_shard).astype(np.int64), minlength=world).tolist()
    good_winners = np.bincount((idx1[real & good] // n_shard).astype(np.int64),
                               minlength=world).tolist()
    rank_rec = D.gather_json({"rank": rank, "comm": cinfo, "shard_winners": winners,
                              "own_shard_winners": winners[rank],
                              "shard_good_winners": good_winners})

    # Hough stage roofline: algorithmic bytes 52 per good match (query kp 16 +
    # model kp 16 + idx 4 + centroid 16) + 4 per bin (the count written out) over the
    # device time of pose_kernel + hist_kernel (stage events)
    n_good = int(good.sum())
    nbins = int(np.prod(bins))
    hough_bytes = 52 * n_good + 4 * nbins
    t_hough = float(stage[2])
    t_hough_full = float(stage_full[2]) if stage_full is not None else t_hough
    roofline_hough = {
        "bound": "hbm", "achieved": hough_bytes / (t_hough * 1e-3) / 1e9, "peak": 8000.0,
        "unit": "GB/s", "frac": hough_bytes / (t_hough * 1e-3) / 1e9 / 8000.0, "traffic": None,
        "algorithmic_bytes": hough_bytes, "kernels": "pose_kernel + hist_kernel",
        "stage_ms": t_hough,
        "cus": 8 * reserve if reserve else "all",
        "whole_chip": {"stage_ms": t_hough_full,
                       "achieved": hough_bytes / (t_hough_full * 1e-3) / 1e9,
                       "frac": hough_bytes / (t_hough_full * 1e-3) / 1e9 / 8000.0},
        "note": "latency-bound, not bandwidth-bound: %d good matches and %d bins move %.1f MB; "
                "the two launches (their fixed cost and one pass of dependent loads / LDS "
                "atomics per work-group) set the time%s" % (
                    n_good, nbins, hough_bytes / 1e6,
                    ", here on the %d CUs the CU split reserves for the tail" % (8 * reserve)
                    if reserve else "")}
    pmc, traffic_src = pmc_traffic(kernel, a.config)
    traffic = pmc.get("hbm_bytes") if pmc else None
    pairs = float(world) * nq * n_shard
    value = pairs / (ms_per_step / 1000.0)
    achieved = OPS_PER_PAIR * nq * n_shard / (match_ms / 1000.0) / 1e12
    # compulsory HBM bytes of one matcher launch: packed DB rows + their norm words, packed
    # queries + norms, merged (d1^2, idx, d2^2) per query
    row_b, norm_b = (128, 8) if dtype == "i8" else (256, 4)
    alg_bytes = n_shard * (row_b + norm_b) + nq * (row_b + 4) + 12 * nq
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "host_enqueue_ms_per_step": 1000.0 * host / a.steps,
        # of which blocked waiting for the device (a launch waits for the merge that last read
        # its partial-result slot: two steps in flight) / the host's own work
        "host_blocked_ms_per_step": blocked_ms / a.steps,
        "host_cpu_enqueue_ms_per_step": (1000.0 * host - blocked_ms) / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (seeded SIFT-like uint8 descriptors, SURVEY.md §8(d))",
        "config": {"workload": "%s: %d query x %d DB/GPU (total %d) + Hough %s%s" % (
            a.config.upper(), nq, n_shard, world * n_shard, "x".join(map(str, bins)),
            " + affine verify" if run_affine else ""),
            "queries": nq, "db_rows_per_gpu": n_shard, "db_rows_total": world * n_shard,
            "bins": list(bins), "parallelism": "db-shard%d" % world,
            "query_streams": ncontexts, "matcher_overlap": bool(overlap),
            "cu_reserve_per_xcd": reserve, "matcher_streams": a.matcher_streams,
            "comm": a.comm if world > 1 else None,
            "rccl_nranks": cinfo["nranks"] if cinfo and cinfo["kind"] == "rccl" else None,
            "rccl_rank": cinfo["rank"] if cinfo and cinfo["kind"] == "rccl" else None},
        "ranks": rank_rec,
        # per shard: queries whose merged nearest row (trainIdx) it holds / of those, good
        "shard_winners": winners,
        "shard_good_winners": good_winners,
        "hough_votes_per_s": n_votes / (ms_per_step / 1000.0),
        "hough_stage_votes_per_s": n_votes / (t_hough / 1000.0),
        "hough_votes": n_votes,
        "good_matches": int(good.sum()),
        "valid_bins": V,
        "surviving_bins": int(aff["survived"].sum()) if aff else None,
        # device time of each stage's own launches (sod_last_stage_ms: per rank, host waits
        # between the calls excluded), isolated steps after the timed region
        "stage_ms": dict({"match_kernel": match_ms, "match_kernel_isolated": match_iso},
                         **{k: float(v) for k, v in zip(_lib.Context.STAGES[1:], stage[1:])},
                         post_process=post_ms),
        "single_step_device_latency_ms": latency_ms,
        "stage_ms_whole_chip": ({k: float(v) for k, v in zip(_lib.Context.STAGES, stage_full)}
                                if stage_full is not None else None),
        "roofline_hough": roofline_hough,
        "final_poses": int(len(post["final_pose"])) if post is not None else None,
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak,
                     "unit": peak_unit, "frac": achieved / peak, "traffic": traffic,
                     "traffic_unit": "bytes/launch (HBM, 2*FETCH_SIZE+WRITE_SIZE)",
                     "traffic_source": traffic_src,
                     # rocprof counters against the gfx950 peaks (north_star): bytes past
                     # L2 per launch over this run's launch time vs ~8 TB/s HBM; MFMA-busy
                     # SIMD cycles / all SIMD cycles and the clock of the PMC passes
                     "traffic_gb_per_s": traffic / (match_ms * 1e6) if traffic else None,
                     "traffic_frac_of_hbm_peak": traffic / (match_ms * 1e6) / 8000.0 if traffic else None,
                     "mfma_busy_frac_pmc": pmc.get("mfma_busy_frac") if pmc else None,
                     # the profiled dispatches' own clock (GRBM_GUI_ACTIVE / 8 over their
                     # own duration): how far below the 2.4 GHz of the quoted peak the chip
                     # ran under the counters; no fraction is derived from it
                     "clock_ghz_pmc_profiled": pmc.get("clock_ghz_profiled") if pmc else None,
                     "algorithmic_bytes": alg_bytes,
                     "kernel": kernel,
                     "algorithmic": "256 op/pair x %d x %d pairs per launch" % (nq, n_shard),
                     "timed_launches": "HIP begin/end events on one matcher launch in %d of "
                                       "the timed region" % stride},
        "matcher_impl": a.impl,
        "exact_order": ctx.exact_order(),
        "datagen_s": gen_s,
    }
    if world == 1 and not a.no_extras:
        # on a context of their own (sharing the resident DB): ctx keeps the timed run's
        # results for the CPU baselines below
        ec = ctxs[-1]
        if ec is ctx:
            ec = _lib.Context(dev)
            ec.set_impl(a.impl)
            ec.share_db(ctx)
        _progress(rank, "extras")
        out["extras"] = extras(ec, ctx, shard, bins)
        if a.config in ("c3", "c5", "img1"):
            from sift_based_od_amd import SiftDatabase
            _progress(rank, "main.py path")
            c3db = SiftDatabase(shard, Keypoints(x, y, ang, octv), img, cent, size)
            out["extras"]["main_path"] = main_path_extras(
                dev, a.impl, (c3db, qs, bins), ("C1", "C2", "C3", "IMG1") if a.config != "img1"
                else ("IMG1",))
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        _progress(rank, "cpu baseline")
        out["cpu_baseline"] = cpu_baseline(qs.des, shard, a.cpu_queries)
        out["cpu_baseline_hough"] = cpu_hough_baseline(qs, (x, y, ang, octv), img, cent, size,
                                                       idx1, good, bins)
        if post is not None:
            out["cpu_baseline_post"] = cpu_post_baseline(ctx, post)
        if not a.no_extras:
            out["cpu_baseline_sift"] = cpu_sift_baseline()
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    for c in ctxs[1:]:
        c.close()
    ctx.close()
    D.close()


if __name__ == "__main__":
    main()
