"""GPU parity: the HIP path (through the C ABI) against the reference's golden vectors
and the oracle.  Bit-exact for matches, bin indices, bin counts, first-touch order and
member lists; PoseBin means within 1e-12 relative (device cos/sin may differ from glibc
by an ulp); affine parameters within 1e-4 (north_star tolerance)."""
import numpy as np
import pytest

from conftest import golden
from helpers import kp
from oracle import oracle as orc
from sift_based_od_amd import _lib, synthetic

pytestmark = pytest.mark.gpu

CASES = ["c1_b15", "planted_b15", "planted_b12"]
AFFINE_ATOL = 1e-4
IMPLS = ["bf16", "i8", "i8w"]


def load_case(ctx, g):
    ctx.set_keypoints(kp(g, "db_"), g["db_img"], g["centroid"], g["size"])
    ctx.upload_db(g["db_des"])
    ctx.upload_queries(g["q_des"], kp(g, "q_"))


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("name", CASES)
def test_matcher_golden(ctx, name, impl):
    g = golden(name)
    ctx.set_impl(impl)
    load_case(ctx, g)
    ctx.match()
    ctx.ratio(0.75)
    idx1, d1, d2, good = ctx.match_result()
    assert np.array_equal(idx1, g["idx1"])
    assert np.array_equal(d1.view(np.uint32), g["d1"].view(np.uint32))
    assert np.array_equal(d2.view(np.uint32), g["d2"].view(np.uint32))
    assert np.array_equal(good, g["good"])
    assert ctx.exact_order()
    ctx.set_impl("bf16")


@pytest.mark.parametrize("impl", IMPLS)
def test_matcher_edges(ctx, impl):
    g = golden("matcher_edges")
    ctx.set_impl(impl)
    ctx.upload_db(g["db_des"])
    ctx.upload_queries(g["q_des"])
    ctx.match()
    ctx.ratio(0.75)
    idx1, d1, d2, good = ctx.match_result()
    assert np.array_equal(idx1, g["idx1"])   # ties -> lowest trainIdx
    assert np.array_equal(d1, g["d1"]) and np.array_equal(d2, g["d2"])
    assert np.array_equal(good, g["good"])


@pytest.mark.parametrize("nq,ndb,seed", [(1, 2, 0), (17, 1000, 1), (500, 1000, 4), (700, 4099, 2),
                                         (513, 77777, 5), (3000, 60000, 3), (500, 400000, 6)])
def test_matcher_shapes_vs_oracle(ctx, nq, ndb, seed):
    """The ring matcher bit for bit against the oracle on edge shapes (the cases written for
    round 5's register-streamed kernel, removed in round 6): one query, partial query tiles
    (17, 513), DB chunks of a few subtiles (1 000 rows), exact duplicates of DB rows (d1 = 0)
    and DB rows repeated in far chunks (cross-chunk ties: the lowest trainIdx wins), two
    launches on the same slots, and the matcher_edges golden."""
    rng = np.random.default_rng(seed)
    db = synthetic.sift_like_descriptors(rng, ndb)
    q = synthetic.sift_like_descriptors(rng, nq)
    if ndb > 8 and nq > 8:
        k = min(nq // 3, ndb // 2)
        q[:k] = db[rng.integers(0, ndb, k)]
        h = ndb // 2
        n = min(200, h)
        db[h:h + n] = db[:n]                       # the same rows in two far ranges
        q[k:k + min(n, nq - k)] = db[:min(n, nq - k)]
    ctx.set_impl("i8")
    ctx.upload_db(db)
    ctx.upload_queries(q)
    for _ in range(2):        # the second launch reuses the reset threshold slots
        ctx.match()
    ctx.ratio(0.75)
    idx1, d1, d2, good = ctx.match_result()
    e1, f1, f2 = orc.knn2_match(q, db)
    assert np.array_equal(idx1, e1)
    assert np.array_equal(d1, f1) and np.array_equal(d2, f2)
    assert np.array_equal(good, orc.ratio_test(f1, f2))
    if seed == 0:
        g = golden("matcher_edges")
        ctx.upload_db(g["db_des"])
        ctx.upload_queries(g["q_des"])
        ctx.match()
        ctx.ratio(0.75)
        idx1, d1, d2, good = ctx.match_result()
        assert np.array_equal(idx1, g["idx1"])
        assert np.array_equal(d1, g["d1"]) and np.array_equal(d2, g["d2"])
        assert np.array_equal(good, g["good"])


@pytest.mark.parametrize("shape", ["pair4", "pair8", "pf2", "w1"])
@pytest.mark.parametrize("nq,ndb,seed", [(1, 2, 0), (17, 1000, 1), (700, 4099, 2), (3000, 60000, 3)])
def test_matcher_vs_oracle_options(ctx, nq, ndb, seed, shape):
    """The matcher shapes behind options, bit for bit against the oracle on odd sizes: paired
    waves at 4 / 8 query tiles (match_pair = 2: partial top-2 lists of the two subtile phases
    merged through LDS), two-ahead LDS prefetch (match_pf = 2, counted asm waits at 2 tiles),
    and the 32x32x32 kernel at one 32-query tile per wave."""
    rng = np.random.default_rng(seed)
    if shape == "w1":
        ctx.set_impl("i8w")
        ctx.set_option("match_qt", 1)
    else:
        ctx.set_impl("i8")
        ctx.set_option("match_qt", {"pair4": 4, "pair8": 8, "pf2": 2}[shape])
        ctx.set_option("match_pair", 2 if shape.startswith("pair") else 1)
        ctx.set_option("match_pf", 2 if shape == "pf2" else 1)
    db = synthetic.sift_like_descriptors(rng, ndb)
    q = synthetic.sift_like_descriptors(rng, nq)
    q[: nq // 3] = db[rng.integers(0, ndb, nq // 3)]      # exact hits (d1 = 0)
    if ndb >= 64:
        db[16:20] = db[0:4]                               # equal rows in neighbouring subtiles
        q[nq // 3: nq // 3 + min(4, nq - nq // 3)] = db[0:min(4, nq - nq // 3)]
    ctx.upload_db(db)
    ctx.upload_queries(q)
    ctx.match()
    ctx.ratio(0.75)
    idx1, d1, d2, good = ctx.match_result()
    e1, f1, f2 = orc.knn2_match(q, db)
    assert np.array_equal(idx1, e1)
    assert np.array_equal(d1, f1) and np.array_equal(d2, f2)
    assert np.array_equal(good, orc.ratio_test(f1, f2))


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("nq,ndb,seed", [(1, 2, 0), (17, 1000, 1), (700, 4099, 2), (3000, 60000, 3)])
def test_matcher_vs_oracle(ctx, nq, ndb, seed, impl):
    rng = np.random.default_rng(seed)
    ctx.set_impl(impl)
    db = synthetic.sift_like_descriptors(rng, ndb)
    q = synthetic.sift_like_descriptors(rng, nq)
    q[: nq // 3] = db[rng.integers(0, ndb, nq // 3)]      # exact hits (d1 = 0)
    ctx.upload_db(db)
    ctx.upload_queries(q)
    ctx.match()
    ctx.ratio(0.75)
    idx1, d1, d2, good = ctx.match_result()
    e1, f1, f2 = orc.knn2_match(q, db)
    assert np.array_equal(idx1, e1)
    assert np.array_equal(d1, f1) and np.array_equal(d2, f2)
    assert np.array_equal(good, orc.ratio_test(f1, f2))


@pytest.mark.parametrize("qt", ["2", "2f", "4", "8", "4p", "8p", "w1", "w2"])
def test_matcher_query_tiles_shared_thresholds(ctx, qt):
    """int8 matcher with each query-tile count per wave (option match_qt; "4p" / "8p": paired
    waves, option match_pair = 2, each wave of a pair taking every other subtile; "2f": 2 tiles
    with the LDS fragments read two subtiles ahead (option match_pf = 2: the inline-asm reads'
    counted waits then leave the next subtile's reads in flight); "w1" / "w2":
    the 32x32x32 kernel, impl i8w, at 1 / 2 tiles of 32 queries per wave) over a DB split into
    many chunks, so the chunks exchange prefilter thresholds mid-run: DB rows duplicated far
    apart (other chunks) make exact distance ties ACROSS chunks -- a shared threshold must
    keep them (lowest trainIdx wins), and queries equal to a DB row (d1 = 0) or near one,
    including runs of equal rows inside a chunk's seed stage."""
    ctx.set_option("match_qt", int(qt.strip("pwf")))
    ctx.set_option("match_pair", 2 if qt.endswith("p") else 1)
    ctx.set_option("match_pf", 2 if qt.endswith("f") else 1)
    rng = np.random.default_rng(31)
    ndb, nq = 150000, 2000
    db = synthetic.sift_like_descriptors(rng, ndb)
    db[100000:100600] = db[0:600]                      # ties across chunks
    db[140000:140300] = db[50000:50300]
    q = synthetic.sift_like_descriptors(rng, nq)
    q[:600] = np.clip(db[:600].astype(int) + rng.integers(-2, 3, (600, 128)), 0, 255)
    q[600:900] = db[50000:50300]                       # d1 = d2 = 0, two equal rows
    # equal rows inside a chunk's first stage (where the seed pass takes its bound) and
    # mid-DB: the seed equals both winners' value, which must still pass (>=)
    db[1:8] = db[0]
    db[75001:75005] = db[75000]
    # equal rows in neighbouring subtiles (the two waves of a pair: even / odd subtiles), the
    # later copy first in its own subtile
    db[16] = db[0]
    db[75017] = db[75000]
    db[75035] = db[75000]
    q[900:950] = db[0]
    q[950:1000] = db[75000]
    # duplicates spread over chunks of both parities (the best-row slots: the even-chunk and
    # odd-chunk bests are then EQUAL, so the bound equals both winners' value)
    for a, b in ((25000, 130000), (33000, 91000), (47000, 118000), (61000, 62000)):
        db[b:b + 100] = db[a:a + 100]
    q[1000:1100] = db[25000:25100]
    q[1100:1200] = db[33000:33100]
    q[1200:1300] = np.clip(db[47000:47100].astype(int) + rng.integers(-1, 2, (100, 128)), 0, 255)
    q[1300:1400] = db[61000:61100]
    ctx.set_impl("i8w" if qt.startswith("w") else "i8")
    ctx.upload_db(db)
    ctx.upload_queries(q)
    for _ in range(2):        # the second launch reuses the reset threshold slot
        ctx.match()
    ctx.ratio(0.75)
    idx1, d1, d2, good = ctx.match_result()
    e1, f1, f2 = orc.knn2_match(q, db)
    assert np.array_equal(idx1, e1)
    assert np.array_equal(d1, f1) and np.array_equal(d2, f2)
    assert np.array_equal(good, orc.ratio_test(f1, f2))


def _bf(impl):
    from sift_based_od_amd.matcher import BFMatcher
    c = _lib.Context(0)
    c.set_impl(impl)
    return BFMatcher(ctx=c)


@pytest.mark.parametrize("impl", ["i8", "bf16"])
@pytest.mark.parametrize("case", ["edges", "dups"])
def test_knnmatch_second_train_idx(case, impl):
    """BFMatcher.knnMatch returns OpenCV's full pair: n.trainIdx = the lowest trainIdx other
    than m's at the second-best distance (sod_match_knn_indices), against the oracle; exact
    duplicate rows make the ties (inside one DB split and across splits)."""
    from sift_based_od_amd.matcher import BFMatcher
    if case == "edges":
        g = golden("matcher_edges")
        q, db = g["q_des"], g["db_des"]
    else:
        rng = np.random.default_rng(17)
        db = synthetic.sift_like_descriptors(rng, 70000)
        db[60000:60500] = db[100:600]              # twins far apart (other DB splits)
        db[30000:30100] = db[100:200]              # triplets
        db[101] = db[100]                          # twins next to each other
        q = synthetic.sift_like_descriptors(rng, 1500)
        q[:500] = db[100:600]                      # d1 == d2 == 0
        q[500:1000] = np.clip(db[100:600].astype(int) + rng.integers(-2, 3, (500, 128)), 0, 255)
    bf = _bf(impl)
    res = bf.knnMatch(q.astype(np.float32), db.astype(np.float32), k=2)
    i1, e1, e2, i2 = orc.knn2_match(q, db, with_idx2=True)
    assert [m.trainIdx for m, _ in res] == i1.tolist()
    assert [n.trainIdx for _, n in res] == i2.tolist()
    assert np.array_equal(np.array([m.distance for m, _ in res], np.float32), e1)
    assert np.array_equal(np.array([n.distance for _, n in res], np.float32), e2)
    assert all(m.queryIdx == i and n.queryIdx == i for i, (m, n) in enumerate(res))


def _float_tie_case(seed=23, nq=96, ndb=3000):
    """Descriptors far apart (distances 2200-2900, beyond 2048): for every query a pair of
    DB rows whose squared distances differ by 1 but share one float sqrtf -- OpenCV then
    sees a tie and keeps the LOWER trainIdx, while the exact squared order prefers the
    other row when it comes later."""
    rng = np.random.default_rng(seed)
    q = rng.integers(250, 256, (nq, 128)).astype(np.int64)
    db = rng.integers(0, 6, (ndb, 128)).astype(np.int64)           # far: ~2860
    placed = 0
    for k in range(nq):
        for _ in range(200):
            a = np.clip(q[k] - rng.integers(185, 230, 128), 0, 255)
            a[0] = q[k][0] - 1                                        # B: d0 = q0 -> sq - 1
            b = a.copy()
            b[0] = q[k][0]
            sa, sb = int(((q[k] - a) ** 2).sum()), int(((q[k] - b) ** 2).sum())
            if np.sqrt(np.float32(sa), dtype=np.float32) == np.sqrt(np.float32(sb), dtype=np.float32):
                i, j = rng.choice(ndb, 2, replace=False)
                db[i], db[j] = (a, b) if k % 2 else (b, a)          # the closer one first or last
                placed += 1
                break
    assert placed > nq // 2
    return q.astype(np.uint8), db.astype(np.uint8)


@pytest.mark.parametrize("impl", ["i8", "bf16"])
def test_knnmatch_float_distance_ties(impl):
    """Inputs beyond SIFT's range (distances >= 2048, exact_order False): knnMatch's indices
    follow OpenCV's float-distance order -- equal float distances keep the lower trainIdx --
    for m and n, against the oracle (float32 sqrt order) and the int64 brute force."""
    q, db = _float_tie_case()
    bf = _bf(impl)
    res = bf.knnMatch(q.astype(np.float32), db.astype(np.float32), k=2)
    assert not bf._context().exact_order()
    i1, e1, e2, i2 = orc.knn2_match(q, db, with_idx2=True)
    j1, f1, f2, j2 = orc.knn2_match_int(q, db, with_idx2=True)
    assert np.array_equal(i1, j1) and np.array_equal(i2, j2)
    assert [m.trainIdx for m, _ in res] == i1.tolist()
    assert [n.trainIdx for _, n in res] == i2.tolist()
    assert np.array_equal(np.array([m.distance for m, _ in res], np.float32), e1)
    assert np.array_equal(np.array([n.distance for _, n in res], np.float32), e2)
    # the float order mattered: the matcher's exact squared order picks other rows here
    raw = bf._context().match_result()[0]
    assert (raw != i1).sum() > 0


def test_knnmatch_resident_train_set():
    """The train set stays on the device: a read-only train array passed again, or OpenCV's
    add() / train() collection, is not uploaded a second time; a writeable array is (it may
    have changed in place).  Results equal the oracle on every call; the collection's
    DMatch carries (imgIdx, trainIdx within the set) as OpenCV's does."""
    rng = np.random.default_rng(41)
    db = synthetic.sift_like_descriptors(rng, 20000)
    q = synthetic.sift_like_descriptors(rng, 700)
    q[:200] = db[rng.integers(0, 20000, 200)]
    i1, e1, e2, i2 = orc.knn2_match(q, db, with_idx2=True)
    bf = _bf("i8")
    ro = db.copy()
    ro.flags.writeable = False
    for call in range(2):
        res = bf.knnMatch(q, ro, k=2)
        assert bf.uploads == 1
        assert [m.trainIdx for m, _ in res] == i1.tolist()
        assert [n.trainIdx for _, n in res] == i2.tolist()
    # the context's DB replaced by another user between calls: uploaded again
    bf._context().upload_db(db[:100])
    res = bf.knnMatch(q, ro, k=2)
    assert bf.uploads == 2
    assert [m.trainIdx for m, _ in res] == i1.tolist()
    # a read-only view of a writeable base is not trusted (it changes through the base)
    base = db.copy()
    view = base[:]
    view.flags.writeable = False
    bf.knnMatch(q, view, k=2)
    base[i1[1]] = 255 - base[i1[1]]
    res = bf.knnMatch(q, view, k=2)
    assert bf.uploads == 4
    k1, _, _ = orc.knn2_match(q, base)
    assert [m.trainIdx for m, _ in res] == k1.tolist()
    wr = db.copy()
    bf.knnMatch(q, wr, k=2)
    wr[i1[0]] = 255 - wr[i1[0]]          # in-place change between calls: must be seen
    res = bf.knnMatch(q, wr, k=2)
    assert bf.uploads == 6
    j1, _, _ = orc.knn2_match(q, wr)
    assert [m.trainIdx for m, _ in res] == j1.tolist()
    # OpenCV's collection: two sets, rows numbered within their set, imgIdx = the set
    bf2 = _bf("i8")
    bf2.add([db[:8000], db[8000:]])
    bf2.train()
    for call in range(2):
        res = bf2.knnMatch(q, k=2)
        assert bf2.uploads == 1
        got = [m.imgIdx * 8000 + m.trainIdx for m, _ in res]
        assert got == i1.tolist()
        assert [n.imgIdx * 8000 + n.trainIdx for _, n in res] == i2.tolist()
        assert np.array_equal(np.array([m.distance for m, _ in res], np.float32), e1)


def test_main_float_order_beyond_sift():
    """Main.run_matcher (main.py:70-86) on uint8 rows whose distances exceed 2048 (norm >
    1024, not SIFT): OpenCV orders knnMatch by the float distance, so m.trainIdx -- and the
    model keypoint of every matching_keypoints tuple -- is the lowest row at the float d1,
    as orc.knn2_match computes it; the fused Main.run then votes with the same indices."""
    from sift_based_od_amd import SiftDatabase
    from sift_based_od_amd.database import Keypoints
    from sift_based_od_amd.pipeline import Main
    q, db = _float_tie_case(seed=29, nq=128, ndb=4000)
    rng = np.random.default_rng(5)
    n = len(db)
    dkp = Keypoints(rng.uniform(0, 1500, n), rng.uniform(0, 1000, n), rng.uniform(0, 360, n),
                    rng.integers(0, 3, n) | (1 << 8), rng.uniform(1, 9, n), rng.uniform(0, 1, n),
                    rng.integers(0, 5, n))
    img = (np.arange(n) * 4 // n).astype(np.int32)
    cen = rng.uniform(200, 900, (4, 2))
    size = np.tile(np.array([[1500, 1000]], np.int32), (4, 1))
    qkp = Keypoints(rng.uniform(0, 1000, len(q)), rng.uniform(0, 800, len(q)),
                    rng.uniform(0, 360, len(q)), rng.integers(0, 3, len(q)))
    with _lib.Context(0) as c:
        m = Main(c)
        m.set_database(SiftDatabase(db, dkp, img, cen, size))
        m.get_query_features(q, qkp, (800, 1000, 3))
        assert not c.exact_order()
        m.run_matcher()
        i1, e1, e2 = orc.knn2_match(q, db)
        good = orc.ratio_test(e1, e2)
        raw = c.match_result()[0]
        assert np.array_equal(raw, i1)         # the device's trainIdx is OpenCV's
        mk = m.matching_keypoints
        assert len(mk) == int(good.sum())
        for (kM, kQ, sz, ce), qi in zip(mk, np.nonzero(good)[0]):
            t = int(i1[qi])
            assert kM.pt == (float(dkp.x[t]), float(dkp.y[t])) and kM.size == float(dkp.size[t])
            assert kM.class_id == int(dkp.class_id[t])
        out = m.run(post_process=False)
        assert np.array_equal(out["idx1"], i1)


@pytest.mark.parametrize("impl", IMPLS)
def test_matcher_f32_input_and_validation(ctx, impl):
    rng = np.random.default_rng(11)
    ctx.set_impl(impl)
    db = rng.integers(0, 256, (500, 128)).astype(np.uint8)
    q = rng.integers(0, 256, (100, 128)).astype(np.uint8)
    ctx.upload_db(db.astype(np.float32))
    ctx.upload_queries(q.astype(np.float32))
    ctx.match()
    ctx.ratio(0.75)
    idx1, d1, d2, _ = ctx.match_result()
    e1, f1, f2 = orc.knn2_match_int(q, db)
    assert np.array_equal(idx1, e1) and np.array_equal(d1, f1) and np.array_equal(d2, f2)
    bad = db.astype(np.float32)
    bad[3, 7] = 0.5
    with pytest.raises(_lib.SodError):
        ctx.upload_db(bad)


def test_pose_sweep(ctx):
    g = golden("pose_sweep")
    shape = tuple(int(v) for v in g["shape"])
    for j, b in enumerate(g["bins"]):
        pose, idx = ctx.pose_batch(g["mx"], g["my"], g["ma"], g["mo"], g["qx"], g["qy"], g["qa"],
                                   g["qo"], g["cx"], g["cy"], shape, int(b))
        assert np.array_equal(idx, g["idx"][j]), "bins=%d: %d index mismatches" % (
            b, int((idx != g["idx"][j]).any(1).sum()))
        if ctx.trig_exact():   # the device's cos / sin are the host libm's: all bit-exact
            assert np.array_equal(pose.view(np.uint64), g["poses"].view(np.uint64))
        np.testing.assert_allclose(pose, g["poses"], rtol=1e-13, atol=1e-10)
        # alpha and scale use no transcendental: bit-exact
        assert np.array_equal(pose[:, 2:], g["poses"][:, 2:])


def test_pose_near_edge_guard(ctx, trig):
    """Poses within a few ulps of an x AND a y bin edge (make_golden.near_edge_sweep):
    indices AND x, y equal the reference's bit for bit.  With the device's glibc cos / sin
    (sod_trig_exact, round 5) no guard is armed and nothing is listed; on a host whose libm
    differs the boundary guard lists every one and redoes x, y with that libm."""
    g = golden("near_edge_sweep")
    shape = tuple(int(v) for v in g["shape"])
    for b in g["bins"]:
        f = {k: g["b%d_%s" % (b, k)] for k in ("mx", "my", "ma", "mo", "qx", "qy", "qa", "qo",
                                                "cx", "cy", "poses", "idx")}
        pose, idx = ctx.pose_batch(f["mx"], f["my"], f["ma"], f["mo"], f["qx"], f["qy"], f["qa"],
                                   f["qo"], f["cx"], f["cy"], shape, int(b))
        flagged, changed, _, _ = ctx.guard_stats()
        assert flagged == (0 if ctx.trig_exact() else len(f["mx"]))
        assert np.array_equal(idx, f["idx"])
        assert np.array_equal(pose.view(np.uint64), f["poses"].view(np.uint64))
        print("bins %d: %d listed, %d bins changed by the guard" % (b, flagged, changed))


def _check_hough(ctx, g):
    keys, votes = ctx.all_bins()
    assert np.array_equal(keys, g["table_keys"]), "bin table (first-touch order) differs"
    assert np.array_equal(votes, g["table_votes"])
    v = ctx.valid_result()
    assert np.array_equal(v["keys"], g["valid_keys"])
    assert np.array_equal(v["votes"], g["valid_votes"])
    assert np.array_equal(v["offsets"], g["valid_off"])
    assert np.array_equal(v["members"], g["valid_members"])
    if ctx.trig_exact():   # device glibc cos / sin: the PoseBin means are main.py's exactly
        assert np.array_equal(v["means"].view(np.uint64),
                              np.asarray(g["valid_means"], np.float64).view(np.uint64))
    np.testing.assert_allclose(v["means"], g["valid_means"], rtol=1e-12, atol=1e-9)
    a = ctx.affine_result()
    surv = np.nonzero(a["survived"])[0]
    assert np.array_equal(surv, g["surv_index"]), "surviving bins differ"
    assert np.array_equal(a["votes"][surv], g["surv_votes"])
    np.testing.assert_allclose(a["params"][surv], g["surv_params"], rtol=0, atol=AFFINE_ATOL)
    for k, i in enumerate(surv):
        lo, hi = v["offsets"][i], v["offsets"][i + 1]
        kept = v["members"][lo:hi][a["alive"][lo:hi]]
        assert np.array_equal(kept, g["surv_members"][g["surv_off"][k]:g["surv_off"][k + 1]])


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("name", CASES)
def test_pipeline_golden(ctx, name, impl):
    g = golden(name)
    ctx.set_impl(impl)
    load_case(ctx, g)
    shape = tuple(int(v) for v in g["shape"])
    ctx.pipeline(shape, int(g["bins"]), ratio=0.75, vote_threshold=5, affine_threshold=4)
    idx1, d1, d2, good = ctx.match_result()
    assert np.array_equal(idx1[good], g["idx1"][g["good"]])
    _check_hough(ctx, g)


@pytest.mark.parametrize("name", ["edge_b15", "edge_b6", "near_edge_b15", "near_edge_b32"])
def test_hough_affine_edges(ctx, name, trig):
    g = golden(name)
    ctx.set_keypoints(kp(g, "db_"), g["db_img"], g["centroid"], g["size"])
    ctx.upload_queries(None, kp(g, "q_"))
    idx1 = np.zeros(len(g["q_x"]), np.int32)
    idx1[g["match_q"]] = g["match_m"]
    good = np.zeros(len(g["q_x"]), bool)
    good[g["match_q"]] = True
    ctx.set_matches(idx1, good)
    shape = tuple(int(v) for v in g["shape"])
    ctx.hough(shape, int(g["bins"]))
    ctx.select(5)
    ctx.affine((shape[1], shape[0]), 128.0, 128.0, 4)
    _check_hough(ctx, g)
    flagged, changed, _, _ = ctx.guard_stats()
    if name.startswith("near_edge"):      # every match sits on an x and a y edge
        assert flagged == (0 if ctx.trig_exact() else len(g["match_q"]))
        print("%s: %d listed, %d bins changed by the guard" % (name, flagged, changed))
    else:
        assert changed == 0


@pytest.mark.parametrize("nq", [40000, 530000])
def test_member_order_at_scale(ctx, nq):
    """Large bins (thousands of members, filled by many waves in arbitrary order): every
    valid bin's member list is in query order, holds exactly its vote count, and only good
    matches.  40 000 queries: small bins sorted in a wave, large ones through the LDS
    bitmap; 530 000 (> 512 Ki): large bins rebuilt by members_kernel's query scan."""
    db = synthetic.make_database(20, 1000, seed=0)
    qs = synthetic.make_queries(nq, seed=5, db_seed=0, kp_per_image=1000, n_objects=2)
    ctx.set_impl("i8")
    ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
    ctx.upload_db(db.des)
    ctx.upload_queries(qs.des, qs.kp)
    ctx.pipeline(qs.shape, (32, 32, 8, 12), ratio=0.75, vote_threshold=5, affine_threshold=4)
    _, _, _, good = ctx.match_result()
    v = ctx.valid_result()
    off, mem = v["offsets"], v["members"]
    sizes = np.diff(off)
    assert sizes.max() > 1000                      # spans many fill blocks
    assert np.array_equal(sizes, v["votes"])
    assert good[mem].all()
    for i in range(len(sizes)):
        seg = mem[off[i]:off[i + 1]]
        assert np.all(np.diff(seg) > 0), "bin %d members not in query order" % i
    ctx.set_impl("bf16")


def _hough_state(c, shape, bins, thr, fused, affine=True):
    c.set_option("hough_fused", int(fused))
    c.hough_select(shape, bins, thr)
    if affine:
        c.affine((shape[1], shape[0]), 128.0, 128.0, 4)
    out = {"valid": c.valid_result(), "bins": c.all_bins(), "guard": c.guard_stats()[:2]}
    if affine:
        out["affine"] = c.affine_result()
    # another threshold on the same votes (needs the dense histogram the fused path skips)
    c.select(max(1, thr - 2))
    out["valid_lo"] = c.valid_result()
    return out


def _same_hough(a, b):
    for k in ("keys", "votes", "offsets", "members"):
        assert np.array_equal(a["valid"][k], b["valid"][k]), k
        assert np.array_equal(a["valid_lo"][k], b["valid_lo"][k]), k
    assert np.array_equal(a["valid"]["means"], b["valid"]["means"])
    assert np.array_equal(a["bins"][0], b["bins"][0]) and np.array_equal(a["bins"][1], b["bins"][1])
    assert a["guard"] == b["guard"]
    if "affine" in a:
        for k in ("survived", "votes", "params", "alive"):
            assert np.array_equal(a["affine"][k], b["affine"][k]), k


@pytest.mark.parametrize("name,ngroups", [("near_edge_b15", 78), ("near_edge_b32", 78),
                                          ("edge_b15", 0), ("edge_b6", 0)])
def test_fused_hough_select_equals_dense(ctx, name, ngroups, trig):
    """The fused one-image launch (hough_small_kernel: pose, votes from a base-key hash, valid
    bins, members, affine inputs) equals the dense path (pose_kernel + hist_kernel +
    select_small_kernel + affine_gather_kernel) bit for bit -- bin table, valid bins, members,
    means, affine results, a second threshold -- on the reference's edge fixtures, including
    matches on bin edges that the boundary guard re-does on the host (<= 1024 of them)."""
    g = golden(name)
    q, m = g["match_q"], g["match_m"]
    if ngroups:
        keep = q < ngroups * 13
        q, m = q[keep], m[keep]
    nq = int(q.max()) + 1
    kq = kp(g, "q_").slice(0, nq)
    shape = tuple(int(v) for v in g["shape"])
    outs = []
    for fused in (True, False):
        ctx.set_keypoints(kp(g, "db_"), g["db_img"], g["centroid"], g["size"])
        ctx.upload_queries(None, kq)
        idx1 = np.zeros(nq, np.int32)
        idx1[q] = m
        good = np.zeros(nq, bool)
        good[q] = True
        ctx.set_matches(idx1, good)
        outs.append(_hough_state(ctx, shape, int(g["bins"]), 5, fused))
    _same_hough(*outs)
    if name.startswith("near_edge"):
        assert outs[0]["guard"][0] == (0 if ctx.trig_exact() else len(q))


@pytest.mark.parametrize("nq,thr,n_objects,decoy", [(500, 5, 4, 0.05), (1024, 5, 2, 0.05),
                                                    (1024, 1, 4, 0.6), (700, 2, 0, 0.05),
                                                    (1, 1, 1, 0.0)])
def test_fused_pipeline_equals_dense(ctx, nq, thr, n_objects, decoy):
    """One query image through the whole pipeline, fused vs dense Hough / select, against
    the 1M-row-shaped DB of 200 images: identical bins, members, means, affine results and
    a second threshold.  thr 1 with many decoys (good matches at random poses) makes
    thousands of valid bins (past the fused kernel's LDS copy of 2048: its global spill
    path); n_objects 0 = no planted object (random votes only)."""
    db = synthetic.make_database(200, 1000, seed=0)
    qs = synthetic.make_queries(nq, seed=9, db_seed=0, kp_per_image=1000,
                                n_objects=max(1, n_objects), planted_frac=0.3 if n_objects else 0.0,
                                decoy_frac=decoy)
    ctx.set_impl("i8")
    ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
    ctx.upload_db(db.des)
    outs = []
    for fused in (True, False):
        ctx.set_option("hough_fused", int(fused))
        ctx.upload_queries(qs.des, qs.kp)
        ctx.pipeline(qs.shape, (32, 32, 8, 12), ratio=0.75, vote_threshold=thr, affine_threshold=4)
        o = {"valid": ctx.valid_result(), "bins": ctx.all_bins(), "guard": ctx.guard_stats()[:2],
             "affine": ctx.affine_result(), "post": ctx.postprocess()}
        ctx.select(max(1, thr - 1))
        o["valid_lo"] = ctx.valid_result()
        outs.append(o)
    _same_hough(*outs)
    assert np.array_equal(outs[0]["post"]["final_pose"], outs[1]["post"]["final_pose"])
    if thr == 1 and nq > 1:
        assert len(outs[0]["valid"]["keys"]) > 2048
    # every result in one transfer (sod_results_fetch) == the per-array getters, with the
    # affine pass and without it (post-processing then over every valid bin: thousands at
    # thr 1, past the staging kernel's 1 024 relation rows -> its host-relations path)
    for run_affine in (True, False):
        for stage in ((), ("match", "valid", "affine", "post")):
            ctx.upload_queries(qs.des, qs.kp)
            ctx.pipeline(qs.shape, (32, 32, 8, 12), ratio=0.75, vote_threshold=thr,
                         affine_threshold=4, run_affine=run_affine, stage=stage)
            _results_equal_getters(ctx, run_affine)
    # staged behind the pipeline, then the selection redone at another threshold: the fetch
    # must not hand back the staged (older) bins
    ctx.upload_queries(qs.des, qs.kp)
    ctx.pipeline(qs.shape, (32, 32, 8, 12), ratio=0.75, vote_threshold=thr, affine_threshold=4,
                 stage=("match", "valid", "affine", "post"))
    ctx.select(thr + 1)
    r = ctx.results(parts=("valid",))
    v = ctx.valid_result()
    for k in ("keys", "votes", "offsets", "members", "means"):
        assert np.array_equal(r["valid"][k], v[k]), k
    r2 = ctx.results(parts=("valid",))               # (a second read of the same staging)
    for k in ("keys", "votes", "offsets", "members", "means"):
        assert np.array_equal(r2["valid"][k], v[k]), k


def _results_equal_getters(ctx, affined=True):
    r = ctx.results(post=True)
    for a, b in zip(r["match"], ctx.match_result()):
        assert np.array_equal(a, b)
    v = ctx.valid_result()
    for k in ("keys", "votes", "offsets", "members", "means"):
        assert np.array_equal(r["valid"][k], v[k]), k
    if affined:
        a = ctx.affine_result()
        for k in ("survived", "votes", "params", "alive"):
            assert np.array_equal(r["affine"][k], a[k]), k
    else:
        assert "affine" not in r
    p = ctx.postprocess_getter()
    for k in p:
        assert np.array_equal(r["post"][k], p[k]), k


def test_knn_indices_refused_after_matches_set(ctx):
    """sod_match_knn_indices after sod_matches_set (matches without distances) is refused
    with SOD_ESTATE instead of returning the caller's indices and a search at distance 0."""
    from sift_based_od_amd.database import Keypoints
    g = golden("matcher_edges")
    n = len(g["db_des"])
    z = np.zeros(n, np.float32)
    ctx.set_keypoints(Keypoints(z, z, z, np.zeros(n, np.int32)), np.zeros(n, np.int32),
                      np.zeros((1, 2)), np.array([[1500, 1000]], np.int32))
    ctx.upload_db(g["db_des"])
    ctx.upload_queries(g["q_des"])
    ctx.set_matches(g["idx1"], g["good"])
    with pytest.raises(_lib.SodError) as e:
        ctx.knn_indices()
    assert e.value.code == _lib.SOD_ESTATE
    ctx.match()                     # a real match makes them available again
    ctx.ratio(0.75)
    i1, i2 = ctx.knn_indices()
    assert np.array_equal(i1, g["idx1"])
