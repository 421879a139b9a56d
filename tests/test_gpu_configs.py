"""GPU parity at BASELINE.json's other configurations, each at its own size:

* configs[1] = C2: 10 000 queries x 100 000 DB rows, BF k=2 + ratio test (bins 15 for the
  Hough stage after it) -- the WHOLE match against the oracle (every query), then the bin
  table / valid bins / members / means against the oracle on those matches;
* the one-query-image regime main.py runs (main.py:36-86: one query image of ~500
  keypoints against the whole DB): 500 x 1 000 000 (query tiles per wave 2, no seed read-back),
  every query against the oracle;
* configs[3] / configs[4] = C4 / C5: 50 000 x 8 000 000 (the DB of 8 GPUs, 1M rows each),
  Hough 32x32x8x12 + affine verify -- on ONE MI355X (an 8M-row int8 DB is 1.1 GB): one
  context holding all 8M rows, checked on a seeded query sample against the oracle over all
  8M rows and stage by stage against the oracle on its good matches; and the DB sharded 8
  ways (8 contexts of 1M rows, C4's decomposition, exchanging through a host communicator),
  equal to the one context bit for bit.  (The RCCL transport of that exchange needs one GPU
  per rank; the driver's 8-GPU bench runs it.)

References: main.py:70-86 (match + ratio), main.py:89-157 (Hough, valid bins, affine),
main.py:139-157 (the verification C5 adds).
"""
import threading

import numpy as np
import pytest

from helpers import ThreadComm, assert_stages_equal_oracle, oracle_inputs
from oracle import oracle as orc
from sift_based_od_amd import _lib, synthetic
import sift_based_od_amd as sod

pytestmark = pytest.mark.gpu

BINS_C3 = (32, 32, 8, 12)


def _stages_vs_oracle(ctx, db, qs, idx1, good, bins, run_affine=True, post=True):
    matches = [(int(q), int(idx1[q])) for q in np.nonzero(good)[0]]
    dbkp, qkp, images = oracle_inputs(db, qs.kp)
    table = orc.hough_vote(matches, qkp, dbkp, images, bins, qs.shape)
    vb = orc.valid_bins(table, 5)
    aff = orc.affine_verify(vb, qkp, dbkp, (qs.shape[1], qs.shape[0]), 4) if run_affine else None
    valid = ctx.valid_result()
    assert len(vb) > 0
    assert_stages_equal_oracle(valid, ctx.affine_result() if run_affine else None, table, vb,
                               aff, bins_all=ctx.all_bins(),
                               post=ctx.postprocess() if post else None)
    return valid


def _set_kernel(ctx, kernel, paired_qt):
    """"auto", or "paired": the ring kernel with paired waves
    (option match_pair = 2) at paired_qt query tiles per wave -- the same queries per
    work-group as the default pick, each wave of a pair taking every other subtile."""
    if kernel == "paired":
        ctx.set_match_kernel("auto")
        ctx.set_option("match_qt", paired_qt)
        ctx.set_option("match_pair", 2)
    else:
        ctx.set_match_kernel(kernel)


@pytest.mark.parametrize("kernel", ["auto", "paired"])
def test_c2_full_match_and_hough(ctx, kernel):
    """configs[1]: 10k x 100k -- every query's trainIdx, d1, d2 and ratio decision against
    the oracle; the chunks are short (4-8 k rows), so the shared thresholds, the seed pass and
    its read-back (<= 64 chunks) and QT 4 are all in play."""
    db = synthetic.make_database(100, 1000, seed=0)
    qs = synthetic.make_queries(10000, seed=1, db_seed=0, kp_per_image=1000)
    _set_kernel(ctx, kernel, 8)
    ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
    ctx.upload_db(db.des)
    ctx.upload_queries(qs.des, qs.kp)
    for _ in range(2):              # the second launch reuses a reset threshold slot
        ctx.pipeline(qs.shape, 15, ratio=0.75, vote_threshold=5, affine_threshold=4)
    idx1, d1, d2, good = ctx.match_result()
    e1, f1, f2 = orc.knn2_match(qs.des, db.des, chunk=512)
    assert np.array_equal(idx1, e1)
    assert np.array_equal(d1.view(np.uint32), f1.view(np.uint32))
    assert np.array_equal(d2.view(np.uint32), f2.view(np.uint32))
    assert np.array_equal(good, orc.ratio_test(f1, f2))
    assert ctx.exact_order()
    _stages_vs_oracle(ctx, db, qs, idx1, good, 15)


@pytest.mark.parametrize("kernel", ["auto", "paired"])
def test_one_query_image_1m(ctx, kernel):
    """main.py's real use: ONE query image (500 keypoints) against a 1M-row DB -- 2 query
    tiles per wave, 124+ DB chunks per query block (no seed read-back); every query against
    the oracle, then the Hough / affine stages."""
    db = synthetic.make_database(1000, 1000, seed=0, workers=8)
    qs = synthetic.make_queries(500, seed=11, db_seed=0, kp_per_image=1000, planted_frac=0.5)
    _set_kernel(ctx, kernel, 4)
    ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
    ctx.upload_db(db.des)
    ctx.upload_queries(qs.des, qs.kp)
    ctx.pipeline(qs.shape, BINS_C3, ratio=0.75, vote_threshold=5, affine_threshold=4)
    idx1, d1, d2, good = ctx.match_result()
    e1, f1, f2 = orc.knn2_match(qs.des, db.des, chunk=128)
    assert np.array_equal(idx1, e1)
    assert np.array_equal(d1, f1) and np.array_equal(d2, f2)
    assert np.array_equal(good, orc.ratio_test(f1, f2))
    _stages_vs_oracle(ctx, db, qs, idx1, good, BINS_C3)


# ---- C4 / C5: the 8M-row DB ---------------------------------------------------------------
N_IMG_C4 = 8000                 # 8 GPUs x 1000 images x 1000 keypoints


@pytest.fixture(scope="module")
def c4():
    db = synthetic.make_database(N_IMG_C4, 1000, seed=0, workers=16)
    qs = synthetic.make_queries(50000, seed=1, db_seed=0, kp_per_image=1000)
    return db, qs


@pytest.fixture(scope="module")
def c5_single(c4):
    """The C5 pipeline (match, ratio, Hough 32x32x8x12, select, affine) with all 8M rows in
    one context."""
    db, qs = c4
    with _lib.Context(0) as c:
        c.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c.upload_db(db.des)
        c.upload_queries(qs.des, qs.kp)
        c.pipeline(qs.shape, BINS_C3, ratio=0.75, vote_threshold=5, affine_threshold=4)
        out = {"match": c.match_result(), "valid": c.valid_result(),
               "affine": c.affine_result(), "bins": c.all_bins(), "post": c.postprocess(),
               "exact": c.exact_order()}
    return out


def test_c5_8m_single_context_vs_oracle(c4, c5_single):
    db, qs = c4
    idx1, d1, d2, good = c5_single["match"]
    assert c5_single["exact"]
    # matcher: a seeded sample against the oracle over ALL 8M rows (blocked by 1M rows)
    sample = np.sort(np.random.default_rng(8).choice(len(qs.des), 192, replace=False))
    e1, f1, f2 = orc.knn2_match_blocked(qs.des[sample], db.des, block=1 << 20, chunk=64)
    assert np.array_equal(idx1[sample], e1)
    assert np.array_equal(d1[sample], f1) and np.array_equal(d2[sample], f2)
    assert np.array_equal(good[sample], orc.ratio_test(f1, f2))
    assert np.array_equal(good, orc.ratio_test(d1, d2))
    # planted queries find their DB row (the synthetic ground truth) wherever they passed
    planted = (qs.planted_db_row >= 0) & good
    assert planted.sum() > 5000
    assert np.mean(idx1[planted] == qs.planted_db_row[planted]) > 0.99
    # every stage after the matcher against the oracle on the same good matches
    matches = [(int(q), int(idx1[q])) for q in np.nonzero(good)[0]]
    dbkp, qkp, images = oracle_inputs(db, qs.kp)
    table = orc.hough_vote(matches, qkp, dbkp, images, BINS_C3, qs.shape)
    vb = orc.valid_bins(table, 5)
    aff = orc.affine_verify(vb, qkp, dbkp, (qs.shape[1], qs.shape[0]), 4)
    assert any(r["survived"] for r in aff)
    assert_stages_equal_oracle(c5_single["valid"], c5_single["affine"], table, vb, aff,
                               bins_all=c5_single["bins"], post=c5_single["post"])


def test_c4_db_sharded_8_ways_equals_single(c4, c5_single):
    """C4's decomposition at its size: 8 contexts (one per would-be GPU) of 1M rows each,
    one host thread each, exchanging the 12 B/query candidates (all-gather + global merge +
    ratio) and the Hough partials (sum / min all-reduce) -- every rank's matches, bin table,
    valid bins, members, means, survivors and parameters equal the 8M-row context's."""
    db, qs = c4
    world = 8
    comm = ThreadComm(world)
    results = [None] * world
    errors = []

    def rank_main(r):
        try:
            lo, hi = sod.shard_range(len(db.des), r, world)
            with _lib.Context(0) as c:
                c.set_keypoints(db.kp, db.img, db.centroid, db.size)
                c.upload_db(db.des[lo:hi], row_offset=lo)
                c.upload_queries(qs.des, qs.kp)
                sod.run_sharded(c, comm.for_rank(r), (lo, hi), qs.shape, BINS_C3)
                results[r] = (c.match_result(), c.valid_result(), c.affine_result(),
                              c.all_bins())
        except Exception as e:  # noqa: BLE001
            errors.append(e)
            comm.bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    m0, v0, a0, b0 = c5_single["match"], c5_single["valid"], c5_single["affine"], c5_single["bins"]
    for m1, v1, a1, b1 in results:
        for x, y in zip(m0, m1):
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
        for k in ("keys", "votes", "offsets", "members", "means"):
            assert np.array_equal(v0[k], v1[k]), k
        assert np.array_equal(b0[0], b1[0]) and np.array_equal(b0[1], b1[1])
        for k in ("survived", "votes", "params", "alive"):
            assert np.array_equal(a0[k], a1[k]), k
