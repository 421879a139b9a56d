"""GPU: the drop-in Python API (reference names) and the sharded path with real kernels.
Sharding is exercised with N contexts on one GPU, one host thread each, exchanging
through a thread-barrier host communicator (the RCCL path needs one GPU per rank)."""
import threading

import numpy as np
import pytest

from conftest import golden
from helpers import ThreadComm, assert_stages_equal_oracle, kp, kp_dict, oracle_inputs
from oracle import oracle as orc
from sift_based_od_amd import _lib, synthetic
import sift_based_od_amd as sod

pytestmark = pytest.mark.gpu


def test_bfmatcher_knnmatch():
    g = golden("c1_b15")
    matches = sod.BFMatcher().knnMatch(g["q_des"].astype(np.float32),
                                       g["db_des"].astype(np.float32), k=2)
    assert len(matches) == len(g["q_des"])
    for q, (m, n) in enumerate(matches):
        assert m.queryIdx == q and m.trainIdx == g["idx1"][q]
        assert np.float32(m.distance) == g["d1"][q] and np.float32(n.distance) == g["d2"][q]
        assert (m.distance < 0.75 * n.distance) == g["good"][q]


def test_bfmatcher_single_train_row():
    q = np.random.default_rng(0).integers(0, 256, (5, 128)).astype(np.uint8)
    out = sod.BFMatcher().knnMatch(q, q[:1], k=2)
    assert all(len(m) == 1 and m[0].trainIdx == 0 for m in out)


def test_bfmatcher_empty_sets():
    """OpenCV's knnMatch: no queries -> no lists; no train rows -> an empty list per query."""
    q = np.random.default_rng(1).integers(0, 256, (4, 128)).astype(np.uint8)
    assert sod.BFMatcher().knnMatch(q[:0], q, k=2) == []
    assert sod.BFMatcher().knnMatch(q, q[:0], k=2) == [[], [], [], []]


def test_scalar_pose_and_bin_index():
    g = golden("pose_sweep")
    shape = tuple(int(v) for v in g["shape"])
    for i in range(0, 20000, 997):
        kM = sod.KeyPoint(g["mx"][i], g["my"][i], 0, g["ma"][i], 0, int(g["mo"][i]))
        kQ = sod.KeyPoint(g["qx"][i], g["qy"][i], 0, g["qa"][i], 0, int(g["qo"][i]))
        p = sod.estimate_object_pose((kM, kQ, (1500, 1000), (g["cx"][i], g["cy"][i])))
        np.testing.assert_allclose(p, g["poses"][i], rtol=1e-13, atol=1e-10)
        for j, b in enumerate(g["bins"]):
            assert sod.calculate_bin_index(tuple(g["poses"][i]), int(b), shape) == \
                tuple(g["idx"][j][i])
    # batch form with per-axis bins reduces to the scalar form
    idx = sod.calculate_bin_index_batch(g["poses"], (15, 15, 15, 15), shape)
    assert np.array_equal(idx, g["idx"][0])


def _tuples(g):
    db_kp, q_kp = kp(g, "db_"), kp(g, "q_")
    out = []
    for q, m in zip(g["match_q"], g["match_m"]):
        im = int(g["db_img"][m])
        out.append((sod.KeyPoint(db_kp.x[m], db_kp.y[m], 0, db_kp.angle[m], 0, int(db_kp.octave[m])),
                    sod.KeyPoint(q_kp.x[q], q_kp.y[q], 0, q_kp.angle[q], 0, int(q_kp.octave[q])),
                    (int(g["size"][im][0]), int(g["size"][im][1])),
                    (float(g["centroid"][im][0]), float(g["centroid"][im][1]))))
    return out


@pytest.mark.parametrize("name", ["edge_b15", "edge_b6"])
def test_perform_hough_transform_and_affine_dropins(name):
    g = golden(name)
    t = _tuples(g)
    b = int(g["bins"])
    shape = tuple(int(v) for v in g["shape"])
    table = sod.perform_hough_transform(t, type("I", (), {"shape": shape})(), b, b, b, b)
    assert [k for k in table] == [tuple(k) for k in g["table_keys"]]
    assert [v.votes for v in table.values()] == list(g["table_votes"])
    valid = [v for v in table.values() if v.votes >= 5]
    assert [v.pose for v in valid] == [tuple(k) for k in g["valid_keys"]]
    # one AffineParameters + remove_outliers round per bin == the oracle's round
    for v in valid[:20]:
        mp = [p[0].pt for p in v.keypoint_pairs]
        qp = [p[1].pt for p in v.keypoint_pairs]
        sod.AffineParameters(v)
        ref = orc.affine_params(mp, qp)
        np.testing.assert_allclose(v.affine_parameters, ref, rtol=1e-6, atol=1e-4)
        keep_ref, ch_ref = orc.remove_outliers(v.affine_parameters, mp, qp, v.pose[3],
                                               (shape[1], shape[0]))
        n0 = v.votes
        _, changed = sod.remove_outliers(v, (shape[1], shape[0]), 128, 128)
        assert changed == ch_ref and v.votes == sum(keep_ref) and n0 == len(keep_ref)


@pytest.mark.parametrize("trig", ["auto", "fallback"])
def test_main_stages_match_golden(trig):
    """main.py's stage sequence through Main against the reference's outputs; "fallback"
    forces the host-libm redo paths (option trig_exact 0: boundary guard, exact means of
    the survivors, pipeline.py) that a host whose libm differs from the device's takes."""
    g = golden("planted_b15")
    db = sod.SiftDatabase(g["db_des"], kp(g, "db_"), g["db_img"], g["centroid"], g["size"])
    m = sod.Main()
    m.ctx.set_option("trig_exact", -1 if trig == "auto" else 0)
    assert trig == "auto" or not m.ctx.trig_exact()
    m.set_database(db)
    m.get_query_features(g["q_des"], kp(g, "q_"), tuple(int(v) for v in g["shape"]))
    m.run_matcher()
    assert len(m.matching_keypoints) == int(g["good"].sum())
    m.apply_hough_transform(int(g["bins"]))
    assert [k for k in m.hough_transform] == [tuple(k) for k in g["table_keys"]]
    m.get_valid_bins(5)
    assert [b.pose for b in m.valid_bins] == [tuple(k) for k in g["valid_keys"]]
    assert [b.votes for b in m.valid_bins] == list(g["valid_votes"])
    for b, mu in zip(m.valid_bins, g["valid_means"]):
        np.testing.assert_allclose([b.centroid[0], b.centroid[1], b.angle, b.scale,
                                    b.img_size[0], b.img_size[1]], mu, rtol=1e-12, atol=1e-9)
    # the x / y means as the reference computes them (glibc per member): bit for bit
    xy = m.ctx.exact_means(np.arange(len(m.valid_bins)))
    ref_xy = np.ascontiguousarray(np.asarray(g["valid_means"], np.float64)[:, :2])
    assert np.array_equal(xy.view(np.uint64), ref_xy.view(np.uint64))
    m.apply_affine_parameters(4)
    assert m.affine_path == "device-resident"
    assert [b.pose for b in m.valid_bins] == [tuple(k) for k in g["surv_keys"]]
    assert [b.votes for b in m.valid_bins] == list(g["surv_votes"])
    for b, prm in zip(m.valid_bins, g["surv_params"]):
        np.testing.assert_allclose(b.affine_parameters, prm, rtol=0, atol=1e-4)
    assert len(m.keypoint_pairs) == int(g["surv_votes"].sum())
    m.post_process()                                   # main.py:186
    got = np.array([[p[0][0], p[0][1], p[1], p[2], p[3][0], p[3][1]] for p in m.final_pose])
    # survivors' centroids redone with glibc (sod_exact_means): main.py's final pose exactly
    assert np.array_equal(got.reshape(-1, 6).view(np.uint64),
                          np.asarray(g["final_pose"], np.float64).reshape(-1, 6).view(np.uint64))


def _main_on_given_matches(g, seed=3):
    """A Main whose run_matcher finds exactly the golden's (match_q, match_m) pairs: random
    DB descriptors, query q's descriptor = DB row match_m[q] (d1 = 0, ratio test passes)."""
    rng = np.random.default_rng(seed)
    ndb, nq = len(g["db_x"]), len(g["q_x"])
    assert np.array_equal(g["match_q"], np.arange(nq))        # every query is matched
    db_des = rng.integers(0, 256, (ndb, 128)).astype(np.uint8)
    m = sod.Main()
    m.set_database(sod.SiftDatabase(db_des, kp(g, "db_"), g["db_img"], g["centroid"], g["size"]))
    m.get_query_features(db_des[g["match_m"]], kp(g, "q_"), tuple(int(v) for v in g["shape"]))
    m.run_matcher()
    assert len(m.matching_keypoints) == nq
    return m


def _pair_queries(m, pairs):
    qid = {id(v): k for k, v in m.kp_query._cache.items()}
    return np.array([qid[id(p[1])] for p in pairs], np.int64)


@pytest.mark.parametrize("name", ["edge_b15", "near_edge_b15"])
@pytest.mark.parametrize("seq", [(5, 7), (7, 5), (9, 3)])
@pytest.mark.parametrize("path", ["device", "tuples"])
def test_get_valid_bins_repeated(name, seq, path):
    """get_valid_bins called twice (main.py:121-132), against the reference run the same way
    (repeat_<case> goldens): valid_bins keeps the first call's bins and appends the second
    call's new ones in insertion order; keypoint_pairs holds only the LATEST threshold's bins'
    pairs, in hough_transform order; apply_affine_parameters then verifies the accumulated
    list.  ``tuples``: the matches assigned as tuples (the host-table path)."""
    g, r = golden(name), golden("repeat_" + name)
    m = _main_on_given_matches(g)
    if path == "tuples":
        m.matching_keypoints = list(m.matching_keypoints)
    m.apply_hough_transform(int(g["bins"]))
    tag = "t%d_%d_" % seq
    for step, thr in enumerate(seq):
        m.get_valid_bins(thr)
        assert [b.pose for b in m.valid_bins] == [tuple(k) for k in r[tag + "valid_keys%d" % step]]
        assert np.array_equal(_pair_queries(m, m.keypoint_pairs), r[tag + "pairs%d" % step])
    m.apply_affine_parameters(4)
    assert [b.pose for b in m.valid_bins] == [tuple(k) for k in r[tag + "surv_keys"]]
    assert [b.votes for b in m.valid_bins] == list(r[tag + "surv_votes"])
    for b, prm in zip(m.valid_bins, r[tag + "surv_params"]):
        np.testing.assert_allclose(b.affine_parameters, prm, rtol=0, atol=1e-4)
    assert np.array_equal(_pair_queries(m, m.keypoint_pairs), r[tag + "surv_pairs"])


def test_hough_read_between_select_and_affine():
    """Reading hough_transform after get_valid_bins selects again on the device (threshold 1);
    apply_affine_parameters must still verify get_valid_bins' bins (the
    device-resident shortcut checks that the device selection is still that one)."""
    g = golden("edge_b15")
    m = _main_on_given_matches(g)
    m.apply_hough_transform(int(g["bins"]))
    m.get_valid_bins(5)
    assert len(m.hough_transform) == len(g["table_keys"])
    m.apply_affine_parameters(4)
    assert [b.pose for b in m.valid_bins] == [tuple(k) for k in g["surv_keys"]]
    assert [b.votes for b in m.valid_bins] == list(g["surv_votes"])
    for b, prm in zip(m.valid_bins, g["surv_params"]):
        np.testing.assert_allclose(b.affine_parameters, prm, rtol=0, atol=1e-4)


def _kf_rows(kps):
    return np.array([[k.pt[0], k.pt[1], k.size, k.angle, k.response, k.octave, k.class_id]
                     for k in kps], np.float64).reshape(-1, 7)


@pytest.mark.parametrize("name", ["c1_b15", "planted_b15"])
def test_main_keypoint_fields(name):
    """Main hands back the reference's KeyPoint objects (SiftHelperFunctions.py:42-49,
    main.py:43,65,85-86): the DB set from the reference's pickle records and the query's
    KeyPoint objects given, matching_keypoints and every valid / surviving bin's
    keypoint_pairs equal the reference's own Main output (kpfields_* goldens) field by field
    -- pt, size, angle, response, octave, class_id -- and the query keypoints are the
    caller's very objects, as in the reference."""
    g, kf = golden(name), golden("kpfields_" + name)
    mk_obj = lambda pre, src, i: sod.KeyPoint(  # noqa: E731
        float(g[pre + "x"][i]), float(g[pre + "y"][i]), float(src[pre + "size"][i]),
        float(g[pre + "angle"][i]), float(src[pre + "response"][i]), int(g[pre + "octave"][i]),
        int(src[pre + "class_id"][i]))
    records = []
    for im in range(len(g["centroid"])):
        rows = np.nonzero(g["db_img"] == im)[0]
        records.append([sod.make_temp_kp([mk_obj("db_", kf, r) for r in rows]), g["db_des"][rows],
                        (int(g["size"][im][0]), int(g["size"][im][1])),
                        (float(g["centroid"][im][0]), float(g["centroid"][im][1])), "img"])
    qk = [mk_obj("q_", kf, i) for i in range(len(g["q_x"]))]
    m = sod.Main()
    m.set_database(records)
    m.get_query_features(g["q_des"], qk, tuple(int(v) for v in g["shape"]))
    m.run_matcher()
    mk = m.matching_keypoints
    assert np.array_equal(_kf_rows([t[0] for t in mk]), kf["mk_model"])
    assert np.array_equal(_kf_rows([t[1] for t in mk]), kf["mk_query"])
    assert all(t[1] is qk[q] for t, q in zip(mk, kf["mk_q"]))           # the caller's objects
    assert np.array_equal(np.array([t[2] for t in mk]).reshape(-1, 2), kf["mk_img_size"])
    assert np.array_equal(np.array([t[3] for t in mk]).reshape(-1, 2), kf["mk_centroid"])
    assert all(m.kp[int(g["idx1"][q])] is t[0] for t, q in zip(mk, kf["mk_q"]))  # one object per row
    m.apply_hough_transform(int(g["bins"]))
    m.get_valid_bins(5)
    for tag, bins in (("valid", m.valid_bins),):
        off = np.concatenate([[0], np.cumsum([len(b.keypoint_pairs) for b in bins])])
        assert np.array_equal(off, kf[tag + "_off"])
        pairs = [p for b in bins for p in b.keypoint_pairs]
        assert np.array_equal(_kf_rows([p[0] for p in pairs]), kf[tag + "_pairs_model"])
        assert np.array_equal(_kf_rows([p[1] for p in pairs]), kf[tag + "_pairs_query"])
    m.apply_affine_parameters(4)
    off = np.concatenate([[0], np.cumsum([len(b.keypoint_pairs) for b in m.valid_bins])])
    assert np.array_equal(off, kf["surv_off"])
    pairs = list(m.keypoint_pairs)
    assert np.array_equal(_kf_rows([p[0] for p in pairs]), kf["surv_pairs_model"])
    assert np.array_equal(_kf_rows([p[1] for p in pairs]), kf["surv_pairs_query"])


def _main_on(g):
    db = sod.SiftDatabase(g["db_des"], kp(g, "db_"), g["db_img"], g["centroid"], g["size"])
    m = sod.Main()
    m.set_database(db)
    m.get_query_features(g["q_des"], kp(g, "q_"), tuple(int(v) for v in g["shape"]))
    m.run_matcher()
    m.apply_hough_transform(int(g["bins"]))
    return m


def test_main_device_resident_members():
    """main.py:121-157 without the PoseBin objects' members ever leaving the device: the
    valid bins' keypoint pairs are not built until read, the affine stage runs on the
    resident members, and survivors / votes / parameters / surviving members equal the
    reference's goldens."""
    g = golden("planted_b12")
    m = _main_on(g)
    m.get_valid_bins(5)
    assert all(b._lazy is not None for b in m.valid_bins)       # nothing materialised yet
    m.apply_affine_parameters(4)
    assert m.affine_path == "device-resident"
    assert [b.pose for b in m.valid_bins] == [tuple(k) for k in g["surv_keys"]]
    assert [b.votes for b in m.valid_bins] == list(g["surv_votes"])
    for k, b in enumerate(m.valid_bins):
        np.testing.assert_allclose(b.affine_parameters, g["surv_params"][k], rtol=0, atol=1e-4)
        want = g["surv_members"][g["surv_off"][k]:g["surv_off"][k + 1]]
        assert [p[1] for p in b.keypoint_pairs] == [m.kp_query[int(q)] for q in want]
    assert len(m.keypoint_pairs) == int(g["surv_votes"].sum())


def test_main_edited_bins_take_the_host_path():
    """A caller that edits the valid bins (drops a member of one bin) gets the affine stage
    on the bins' own pairs -- the edit counts; every other bin's outcome is the reference's."""
    g = golden("planted_b12")
    m = _main_on(g)
    m.get_valid_bins(5)
    edited = m.valid_bins[0]
    edited.keypoint_pairs.pop()
    edited.votes -= 1
    others = [b.pose for b in m.valid_bins[1:]]
    m.apply_affine_parameters(4)
    assert m.affine_path == "host-pairs"
    surv = [tuple(k) for k in g["surv_keys"]]
    got = [b.pose for b in m.valid_bins if b.pose != edited.pose]
    assert got == [p for p in surv if p in others]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_in_process_equals_single(world):
    db = synthetic.make_database(12, 500, seed=31)
    qs = synthetic.make_queries(3000, seed=32, db_seed=31, kp_per_image=500)
    bins = (32, 32, 8, 12)
    # single context
    with _lib.Context(0) as c:
        c.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c.upload_db(db.des)
        c.upload_queries(qs.des, qs.kp)
        c.pipeline(qs.shape, bins)
        ref = (c.match_result(), c.valid_result(), c.affine_result())
    comm = ThreadComm(world)
    results = [None] * world
    errors = []

    def rank_main(r):
        try:
            lo, hi = sod.shard_range(len(db), r, world)
            with _lib.Context(0) as c:
                c.set_keypoints(db.kp, db.img, db.centroid, db.size)
                c.upload_db(db.des[lo:hi], row_offset=lo)
                c.upload_queries(qs.des, qs.kp)
                sod.run_sharded(c, comm.for_rank(r), (lo, hi), qs.shape, bins)
                results[r] = (c.match_result(), c.valid_result(), c.affine_result())
        except Exception as e:  # noqa: BLE001
            errors.append(e)
            comm.bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    (i1, d1, d2, g1), v1, a1 = ref
    assert v1["keys"].shape[0] > 0
    for (i2, e1, e2, g2), v2, a2 in results:
        assert np.array_equal(i1, i2) and np.array_equal(d1, e1) and np.array_equal(d2, e2)
        assert np.array_equal(g1, g2)
        for k in ("keys", "votes", "offsets", "members"):
            assert np.array_equal(v1[k], v2[k]), k
        assert np.array_equal(v1["means"], v2["means"])
        assert np.array_equal(a1["survived"], a2["survived"])
        assert np.array_equal(a1["params"], a2["params"])


def test_rccl_single_rank_collectives():
    """The RCCL exchange on real hardware: a 1-rank communicator runs the all-gather of
    the match candidates and the (sum, min) all-reduce of the Hough partials (as copies);
    the pipeline result must equal the communicator-less one bit for bit."""
    db = synthetic.make_database(12, 500, seed=41)
    qs = synthetic.make_queries(3000, seed=42, db_seed=41, kp_per_image=500)
    bins = (32, 32, 8, 12)
    out = []
    for use_comm in (False, True):
        with _lib.Context(0) as c:
            if use_comm:
                c.comm_init(1, 0, _lib.unique_id())
                assert c.comm_info() == (1, 0)          # as RCCL reports it
            else:
                with pytest.raises(_lib.SodError):      # no communicator yet
                    c.comm_info()
            c.set_keypoints(db.kp, db.img, db.centroid, db.size)
            c.upload_db(db.des)
            c.upload_queries(qs.des, qs.kp)
            c.pipeline(qs.shape, bins)
            out.append((c.match_result(), c.valid_result(), c.affine_result(), c.all_bins()))
    (m0, v0, a0, b0), (m1, v1, a1, b1) = out
    for x, y in zip(m0, m1):
        assert np.array_equal(x, y)
    for k in ("keys", "votes", "offsets", "members"):
        assert np.array_equal(v0[k], v1[k]), k
    assert np.array_equal(b0[0], b1[0]) and np.array_equal(b0[1], b1[1])
    assert np.array_equal(a0["survived"], a1["survived"])
    assert np.array_equal(a0["params"], a1["params"])


@pytest.mark.parametrize("impl", ["i8", "bf16", "i8w"])
def test_packed_db_roundtrip(tmp_path, impl):
    """save the DB with its device-packed image, load it (no pickle) and
    upload with one copy -- the pipeline results equal the upload + pack path's."""
    db = synthetic.make_database(10, 400, seed=51)
    qs = synthetic.make_queries(2500, seed=52, db_seed=51, kp_per_image=400)
    with _lib.Context(0) as c:
        c.set_impl(impl)
        path = tmp_path / "db.npz"
        db.save(path, ctx=c, keep_descriptors=False)
        loaded = sod.SiftDatabase.load(path)
        assert loaded.des is None and loaded.packed is not None
        c.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c.upload_db(db.des)
        c.upload_queries(qs.des, qs.kp)
        c.pipeline(qs.shape, 15)
        ref = (c.match_result(), c.valid_result())
    with _lib.Context(0) as c:
        c.set_impl(impl)
        loaded.upload(c)
        c.upload_queries(qs.des, qs.kp)
        c.pipeline(qs.shape, 15)
        got = (c.match_result(), c.valid_result())
        assert c.exact_order()
        other = "bf16" if impl != "bf16" else "i8"
        c.set_impl(other)
        with pytest.raises(_lib.SodError):
            c.import_packed(loaded.packed)      # laid out for another matcher
    for x, y in zip(ref[0], got[0]):
        assert np.array_equal(x, y)
    for k in ("keys", "votes", "offsets", "members"):
        assert np.array_equal(ref[1][k], got[1][k])
    # oracle leg: the packed-image upload's pipeline against the oracle run on the raw
    # descriptors (main.py:50-86 flattening + match, then main.py:89-132)
    dbkp, qkp, images = oracle_inputs(db, qs.kp)
    o = orc.run_pipeline(qs.des, qkp, db.des, dbkp, images, 15, qs.shape)
    i1, d1, d2, g = got[0]
    assert np.array_equal(i1, o["idx1"]) and np.array_equal(g, o["good"])
    assert np.array_equal(d1, o["d1"]) and np.array_equal(d2, o["d2"])
    assert len(o["valid"]) > 0
    assert_stages_equal_oracle(got[1], None, o["table"], o["valid"], None)


@pytest.mark.parametrize("fused", [False, True])
def test_query_batch_equals_per_image(fused):
    """three query images matched in one DB pass, then the per-image
    Hough / select / affine / post-processing (on query windows, or fused into one launch
    per stage with image-major bin keys) == each image alone."""
    db = synthetic.make_database(8, 500, seed=61)
    imgs = []
    for k, (nq, shape) in enumerate(((1200, (800, 1000, 3)), (700, (600, 900, 3)),
                                     (1500, (1000, 1200, 3)))):
        qs = synthetic.make_queries(nq, seed=62 + k, db_seed=61, kp_per_image=500,
                                    n_objects=3, shape=shape)
        imgs.append((qs.des, qs.kp, qs.shape))
    with _lib.Context(0) as c:
        c.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c.upload_db(db.des)
        batch = sod.run_query_batch(c, imgs, bins=15, fused=fused)
        for (des, kp_, shape), b in zip(imgs, batch):
            c.upload_queries(des, kp_)
            c.pipeline(shape, 15)
            i1, d1, d2, g = c.match_result()
            assert np.array_equal(i1, b["idx1"]) and np.array_equal(d1, b["d1"])
            assert np.array_equal(d2, b["d2"]) and np.array_equal(g, b["good"])
            v = c.valid_result()
            assert len(v["keys"]) > 0
            for k in ("keys", "votes", "offsets", "members"):
                assert np.array_equal(v[k], b["valid"][k]), k
            np.testing.assert_array_equal(v["means"], b["valid"]["means"])
            a = c.affine_result()
            assert np.array_equal(a["survived"], b["affine"]["survived"])
            np.testing.assert_array_equal(a["params"], b["affine"]["params"])
            p = c.postprocess()
            np.testing.assert_array_equal(p["final_pose"], b["post"]["final_pose"])
            # oracle leg: the batch's per-image results against the oracle's pipeline of
            # that image alone (main.py:68-157 per query image, main.py:178-188)
            dbkp, qkp, images = oracle_inputs(db, kp_)
            o = orc.run_pipeline(des, qkp, db.des, dbkp, images, 15, shape)
            assert np.array_equal(b["idx1"], o["idx1"]) and np.array_equal(b["good"], o["good"])
            assert np.array_equal(b["d1"], o["d1"]) and np.array_equal(b["d2"], o["d2"])
            assert_stages_equal_oracle(b["valid"], b["affine"], o["table"], o["valid"],
                                       o["affine"])
            ref = orc.post_process(b["valid"]["means"][b["post"]["bin_index"]])
            fp = np.array([[q[0][0], q[0][1], q[1], q[2], q[3][0], q[3][1]]
                           for q in ref["final_pose"]]).reshape(-1, 6)
            np.testing.assert_allclose(b["post"]["final_pose"], fp, rtol=1e-12, atol=1e-9)


def test_shared_db_contexts():
    """sod_db_share: a second context over the first one's resident DB (no copy) gives the
    same results, also while both run interleaved on their own streams."""
    db = synthetic.make_database(10, 500, seed=71)
    qa = synthetic.make_queries(2000, seed=72, db_seed=71, kp_per_image=500)
    qb = synthetic.make_queries(1500, seed=73, db_seed=71, kp_per_image=500)
    with _lib.Context(0) as c0:
        c0.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c0.upload_db(db.des)
        c0.upload_queries(qb.des, qb.kp)
        c0.pipeline(qb.shape, 15)
        ref_b = (c0.match_result(), c0.valid_result(), c0.affine_result())
        c0.upload_queries(qa.des, qa.kp)
        with _lib.Context(0) as c1:
            c1.share_db(c0)
            c1.upload_queries(qb.des, qb.kp)
            for _ in range(3):            # interleaved on two streams
                c0.pipeline(qa.shape, 15)
                c1.pipeline(qb.shape, 15)
            got_b = (c1.match_result(), c1.valid_result(), c1.affine_result())
            assert c1.exact_order()
    for x, y in zip(ref_b[0], got_b[0]):
        assert np.array_equal(x, y)
    for k in ("keys", "votes", "offsets", "members"):
        assert np.array_equal(ref_b[1][k], got_b[1][k])
    np.testing.assert_array_equal(ref_b[2]["params"], got_b[2]["params"])


def test_shared_db_write_rules():
    """sod_db_share bookkeeping: the owner refuses DB writes while a context aliases its DB;
    sharing from a sharer shares from the owner; a DB write on a sharer detaches it (its
    own buffers, never the owner's); destroying the owner detaches what is left."""
    db = synthetic.make_database(4, 300, seed=81)
    db2 = synthetic.make_database(4, 300, seed=82)
    qs = synthetic.make_queries(600, seed=83, db_seed=81, kp_per_image=300)
    with _lib.Context(0) as c0:
        c0.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c0.upload_db(db.des)
        c0.upload_queries(qs.des, qs.kp)
        c0.pipeline(qs.shape, 15)
        ref = c0.match_result()
        c1, c2 = _lib.Context(0), _lib.Context(0)
        c1.share_db(c0)
        c2.share_db(c1)                              # shares from the owner, c0
        for bad in (lambda: c0.upload_db(db2.des),
                    lambda: c0.set_keypoints(db2.kp, db2.img, db2.centroid, db2.size),
                    lambda: c0.set_impl("bf16")):
            with pytest.raises(_lib.SodError, match="sod_db_share"):
                bad()
        # c1 takes a DB of its own: c0's stays intact for c0 and c2
        c1.set_keypoints(db2.kp, db2.img, db2.centroid, db2.size)
        c1.upload_db(db2.des)
        for c in (c0, c2):
            c.upload_queries(qs.des, qs.kp)
            c.pipeline(qs.shape, 15)
            for x, y in zip(ref, c.match_result()):
                assert np.array_equal(x, y)
        c1.close()
        with pytest.raises(_lib.SodError, match="sod_db_share"):
            c0.upload_db(db.des)                     # c2 still aliases it
        c2.close()
        c0.upload_db(db.des)                         # no sharer left
        # the owner destroyed first: its sharer reports "no database", reads nothing freed
        c3 = _lib.Context(0)
        c3.share_db(c0)
        c3.upload_queries(qs.des, qs.kp)
    with pytest.raises(_lib.SodError):
        c3.pipeline(qs.shape, 15)
    c3.close()


@pytest.mark.parametrize("use_comm,reserve,affine", [(False, 0, True), (True, 0, True),
                                                     (False, 1, True), (True, 1, True),
                                                     (False, 1, False)])
def test_matcher_overlap_equals_serial(use_comm, reserve, affine):
    """sod_match_set_overlap: the matcher kernel on its own stream, overlapping the previous
    query's Hough / select / affine stages (several pipelines enqueued back to back with
    different vote thresholds -- so consecutive steps have different valid-bin and member
    counts while the PoseBin means of the step before still run on the side stream over
    their double-buffered inputs -- a new query upload in between, optionally a 1-rank RCCL
    communicator on the context stream); with `reserve` the chip is split by CU masks
    (sod_set_cu_reserve: matcher on all but one CU per XCD, the other stages on those) --
    every result equals the serial context's bit for bit."""
    db = synthetic.make_database(30, 1000, seed=51)
    qsets = [synthetic.make_queries(5000, seed=52 + k, db_seed=51, kp_per_image=1000)
             for k in range(2)]
    bins = (32, 32, 8, 12)

    def collect(c):
        return (c.match_result(), c.valid_result(), c.affine_result() if affine else None,
                c.all_bins())

    ref = []
    with _lib.Context(0) as c:
        c.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c.upload_db(db.des)
        for qs in qsets:
            c.upload_queries(qs.des, qs.kp)
            c.pipeline(qs.shape, bins, run_affine=affine)
            ref.append(collect(c))
    with _lib.Context(0) as c:
        if reserve:
            c.set_cu_reserve(reserve)
        else:
            c.set_overlap(True)
        if use_comm:      # under the split: channels capped at the reserved CU count
            c.comm_init(1, 0, _lib.unique_id())
        c.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c.upload_db(db.des)
        c.set_match_timing(True)                # (off by default)
        got = []
        for qs in qsets:
            c.upload_queries(qs.des, qs.kp)
            for thr in (3, 8, 5):               # back to back: matcher k+1 beside tail k
                c.pipeline(qs.shape, bins, vote_threshold=thr, run_affine=affine)
            c.synchronize()
            got.append(collect(c))
        times = c.match_times(3)                # the last three launches, timed live
        assert times.shape == (3,) and np.all(times > 0)
        if reserve:
            with pytest.raises(_lib.SodError):  # the split needs the matcher stream
                c.set_overlap(False)
            c.set_cu_reserve(0)
        c.set_overlap(False)
    for (m0, v0, a0, b0), (m1, v1, a1, b1) in zip(ref, got):
        for x, y in zip(m0, m1):
            assert np.array_equal(x, y)
        for k in ("keys", "votes", "offsets", "members", "means"):
            assert np.array_equal(v0[k], v1[k]), k
        assert np.array_equal(b0[0], b1[0]) and np.array_equal(b0[1], b1[1])
        if affine:
            assert np.array_equal(a0["survived"], a1["survived"])
            assert np.array_equal(a0["params"], a1["params"])


def test_cu_reserve_toggle_stress():
    """The round-4 hang (sod_set_cu_reserve 1 -> 0 never returning from hipStreamDestroy of
    the old CU-masked streams, about one suite run in three): the split switched on and off
    24 times, each time with pipelines in flight (overlapped matcher, PoseBin means on the
    side stream, timed launches -- every kind of event recorded on the streams being
    destroyed); results stay equal to the first round's.  The test's own timeout catches a
    hang."""
    db = synthetic.make_database(8, 1000, seed=71)
    qs = synthetic.make_queries(3000, seed=72, db_seed=71, kp_per_image=1000)
    bins = (32, 32, 8, 12)
    with _lib.Context(0) as c:
        c.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c.upload_db(db.des)
        c.upload_queries(qs.des, qs.kp)
        first = None
        for k in range(24):
            c.set_cu_reserve(1 if k % 2 == 0 else 0)
            if k % 2:
                c.set_overlap(k % 4 == 1)
            for thr in (3, 5):
                c.pipeline(qs.shape, bins, vote_threshold=thr)
            v = c.valid_result()
            if first is None:
                first = v
            for key in ("keys", "votes", "offsets", "members"):
                assert np.array_equal(v[key], first[key]), (k, key)
        c.set_cu_reserve(0)
        c.set_overlap(False)


@pytest.mark.parametrize("nq,streams", [(600, 1), (3000, 1), (600, 2), (3000, 2)])
def test_untimed_split_launches_equal_serial(nq, streams):
    """Under the CU split a matcher launch without timing events signals the context stream
    by the completion event its own dispatch records (no marker packet): back-to-back
    pipelines with different thresholds and a new query upload in between -- the merge must
    still wait for the kernel, and the upload for the kernel reading the old queries; every
    result equals the serial context's."""
    db = synthetic.make_database(60, 1000, seed=61)
    qsets = [synthetic.make_queries(nq, seed=62 + k, db_seed=61, kp_per_image=1000)
             for k in range(3)]
    bins = (32, 32, 8, 12)

    def collect(c):
        return c.match_result(), c.valid_result(), c.affine_result(), c.all_bins()

    ref = []
    with _lib.Context(0) as c:
        c.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c.upload_db(db.des)
        for qs in qsets:
            c.upload_queries(qs.des, qs.kp)
            for thr in (3, 5):
                c.pipeline(qs.shape, bins, vote_threshold=thr)
                ref.append(collect(c))
    got = []
    with _lib.Context(0) as c:
        c.set_cu_reserve(1)
        c.set_matcher_streams(streams)   # 2: consecutive launches overlap on two streams
        c.set_match_timing(0)
        c.set_stage_timing(False)
        c.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c.upload_db(db.des)
        for qs in qsets:
            # right behind the previous set's back-to-back matchers; the first two launches
            # after it find both partial-result slots holding the previous queries' results
            # (a merge that did not wait for its kernel would read those)
            c.upload_queries(qs.des, qs.kp)
            for thr in (3, 5):
                c.pipeline(qs.shape, bins, vote_threshold=thr)
                got.append(collect(c))
            for _ in range(3):                # back to back, nothing read in between
                c.pipeline(qs.shape, bins, vote_threshold=5)
        c.set_cu_reserve(0)
    for (m0, v0, a0, b0), (m1, v1, a1, b1) in zip(ref, got):
        for x, y in zip(m0, m1):
            assert np.array_equal(x, y)
        for k in ("keys", "votes", "offsets", "members", "means"):
            assert np.array_equal(v0[k], v1[k]), k
        assert np.array_equal(b0[0], b1[0]) and np.array_equal(b0[1], b1[1])
        assert np.array_equal(a0["survived"], a1["survived"])
        assert np.array_equal(a0["params"], a1["params"])


def test_cu_reserve_channel_cap():
    """The CU split runs collectives on the reserved CUs only, so every block of an RCCL
    kernel must fit there: a communicator created under the split gets maxCTAs = the reserved
    CU count (per communicator, ncclConfig_t); one created without a split, or with more
    blocks than a later, smaller split reserves, is refused.  The environment is not used."""
    with _lib.Context(0) as c:
        c.comm_init(1, 0, _lib.unique_id())           # RCCL's default block count
        with pytest.raises(_lib.SodError, match="maxCTAs"):
            c.set_cu_reserve(1)
    with _lib.Context(0) as c:
        c.set_cu_reserve(2)                           # 16 reserved CUs
        c.comm_init(1, 0, _lib.unique_id())           # maxCTAs 16
        with pytest.raises(_lib.SodError, match="maxCTAs"):
            c.set_cu_reserve(1)                       # 8 CUs < 16 blocks
        c.set_cu_reserve(2)
        c.set_cu_reserve(0)
    with _lib.Context(0) as c:
        c.set_cu_reserve(1)
        c.comm_init(1, 0, _lib.unique_id())           # maxCTAs 8
        c.set_cu_reserve(1)
        c.set_cu_reserve(0)


@pytest.mark.parametrize("switch", ["overlap", "cu_reserve"])
def test_threshold_slots_after_overlap_switch(switch):
    """The int8 matcher's shared-threshold slots: a context matches once with overlap off
    (one slot in use), then switches the matcher stream on with the SAME query count -- the
    second slot must start from "nothing known", never from uninitialised memory."""
    rng = np.random.default_rng(91)
    db = synthetic.sift_like_descriptors(rng, 120000)
    q = synthetic.sift_like_descriptors(rng, 3000)
    e1, f1, f2 = orc.knn2_match(q, db)
    with _lib.Context(0) as c:
        c.upload_db(db)
        c.upload_queries(q)
        c.match()
        c.ratio(0.75)
        if switch == "overlap":
            c.set_overlap(True)
        else:
            c.set_cu_reserve(1)
        for _ in range(3):          # slots 1, 0, 1
            c.match()
            c.ratio(0.75)
            idx1, d1, d2, _ = c.match_result()
            assert np.array_equal(idx1, e1)
            assert np.array_equal(d1, f1) and np.array_equal(d2, f2)


def test_ratio_argument_validation():
    """A negative or NaN ratio is refused (it used to collide with the 'not fused' marker)."""
    db = synthetic.make_database(2, 300, seed=93)
    qs = synthetic.make_queries(400, seed=94, db_seed=93, kp_per_image=300)
    with _lib.Context(0) as c:
        c.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c.upload_db(db.des)
        c.upload_queries(qs.des, qs.kp)
        c.match()
        for bad in (-1.0, float("nan"), float("inf")):
            with pytest.raises(_lib.SodError, match="ratio"):
                c.ratio(bad)
            with pytest.raises(_lib.SodError, match="ratio"):
                c.pipeline(qs.shape, 15, ratio=bad)
        c.pipeline(qs.shape, 15, ratio=0.75)
        good = c.match_result()[3]
        c.ratio(0.5)                 # a different ratio after a fused one is re-applied
        _, d1, d2, g2 = c.match_result()
        assert np.array_equal(g2, orc.ratio_test(d1, d2, 0.5))
        assert g2.sum() <= good.sum()


@pytest.mark.parametrize("case", ["no_good_matches", "no_valid_bins", "one_query", "ragged"])
def test_pipeline_empty_and_ragged(ctx, case):
    """Edge sizes through the whole device pipeline, against the oracle: no match passes the
    ratio test (ratio 0), no bin reaches the vote threshold, a single query, and query / DB
    counts that fill no tile or stage (17 queries, 1 000 + 3 rows)."""
    nimg, kpi = (1, 1003) if case == "ragged" else (3, 400)
    nq = {"one_query": 1, "ragged": 17}.get(case, 600)
    db = synthetic.make_database(nimg, kpi, seed=41)
    qs = synthetic.make_queries(nq, seed=42, db_seed=41, kp_per_image=kpi, planted_frac=0.6,
                                n_objects=1)
    ratio = 0.0 if case == "no_good_matches" else 0.75
    vthr = 10 ** 6 if case == "no_valid_bins" else 5
    ctx.set_keypoints(db.kp, db.img, db.centroid, db.size)
    ctx.upload_db(db.des)
    ctx.upload_queries(qs.des, qs.kp)
    ctx.pipeline(qs.shape, 15, ratio=ratio, vote_threshold=vthr, affine_threshold=4)
    idx1, d1, d2, good = ctx.match_result()
    e1, f1, f2 = orc.knn2_match(qs.des, db.des)
    assert np.array_equal(idx1, e1) and np.array_equal(d1, f1) and np.array_equal(d2, f2)
    assert np.array_equal(good, orc.ratio_test(f1, f2, ratio))
    matches = [(int(q), int(idx1[q])) for q in np.nonzero(good)[0]]
    dbkp, qkp, images = oracle_inputs(db, qs.kp)
    table = orc.hough_vote(matches, qkp, dbkp, images, 15, qs.shape)
    vb = orc.valid_bins(table, vthr)
    aff = orc.affine_verify(vb, qkp, dbkp, (qs.shape[1], qs.shape[0]), 4)
    keys, votes = ctx.all_bins()
    assert [tuple(k) for k in keys] == list(table.keys())
    assert list(votes) == [b.votes for b in table.values()]
    v = ctx.valid_result()
    assert [tuple(k) for k in v["keys"]] == [b.pose for b in vb]
    a = ctx.affine_result()
    assert list(a["survived"].astype(bool)) == [r["survived"] for r in aff]
    if case == "no_good_matches":
        assert not good.any() and len(keys) == 0 and len(v["keys"]) == 0
    if case == "no_valid_bins":
        assert len(keys) > 0 and len(v["keys"]) == 0
    post = ctx.postprocess()                     # clustering of the survivors: also empty-safe
    if not any(r["survived"] for r in aff):
        assert len(post["final_pose"]) == 0


@pytest.mark.parametrize("bins", [15, (32, 32, 8, 12)])
def test_select_one_workgroup_equals_multi_kernel(bins):
    """Windows of <= 2048 queries take select + member lists in one work-group
    (select_small_kernel); option select_multi 1 forces the multi-kernel path.  Both equal the
    oracle and each other bit for bit (valid bins, votes, offsets, members, means, affine),
    for a plain query window and for a fused batch of two images (image-major bin keys)."""
    db = synthetic.make_database(12, 500, seed=91)
    imgs = []
    for k, (nq, shape) in enumerate(((1900, (800, 1000, 3)), (800, (600, 900, 3)),
                                     (900, (1000, 1200, 3)))):
        qs = synthetic.make_queries(nq, seed=92 + k, db_seed=91, kp_per_image=500,
                                    n_objects=3, shape=shape)
        imgs.append((qs.des, qs.kp, qs.shape))
    res = {}
    with _lib.Context(0) as c:
        c.set_keypoints(db.kp, db.img, db.centroid, db.size)
        c.upload_db(db.des)
        for multi in ("0", "1"):
            c.set_option("select_multi", int(multi))
            des, kp_, shape = imgs[0]
            c.upload_queries(des, kp_)
            c.pipeline(shape, bins)
            one = (c.valid_result(), c.affine_result())
            batch = sod.run_query_batch(c, imgs[1:], bins=bins, fused=True)   # 1700 queries
            res[multi] = (one, batch)
    (one0, b0), (one1, b1) = res["0"], res["1"]
    for x, y in ((one0[0], one1[0]),) + tuple((p["valid"], q["valid"]) for p, q in zip(b0, b1)):
        assert len(x["keys"]) > 0
        for k in ("keys", "votes", "offsets", "members"):
            assert np.array_equal(x[k], y[k]), k
        np.testing.assert_array_equal(x["means"], y["means"])
    for x, y in ((one0[1], one1[1]),) + tuple((p["affine"], q["affine"]) for p, q in zip(b0, b1)):
        assert np.array_equal(x["survived"], y["survived"])
        np.testing.assert_array_equal(x["params"], y["params"])
    # oracle leg for the one-work-group results
    des, kp_, shape = imgs[0]
    dbkp, qkp, images = oracle_inputs(db, kp_)
    o = orc.run_pipeline(des, qkp, db.des, dbkp, images, bins, shape)
    assert_stages_equal_oracle(one0[0], one0[1], o["table"], o["valid"], o["affine"])
    for (des, kp_, shape), b in zip(imgs[1:], b0):
        dbkp, qkp, images = oracle_inputs(db, kp_)
        o = orc.run_pipeline(des, qkp, db.des, dbkp, images, bins, shape)
        assert_stages_equal_oracle(b["valid"], b["affine"], o["table"], o["valid"], o["affine"])


def _threshold_members(n, seed):
    """Members whose outlier test (AffineParameters.py:145-158) sits exactly on the x
    tolerance under numpy's rounding of np.matmul(M, X) and one ulp past it under the
    other rounding: tx chosen so that np.matmul(M, X)[0] + tx - u == x_ref exactly."""
    rng = np.random.default_rng(seed)
    prm, pts = [], []
    while len(pts) < n:
        m = rng.uniform(-1.5, 1.5, 4)
        x, y = float(np.float32(rng.uniform(0, 1500))), float(np.float32(rng.uniform(0, 1000)))
        u, v = float(np.float32(rng.uniform(0, 1500))), float(np.float32(rng.uniform(0, 1000)))
        r = np.matmul([[m[0], m[1]], [m[2], m[3]]], [x, y])
        plain = m[0] * x + m[1] * y
        if r[0] == plain:
            continue                     # this member does not tell the roundings apart
        x_ref = 16.0                      # query width 2048, i_sigma 1, x_factor 128
        tx = u + x_ref - r[0]
        if (r[0] + tx) - u != x_ref:
            continue
        if ((plain + tx) - u > x_ref) == ((r[0] + tx) - u > x_ref):
            continue
        ty = v - r[1]                     # v well inside its tolerance
        prm.append([m[0], m[1], m[2], m[3], tx, ty])
        pts.append((x, y, u, v))
    return np.array(prm), np.array(pts)


def test_outlier_test_rounding_follows_numpy():
    """remove_outliers' np.matmul(M, X) (AffineParameters.py:145) is evaluated with this
    host's numpy rounding (option affine_fma, probed by the Python layer): members placed
    exactly on the x tolerance under that rounding -- and one ulp off it under the other --
    get the reference's keep / drop decision, bin by bin (one member per bin, params
    given: one remove_outliers round, sod_affine_batch max_iter 1)."""
    prm, pts = _threshold_members(64, 7)
    n = len(prm)
    with _lib.Context(0) as c:
        fma = c.get_option("affine_fma")
        assert fma == _lib.numpy_matmul_fma()
        r = c.affine_batch(np.arange(n + 1), pts[:, 0], pts[:, 1], pts[:, 2], pts[:, 3],
                           np.ones(n, np.int32), (2048, 2048), 128.0, 128.0, threshold=0,
                           max_iter=1, params_in=prm)
        ref = [orc.remove_outliers(p, [(q[0], q[1])], [(q[2], q[3])], 1, (2048, 2048),
                                   128.0, 128.0)[0][0] for p, q in zip(prm, pts)]
        assert np.array_equal(r["alive"], np.array(ref)), (fma, int((r["alive"] != ref).sum()))
        c.set_option("affine_fma", 0 if fma else 1)   # the other rounding disagrees on every member
        r2 = c.affine_batch(np.arange(n + 1), pts[:, 0], pts[:, 1], pts[:, 2], pts[:, 3],
                            np.ones(n, np.int32), (2048, 2048), 128.0, 128.0, threshold=0,
                            max_iter=1, params_in=prm)
        assert not np.any(r2["alive"] == np.array(ref))


def test_set_option_validation(ctx):
    """option values outside the int range are refused (not wrapped: 2^32-2 would
    become -2, a 'default' sentinel); trig_exact takes -1 / 0 / 1, and 1 only when the host
    libm probe agrees; debug_sync is counted per context (one context turning it off leaves
    another's on)."""
    for v in (2 ** 32 - 2, -(2 ** 31) - 1, 2 ** 40):
        with pytest.raises(_lib.SodError):
            ctx.set_option("sift_sort_max", v)
    assert ctx.get_option("sift_sort_max") == -2
    with pytest.raises(_lib.SodError):
        ctx.set_option("trig_exact", 2)
    ctx.set_option("trig_exact", 0)
    assert not ctx.trig_exact()
    ctx.set_option("trig_exact", -1)
    if ctx.trig_exact():
        ctx.set_option("trig_exact", 1)
        assert ctx.trig_exact()
    else:
        with pytest.raises(_lib.SodError):
            ctx.set_option("trig_exact", 1)
    with pytest.raises(_lib.SodError):            # the streamed kernel was removed (round 6)
        ctx.set_match_kernel(2)
    with _lib.Context(0) as other:
        other.set_option("debug_sync", 1)
        ctx.set_option("debug_sync", 0)
        assert other.get_option("debug_sync") == 1


@pytest.mark.parametrize("case", ["no_good_matches", "no_valid_bins", "one_query"])
def test_main_run_empty_stages(case):
    """Main.run (the staged one-transfer read, main.py's sequence in one enqueue) on edge
    sizes: nothing passes the ratio test, no bin reaches the vote threshold, one query -- the
    results equal the stage-by-stage getters' and the final pose list is empty when nothing
    survives."""
    nq = 1 if case == "one_query" else 600
    db = synthetic.make_database(3, 400, seed=41)
    qs = synthetic.make_queries(nq, seed=42, db_seed=41, kp_per_image=400, planted_frac=0.6,
                                n_objects=1)
    ratio = 0.0 if case == "no_good_matches" else 0.75
    vthr = 10 ** 6 if case == "no_valid_bins" else 5
    m = sod.Main()
    m.set_database(sod.SiftDatabase(db.des, db.kp, db.img, db.centroid, db.size))
    m.get_query_features(qs.des, qs.kp, qs.shape)
    out = m.run(15, vote_threshold=vthr, affine_threshold=4, ratio=ratio)
    c = m.ctx
    idx1, d1, d2, good = c.match_result()
    assert np.array_equal(out["idx1"], idx1) and np.array_equal(out["good"], good)
    v = c.valid_result()
    for k in ("keys", "votes", "offsets", "members"):
        assert np.array_equal(out["valid"][k], v[k]), k
    a = c.affine_result()
    assert np.array_equal(out["affine"]["survived"], a["survived"])
    if case == "no_good_matches":
        assert not good.any()
    if case in ("no_good_matches", "no_valid_bins"):
        assert len(out["valid"]["keys"]) == 0 and m.final_pose == []
    assert len(m.final_pose) == len(out["post"]["final_pose"])
