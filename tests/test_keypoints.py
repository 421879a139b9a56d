"""The drop-in's KeyPoint objects are the reference's: every field of
cv2.KeyPoint -- pt, size, angle, response, octave, class_id -- survives the flat database
(``from_records`` of the reference's pickle records, ``from_cv``, ``save / load``), and the
caller's own objects are handed back where they were given (main.py:43,65,85-86).
CPU only: the golden kpfields_* fixtures (made by the reference's own Main stages,
tests/golden/make_golden.py keypoints) are checked against their inputs here; the device
path is compared with them in test_gpu_api.py::test_main_keypoint_fields."""
import numpy as np
import pytest

from conftest import golden
from sift_based_od_amd import KeyPoint, make_kp, make_temp_kp
from sift_based_od_amd.database import Keypoints, SiftDatabase

ROW = ("x", "y", "size", "angle", "response", "octave", "class_id")


def rows_of(g, kf, pre, idx):
    return np.stack([np.asarray((g if f in ("x", "y", "angle", "octave") else kf)[pre + f],
                                np.float64)[idx] for f in ROW], 1)


@pytest.mark.parametrize("name", ["c1_b15", "planted_b15"])
def test_golden_keypoint_fields_pin_inputs(name):
    """matching_keypoints = (kp[trainIdx], kp_query[queryIdx], ...) for the good matches in
    query order; the bins' keypoint_pairs are those of their members, every field intact."""
    g, kf = golden(name), golden("kpfields_" + name)
    q = np.nonzero(g["good"])[0]
    assert np.array_equal(kf["mk_q"], q)
    assert np.array_equal(kf["mk_model"], rows_of(g, kf, "db_", g["idx1"][q]))
    assert np.array_equal(kf["mk_query"], rows_of(g, kf, "q_", q))
    im = g["db_img"][g["idx1"][q]]
    assert np.array_equal(kf["mk_img_size"], g["size"][im])
    assert np.array_equal(kf["mk_centroid"], g["centroid"][im])
    for tag in ("valid", "surv"):
        mem = g[tag + "_members"]
        assert np.array_equal(kf[tag + "_off"], g[tag + "_off"])
        assert np.array_equal(kf[tag + "_pairs_query"], rows_of(g, kf, "q_", mem))
        assert np.array_equal(kf[tag + "_pairs_model"], rows_of(g, kf, "db_", g["idx1"][mem]))


def _fields(k):
    return (k.pt, k.size, k.angle, k.response, k.octave, k.class_id)


def test_records_save_load_keep_every_field(tmp_path):
    rng = np.random.default_rng(3)
    kps = [KeyPoint(float(x), float(y), float(s), float(a), float(r), int(o), int(c))
           for x, y, s, a, r, o, c in zip(rng.uniform(0, 900, 50), rng.uniform(0, 700, 50),
                                          rng.uniform(1, 30, 50), rng.uniform(0, 360, 50),
                                          rng.uniform(0, 0.1, 50), rng.integers(0, 4, 50) | 256,
                                          rng.integers(-1, 9, 50))]
    recs = [[make_temp_kp(kps[:20]), rng.integers(0, 256, (20, 128)), (900, 700), (1.0, 2.0), "a"],
            [make_temp_kp(kps[20:]), rng.integers(0, 256, (30, 128)), (800, 600), (3.0, 4.0), "b"]]
    ref = make_kp(make_temp_kp(kps))            # main.py:65's objects
    db = SiftDatabase.from_records(recs)
    assert [_fields(db.kp.keypoint(i)) for i in range(50)] == [_fields(k) for k in ref]
    db.save(tmp_path / "db.npz")
    back = SiftDatabase.load(tmp_path / "db.npz")
    assert [_fields(back.kp.keypoint(i)) for i in range(50)] == [_fields(k) for k in ref]
    # a file written before the extra fields existed loads with cv2.KeyPoint's defaults
    with np.load(tmp_path / "db.npz", allow_pickle=False) as z:
        old = {k: z[k] for k in z.files if not k.startswith("kp_")}
    np.savez(tmp_path / "old.npz", **old)
    k0 = SiftDatabase.load(tmp_path / "old.npz").kp.keypoint(0)
    assert (k0.size, k0.response, k0.class_id) == (0.0, 0.0, -1)


def test_from_cv_hands_back_the_callers_objects():
    kps = [KeyPoint(1.5, 2.5, 7.0, 33.0, 0.03, 0x101, 4), KeyPoint(3.0, 4.0, 2.0, 9.0, 0.5, 2, -1)]
    t = Keypoints.from_cv(kps)
    assert t.keypoint(0) is kps[0] and t.keypoint(1) is kps[1]
    assert t.size.tolist() == [7.0, 2.0] and t.class_id.tolist() == [4, -1]
    assert t.slice(1, 2).keypoint(0) is kps[1]
    c = Keypoints.concat([t, t.slice(0, 1)])
    assert c.keypoint(2) is kps[0] and len(c) == 3
    # without objects: new ones with every field
    bare = Keypoints(t.x, t.y, t.angle, t.octave, t.size, t.response, t.class_id)
    assert _fields(bare.keypoint(0)) == _fields(kps[0])


def test_posebins_from_device_equal_two_call_construction():
    """hough.posebins_from_device builds each bin's attributes in one dict; it must give the
    same object as PoseBin(...) followed by bind_device(...) (CPU only: a synthetic
    selection)."""
    from sift_based_od_amd.hough import posebins_from_device
    from sift_based_od_amd.posebin import PoseBin
    rng = np.random.default_rng(3)
    V = 40
    votes = rng.integers(1, 6, V).astype(np.int32)
    votes[:3] = 1
    off = np.concatenate([[0], np.cumsum(votes)]).astype(np.int64)
    res = {"keys": rng.integers(0, 32, (V, 4)).astype(np.int32), "votes": votes,
           "offsets": off, "members": rng.integers(0, 900, off[-1]).astype(np.int32),
           "means": rng.random((V, 6))}

    def pair_of(q):
        return ("m%d" % q, "q%d" % q)

    def size_of(q):
        return (640 + q % 3, 480)

    got = posebins_from_device(res, pair_of, size_of, token=9)
    for i, b in enumerate(got):
        m = res["members"][off[i]:off[i + 1]]
        mu = res["means"][i]
        size = size_of(int(m[0])) if votes[i] == 1 else (float(mu[4]), float(mu[5]))
        ref = PoseBin(tuple(int(v) for v in res["keys"][i]), size, int(votes[i]), None,
                      tuple(float(v) for v in mu[:4]))
        ref.bind_device(9, i, m, pair_of)
        assert sorted(b.__dict__) == sorted(ref.__dict__)
        for k, v in ref.__dict__.items():
            w = b.__dict__[k]
            if k in ("_lazy", "_dev"):
                assert len(v) == len(w) and all(
                    (x is y) or np.array_equal(x, y) if isinstance(x, np.ndarray) else x == y
                    for x, y in zip(v, w)), k
            else:
                assert type(w) is type(v) and w == v, k
        assert b.device_index(9) == i and b.keypoint_pairs == ref.keypoint_pairs
        assert type(b.votes) is int and all(type(x) is float for x in b.centroid)
