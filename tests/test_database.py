"""SURVEY 8(f) row 2 / A3 on the CPU: the flat database built from the reference's pickle
payload (``GenerateDatabaseInfo.py:35`` records) equals the oracle's restatement of
``main.py:50-66`` row for row -- trainIdx order, keypoint fields as cv2.KeyPoint stores them
(float32), each row's model image size and centroid, descriptors -- and survives the on-disk
format (``SiftDatabase.save/load``, no pickle)."""
import numpy as np

from oracle import oracle as orc
from sift_based_od_amd.database import SiftDatabase, centroid_of


def _records(seed=0, n_images=5):
    """Records shaped like the reference's pickle: temp_kp tuples (pt, size, angle,
    response, octave, class_id) with Python floats, float32 descriptors, (w, h), centroid
    (get_centroid: sequential sum of the pt values), path."""
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n_images):
        n = int(rng.integers(1, 40)) if i != 2 else 1          # a one-keypoint image too
        w, h = 1500, int(rng.integers(800, 1201))
        x = rng.uniform(0, w, n)                                # float64: KeyPoint rounds
        y = rng.uniform(0, h, n)
        ang = rng.uniform(0, 360, n)
        octv = rng.integers(-1, 4, n) & 0xFF | (rng.integers(1, 4, n) << 8)
        temp_kp = [((float(np.float32(a)), float(np.float32(b))), 3.5, float(c), 0.01, int(o), -1)
                   for a, b, c, o in zip(x, y, ang, octv)]
        des = rng.integers(0, 256, (n, 128)).astype(np.float32)
        cx = cy = 0.0
        for t in temp_kp:                                       # get_centroid's loop
            cx += t[0][0]
            cy += t[0][1]
        recs.append([temp_kp, des, (w, h), (cx / n, cy / n), "img%d.png" % i])
    return recs


def test_from_records_equals_reference_flattening(tmp_path):
    recs = _records()
    ref = orc.flatten_records(recs)
    db = SiftDatabase.from_records(recs)
    n = len(ref["x"])
    assert len(db) == n
    assert np.array_equal(db.kp.x, np.array(ref["x"], np.float32))
    assert np.array_equal(db.kp.y, np.array(ref["y"], np.float32))
    assert np.array_equal(db.kp.angle, np.array(ref["angle"], np.float32))
    assert np.array_equal(db.kp.octave, np.array(ref["octave"], np.int32))
    assert np.array_equal(np.asarray(db.des, np.float32), ref["des"])
    for i in range(n):                                          # per-row image tables
        im = db.img[i]
        assert tuple(int(v) for v in db.size[im]) == tuple(ref["img_size"][i])
        assert tuple(float(v) for v in db.centroid[im]) == tuple(ref["centroid"][i])
    # get_centroid of the rows equals the stored centroid (centroid_of: sequential sum)
    for im in range(db.n_images):
        rows = db.img == im
        assert centroid_of(db.kp.x[rows], db.kp.y[rows]) == tuple(db.centroid[im])
    # on-disk format round trip (numpy, allow_pickle=False)
    path = tmp_path / "db.npz"
    db.save(path)
    back = SiftDatabase.load(path)
    for a, b in ((db.kp.x, back.kp.x), (db.kp.octave, back.kp.octave), (db.img, back.img),
                 (db.centroid, back.centroid), (db.size, back.size)):
        assert np.array_equal(a, b)
    assert np.array_equal(np.asarray(db.des, np.uint8), back.des)
