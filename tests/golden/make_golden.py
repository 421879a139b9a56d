"""Generate the committed golden fixtures by running the REFERENCE'S OWN Python
code (build container only; ``/root/reference`` does not exist on the GPU box).

    python tests/golden/make_golden.py

The reference modules import ``cv2`` (OpenCV, absent here), so a stub module
providing only ``cv2.KeyPoint`` is injected (the hot-path modules touch nothing
else of cv2 at import or in the stages used: ``SiftHelperFunctions.py:47``).
``Main()`` needs matplotlib (present; Agg backend).  Inputs are seeded synthetic
workloads; matches are produced by the oracle's exact brute-force matcher
(OpenCV's matcher is not available -- see oracle/oracle.py header) and fed to
``Main.matching_keypoints`` in the reference's tuple format
(``main.py:85-86``).  The reference stages then run unchanged:
``apply_hough_transform`` -> ``get_valid_bins`` -> ``apply_affine_parameters``
(-> ``post_process``), and their outputs are stored as plain arrays (.npz,
no pickles).

Only data is written: inputs and the reference's outputs.
"""
import math
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)


class KeyPoint:
    """Stand-in for cv2.KeyPoint: pt/size/angle/response are float32 fields in
    OpenCV (cv::Point2f, float), octave/class_id ints."""

    def __init__(self, x=0.0, y=0.0, _size=0.0, _angle=-1.0, _response=0.0,
                 _octave=0, _class_id=-1):
        self.pt = (float(np.float32(x)), float(np.float32(y)))
        self.size = float(np.float32(_size))
        self.angle = float(np.float32(_angle))
        self.response = float(np.float32(_response))
        self.octave = int(_octave)
        self.class_id = int(_class_id)


def import_reference():
    import matplotlib
    matplotlib.use("Agg")
    cv2 = types.ModuleType("cv2")
    cv2.KeyPoint = KeyPoint
    sys.modules["cv2"] = cv2
    sys.path.insert(0, REF)
    import main as ref_main  # noqa: E402
    import HoughTransformHelperFunctions as ref_ht  # noqa: E402
    return ref_main, ref_ht


def kp_objects(kp):
    return [KeyPoint(x=float(kp.x[i]), y=float(kp.y[i]), _size=2.0,
                     _angle=float(kp.angle[i]), _octave=int(kp.octave[i]))
            for i in range(len(kp))]


def run_reference(ref_main, qkp, dbkp, db_img, centroid, size, matches, shape, bins,
                  vote_thr=5, affine_thr=4, post=True):
    """Drive the reference stages on a given match list [(q, m), ...]."""
    M = ref_main.Main()
    M.rgb_query = types.SimpleNamespace(shape=tuple(shape))
    M.image_query_size = (shape[1], shape[0])        # main.py:45 (width, height)
    kq = kp_objects(qkp)
    km = kp_objects(dbkp)
    ident = {}
    for q, m in matches:
        im = int(db_img[m])
        tup = (km[m], kq[q], (int(size[im][0]), int(size[im][1])),
               (float(centroid[im][0]), float(centroid[im][1])))
        M.matching_keypoints.append(tup)
        ident[(id(km[m]), id(kq[q]))] = (q, m)

    M.apply_hough_transform(bins)
    keys = list(M.hough_transform.keys())
    table_keys = np.array(keys, np.int32).reshape(-1, 4)
    table_votes = np.array([M.hough_transform[k].votes for k in keys], np.int32)

    M.get_valid_bins(vote_thr)
    vb = M.valid_bins
    v_keys = np.array([b.pose for b in vb], np.int32).reshape(-1, 4)
    v_votes = np.array([b.votes for b in vb], np.int32)
    v_off = np.zeros(len(vb) + 1, np.int64)
    v_mem = []
    for i, b in enumerate(vb):
        mem = [ident[(id(p[0]), id(p[1]))][0] for p in b.keypoint_pairs]
        v_mem.extend(mem)
        v_off[i + 1] = len(v_mem)
    v_means = np.array([[b.centroid[0], b.centroid[1], b.angle, b.scale,
                         float(b.img_size[0]), float(b.img_size[1])] for b in vb],
                       np.float64).reshape(-1, 6)

    pre_poses = [b.pose for b in vb]
    M.apply_affine_parameters(affine_thr)
    sv = M.valid_bins
    s_keys = np.array([b.pose for b in sv], np.int32).reshape(-1, 4)
    s_index = np.array([pre_poses.index(b.pose) for b in sv], np.int32)
    s_votes = np.array([b.votes for b in sv], np.int32)
    s_params = np.array([list(map(float, b.affine_parameters)) for b in sv],
                        np.float64).reshape(-1, 6)
    s_off = np.zeros(len(sv) + 1, np.int64)
    s_mem = []
    for i, b in enumerate(sv):
        s_mem.extend(ident[(id(p[0]), id(p[1]))][0] for p in b.keypoint_pairs)
        s_off[i + 1] = len(s_mem)
    out = dict(table_keys=table_keys, table_votes=table_votes,
               valid_keys=v_keys, valid_votes=v_votes, valid_off=v_off,
               valid_members=np.array(v_mem, np.int32), valid_means=v_means,
               surv_keys=s_keys, surv_index=s_index, surv_votes=s_votes,
               surv_params=s_params, surv_off=s_off,
               surv_members=np.array(s_mem, np.int32))
    if post:
        try:
            M.post_process()
            fp = M.final_pose
            out["final_pose"] = np.array(
                [[p[0][0], p[0][1], p[1], p[2], float(p[3][0]), float(p[3][1])] for p in fp],
                np.float64).reshape(-1, 6)
        except Exception as e:  # post-processing is out of scope; record only
            print("post_process failed:", e)
    return out


def pose_sweep(ref_ht, rng, n, bins_list, shape):
    """Per-element golden vectors for estimate_object_pose/calculate_bin_index."""
    mx = rng.uniform(-50, 1600, n).astype(np.float32)
    my = rng.uniform(-50, 1300, n).astype(np.float32)
    qx = rng.uniform(-100, 1100, n).astype(np.float32)
    qy = rng.uniform(-100, 900, n).astype(np.float32)
    ma = rng.uniform(0, 360, n).astype(np.float32)
    qa = rng.uniform(0, 360, n).astype(np.float32)
    # exact-angle edge cases: equal angles, 0/360-ish, theta near bin edges
    ma[:64] = qa[:64]
    qa[64:96] = 0.0
    ma[64:96] = np.float32(359.99997)
    moct = rng.integers(-1, 8, n)
    qoct = rng.integers(-1, 8, n)
    moct[:200] = rng.integers(-128, 127, 200)
    qoct[:200] = rng.integers(-128, 127, 200)
    mlay = rng.integers(0, 4, n)
    qlay = rng.integers(0, 4, n)
    mo = ((moct & 0xFF) | (mlay << 8)).astype(np.int32)
    qo = ((qoct & 0xFF) | (qlay << 8)).astype(np.int32)
    cx = rng.uniform(0, 1500, n)
    cy = rng.uniform(0, 1200, n)
    poses = np.zeros((n, 4), np.float64)
    idx = np.zeros((len(bins_list), n, 4), np.int32)
    for i in range(n):
        kM = KeyPoint(x=mx[i], y=my[i], _angle=ma[i], _octave=int(mo[i]))
        kQ = KeyPoint(x=qx[i], y=qy[i], _angle=qa[i], _octave=int(qo[i]))
        p = ref_ht.estimate_object_pose((kM, kQ, (1500, 1000), (cx[i], cy[i])))
        poses[i] = p
        for j, b in enumerate(bins_list):
            idx[j, i] = ref_ht.calculate_bin_index(p, b, shape)
    return dict(mx=mx, my=my, ma=ma, mo=mo, qx=qx, qy=qy, qa=qa, qo=qo, cx=cx, cy=cy,
                poses=poses, idx=idx, bins=np.array(bins_list, np.int32),
                shape=np.array(shape, np.int32))


def _near_edge_inputs(rng, n, bins, shape, ulps):
    """Inputs whose pose (x, y) lands within a few ulps of a bin edge on BOTH axes: the
    model centroid (an f64 input, main.py:66) is solved so that R(alpha) t + q = (X, Y) with
    X = nx W / b, Y = ny H / b, then nudged by `ulps` ulps -- the bin index of such a pose
    depends on the last bit of cos / sin (HTHF:31-35,49-58)."""
    H, W = shape[0], shape[1]
    b = np.asarray(bins)
    mx = rng.uniform(0, 1500, n).astype(np.float32)
    my = rng.uniform(0, 1000, n).astype(np.float32)
    ma = rng.uniform(0, 360, n).astype(np.float32)
    qa = rng.uniform(0, 360, n).astype(np.float32)
    qx = rng.uniform(0, W, n).astype(np.float32)
    qy = rng.uniform(0, H, n).astype(np.float32)
    moct = rng.integers(-1, 3, n)
    qoct = moct + rng.integers(0, 2, n)
    mo = ((moct & 0xFF) | (1 << 8)).astype(np.int32)
    qo = ((qoct & 0xFF) | (2 << 8)).astype(np.int32)
    nx = rng.integers(2, b + 1)
    ny = rng.integers(2, b + 1)
    cx = np.zeros(n)
    cy = np.zeros(n)
    for i in range(n):
        s = 2.0 ** (int(qoct[i]) - int(moct[i]))
        a = math.radians(float(qa[i]) - float(ma[i]))
        a = (a + 2 * math.pi) % (2 * math.pi)
        ca, sa = math.cos(a), math.sin(a)
        X, Y = nx[i] * W / int(b[i]), ny[i] * H / int(b[i])
        dx, dy = X - float(qx[i]), Y - float(qy[i])
        tx, ty = ca * dx + sa * dy, -sa * dx + ca * dy
        cx[i] = tx / s + float(mx[i])
        cy[i] = ty / s + float(my[i])
        for _ in range(abs(int(ulps[i]))):
            cx[i] = np.nextafter(cx[i], np.inf if ulps[i] > 0 else -np.inf)
            cy[i] = np.nextafter(cy[i], np.inf if ulps[i] < 0 else -np.inf)
    return mx, my, ma, mo, qx, qy, qa, qo, cx, cy


def near_edge_sweep(ref_ht, rng, n, bins_list, shape):
    """pose_sweep's layout for poses within a few ulps of an x AND a y bin edge, outputs
    from the reference's own estimate_object_pose / calculate_bin_index."""
    out = {}
    for j, b in enumerate(bins_list):
        ulps = rng.integers(-6, 7, n)
        mx, my, ma, mo, qx, qy, qa, qo, cx, cy = _near_edge_inputs(
            rng, n, np.full(n, b), shape, ulps)
        poses = np.zeros((n, 4), np.float64)
        idx = np.zeros((n, 4), np.int32)
        for i in range(n):
            kM = KeyPoint(x=mx[i], y=my[i], _angle=ma[i], _octave=int(mo[i]))
            kQ = KeyPoint(x=qx[i], y=qy[i], _angle=qa[i], _octave=int(qo[i]))
            p = ref_ht.estimate_object_pose((kM, kQ, (1500, 1000), (cx[i], cy[i])))
            poses[i] = p
            idx[i] = ref_ht.calculate_bin_index(p, b, shape)
        for k, v in dict(mx=mx, my=my, ma=ma, mo=mo, qx=qx, qy=qy, qa=qa, qo=qo, cx=cx, cy=cy,
                         poses=poses, idx=idx).items():
            out["b%d_%s" % (b, k)] = v
    out["bins"] = np.array(bins_list, np.int32)
    out["shape"] = np.array(shape, np.int32)
    return out


def near_edge_case(rng, groups, per_group, bins, shape):
    """Matches whose poses straddle bin edges: groups of `per_group` matches aimed at one
    (x, y) edge with one rotation / octave pair each, nudged -k..+k ulps, so a group's votes
    split across neighbouring bins exactly where cos / sin's last bit decides.  Every DB
    keypoint is its own model image (its centroid is the solved input)."""
    from sift_based_od_amd.database import Keypoints
    n = groups * per_group
    g = np.repeat(np.arange(groups), per_group)
    ulps = np.tile(np.arange(per_group) - per_group // 2, groups)
    H, W = shape[0], shape[1]
    mx = rng.uniform(0, 1500, n).astype(np.float32)
    my = rng.uniform(0, 1000, n).astype(np.float32)
    ma = rng.uniform(0, 360, n).astype(np.float32)
    qa = ((ma.astype(np.float64) + rng.uniform(0, 360, groups)[g]) % 360.0).astype(np.float32)
    qx = rng.uniform(0, W, n).astype(np.float32)
    qy = rng.uniform(0, H, n).astype(np.float32)
    moct = rng.integers(-1, 3, groups)[g]
    qoct = moct + rng.integers(0, 2, groups)[g]
    mo = ((moct & 0xFF) | (1 << 8)).astype(np.int32)
    qo = ((qoct & 0xFF) | (2 << 8)).astype(np.int32)
    mx, my, ma, mo, qx, qy, qa, qo, cx, cy = _resolve_group(rng, mx, my, ma, mo, qx, qy, qa, qo,
                                                            g, ulps, bins, shape)
    qkp = Keypoints(qx, qy, qa, qo)
    dbkp = Keypoints(mx, my, ma, mo)
    img = np.arange(n, dtype=np.int32)
    cen = np.stack([cx, cy], 1)
    size = np.tile(np.array([[1500, 1000]], np.int32), (n, 1))
    matches = [(i, i) for i in range(n)]
    return qkp, dbkp, img, cen, size, matches


def _resolve_group(rng, mx, my, ma, mo, qx, qy, qa, qo, g, ulps, bins, shape):
    """Re-solve every match's centroid for its group's shared edge (nx, ny) after the
    group's angles / octaves were unified."""
    H, W = shape[0], shape[1]
    groups = int(g.max()) + 1
    nx = rng.integers(2, bins + 1, groups)
    ny = rng.integers(2, bins + 1, groups)
    n = len(mx)
    cx = np.zeros(n)
    cy = np.zeros(n)
    for i in range(n):
        om = int(mo[i] & 0xFF); om = om - 256 if om >= 128 else om
        oq = int(qo[i] & 0xFF); oq = oq - 256 if oq >= 128 else oq
        s = 2.0 ** (oq - om)
        a = math.radians(float(qa[i]) - float(ma[i]))
        a = (a + 2 * math.pi) % (2 * math.pi)
        ca, sa = math.cos(a), math.sin(a)
        X, Y = nx[g[i]] * W / bins, ny[g[i]] * H / bins
        dx, dy = X - float(qx[i]), Y - float(qy[i])
        tx, ty = ca * dx + sa * dy, -sa * dx + ca * dy
        cx[i] = tx / s + float(mx[i])
        cy[i] = ty / s + float(my[i])
        for _ in range(abs(int(ulps[i]))):
            cx[i] = np.nextafter(cx[i], np.inf if ulps[i] > 0 else -np.inf)
            cy[i] = np.nextafter(cy[i], np.inf if ulps[i] < 0 else -np.inf)
    return mx, my, ma, mo, qx, qy, qa, qo, cx, cy


def edge_case(rng):
    """Hand-shaped matches: a tight planted cluster with outliers, a cluster of
    queries all matched to ONE model keypoint (rank-deficient A^T A), a cluster
    whose scale bin is 0 (zero outlier tolerance), off-image poses and theta
    near 2*pi."""
    from sift_based_od_amd.database import Keypoints
    nimg = 2
    size = np.array([[1500, 1000], [1500, 900]], np.int32)
    nm = 400
    mx = rng.uniform(0, 1500, nm).astype(np.float32)
    my = rng.uniform(0, 900, nm).astype(np.float32)
    ma = rng.uniform(0, 360, nm).astype(np.float32)
    mo = np.zeros(nm, np.int32) | (1 << 8)
    img = (np.arange(nm) >= 200).astype(np.int32)
    cen = np.array([[float(np.cumsum(mx[:200].astype(np.float64))[-1]) / 200,
                     float(np.cumsum(my[:200].astype(np.float64))[-1]) / 200],
                    [float(np.cumsum(mx[200:].astype(np.float64))[-1]) / 200,
                     float(np.cumsum(my[200:].astype(np.float64))[-1]) / 200]])
    qx, qy, qa, qo, mlist = [], [], [], [], []

    def add(m, x, y, a, o):
        mlist.append(m); qx.append(x); qy.append(y); qa.append(a); qo.append(o)

    # (1) planted similarity cluster, scale 2 (octave +1), theta 30deg, + outliers
    th = math.radians(30.0)
    for m in range(0, 60):
        dx, dy = float(mx[m]) - cen[0, 0], float(my[m]) - cen[0, 1]
        add(m, 500 + 2 * (math.cos(th) * dx - math.sin(th) * dy) + rng.normal(0, 0.5),
            400 + 2 * (math.sin(th) * dx + math.cos(th) * dy) + rng.normal(0, 0.5),
            (float(ma[m]) + 30.0) % 360.0, 2 | (1 << 8))
    for m in range(60, 70):   # gross outliers inside the same pose bin
        dx, dy = float(mx[m]) - cen[0, 0], float(my[m]) - cen[0, 1]
        add(m, 500 + 2 * (math.cos(th) * dx - math.sin(th) * dy) + rng.normal(0, 40),
            400 + 2 * (math.sin(th) * dx + math.cos(th) * dy) + rng.normal(0, 40),
            (float(ma[m]) + 30.0) % 360.0, 2 | (1 << 8))
    # (2) twelve queries all matched to model keypoint 210 (same model point)
    for j in range(12):
        add(210, 300 + rng.normal(0, 0.3), 200 + rng.normal(0, 0.3),
            (float(ma[210]) + 359.9) % 360.0, 1 | (2 << 8))
    # (3) scale bin 0 cluster: query octave <= model octave
    for m in range(220, 250):
        dx, dy = float(mx[m]) - cen[1, 0], float(my[m]) - cen[1, 1]
        add(m, 700 + 0.5 * dx, 300 + 0.5 * dy, float(ma[m]), 0xFF)
    # (4) off-image poses (negative / beyond width) and theta wrap
    for m in range(250, 280):
        add(m, float(rng.uniform(-400, 0)), float(rng.uniform(1000, 1500)),
            float(rng.uniform(0, 360)), int(rng.integers(0, 4)))
    n = len(mlist)
    qkp = Keypoints(np.array(qx, np.float32), np.array(qy, np.float32),
                    np.array(qa, np.float32), np.array(qo, np.int32))
    dbkp = Keypoints(mx, my, ma, mo)
    matches = [(i, mlist[i]) for i in range(n)]
    return qkp, dbkp, img, cen, size, matches


def post_case(rng, n, n_centers, spread, ang_spread, field=(1000, 800)):
    """Synthetic PoseBin means (x, y, angle, scale, w, h) for the post-processing stage:
    positions around n_centers centres (spread in units of the w*s/4 threshold, so
    clusters chain, touch and separate), angles around per-centre values (spread in
    degrees around the 1 degree threshold), model sizes / scales like the DB's."""
    cx = rng.uniform(0, field[0], n_centers)
    cy = rng.uniform(0, field[1], n_centers)
    ca = rng.uniform(0, 2 * math.pi, n_centers)
    c = rng.integers(0, n_centers, n)
    s = 2.0 ** rng.integers(-1, 2, n) * rng.uniform(0.9, 1.1, n)
    w = rng.choice([1500.0, 1200.0, 900.0], n)
    h = rng.uniform(800, 1200, n)
    x = cx[c] + rng.normal(0, spread, n) * w * s / 4
    y = cy[c] + rng.normal(0, spread, n) * h * s / 4
    a = ca[c] + np.radians(rng.normal(0, ang_spread, n))
    return np.stack([x, y, a, s, w, h], 1)


def post_edge_case():
    """Exact threshold equalities, orientation-cluster size ties (the LAST largest wins),
    equal minimum areas (the FIRST wins), a singleton."""
    rows = [
        # x, y, angle, scale, w, h
        (100.0, 100.0, 1.0, 1.0, 1500.0, 1000.0),
        (475.0, 100.0, 1.0, 1.0, 1500.0, 1000.0),     # |dx| == 1500*1/4: close
        (850.0000000001, 100.0, 1.0, 1.0, 1500.0, 1000.0),   # just beyond 475 + 375
        (100.0, 350.0, 1.0 + math.radians(1.0), 1.0, 1500.0, 1000.0),  # |dy| == 250
        (100.0, 350.0, 1.0 + math.radians(2.5), 1.0, 1500.0, 1000.0),
        (100.0, 350.0, 1.0 + math.radians(2.5), 1.0, 1500.0, 1000.0),
        (3000.0, 3000.0, 0.5, 2.0, 900.0, 800.0),      # far away: own cluster
        (3000.0, 3000.0, 0.5 + math.radians(5.0), 2.0, 900.0, 800.0),
        (3000.0, 3000.0, 0.5 + math.radians(10.0), 1.0, 1800.0, 1600.0),  # equal area
        (9000.0, 9000.0, 0.0, 0.5, 1500.0, 800.0),     # singleton
    ]
    return np.array(rows, np.float64)


def run_post(ref_pp, ref_pb, means):
    bins = [ref_pb.PoseBin((0, 0, 0, 0), (float(r[4]), float(r[5])), 1, [],
                           (float(r[0]), float(r[1]), float(r[2]), float(r[3])))
            for r in means]
    ident = {id(b): i for i, b in enumerate(bins)}
    pc = ref_pp.group_position(bins)
    oc = ref_pp.group_orientation(pc)
    fo = ref_pp.find_max_orientation(oc)
    fp = ref_pp.get_final_pose(pc, fo)
    pos_off, pos_mem = [0], []
    for cl in pc:
        pos_mem.extend(ident[id(b)] for b in cl)
        pos_off.append(len(pos_mem))
    ori_pos_off, ori_off, ori_mem = [0], [0], []
    for clusters in oc:
        for comp in clusters:
            ori_mem.extend(ident[id(b)] for b in comp)
            ori_off.append(len(ori_mem))
        ori_pos_off.append(len(ori_off) - 1)
    return dict(means=means, pos_off=np.array(pos_off, np.int32),
                pos_members=np.array(pos_mem, np.int32),
                ori_pos_off=np.array(ori_pos_off, np.int32),
                ori_off=np.array(ori_off, np.int32), ori_members=np.array(ori_mem, np.int32),
                final_orientation=np.array(fo, np.float64),
                final_pose=np.array([[p[0][0], p[0][1], p[1], p[2], float(p[3][0]),
                                      float(p[3][1])] for p in fp], np.float64).reshape(-1, 6))


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, os.path.getsize(path), "bytes")


def kp_arrays(prefix, kp):
    return {prefix + "x": kp.x, prefix + "y": kp.y, prefix + "angle": kp.angle,
            prefix + "octave": kp.octave}


def main_near_edge():
    """Only the near-bin-edge fixtures (the boundary guard, hough.hip)."""
    import sod_pkg
    sod_pkg.load()
    ref_main, ref_ht = import_reference()
    shape = (800, 1000, 3)
    rng = np.random.default_rng(4321)
    save("near_edge_sweep", **near_edge_sweep(ref_ht, rng, 10000, [15, 32], shape))
    for bins in (15, 32):
        qkp, dbkp, img, cen, size, matches = near_edge_case(rng, 300, 13, bins, shape)
        out = run_reference(ref_main, qkp, dbkp, img, cen, size, matches, shape, bins)
        print("near_edge", bins, "bins", len(out["table_votes"]), "valid",
              len(out["valid_votes"]), "surv", len(out["surv_votes"]))
        save("near_edge_b%d" % bins, db_img=img, centroid=cen, size=size,
             shape=np.array(shape, np.int32), bins=np.int32(bins),
             match_q=np.array([q for q, _ in matches], np.int32),
             match_m=np.array([m for _, m in matches], np.int32),
             **kp_arrays("q_", qkp), **kp_arrays("db_", dbkp), **out)


def main():
    import sod_pkg
    sod_pkg.load()
    from sift_based_od_amd import synthetic
    from oracle import oracle as orc

    ref_main, ref_ht = import_reference()

    # ---- per-element pose / bin-index sweep (A4-A6) ----
    rng = np.random.default_rng(1234)
    sweep = pose_sweep(ref_ht, rng, 20000, [15, 12, 8, 32], (800, 1000, 3))
    save("pose_sweep", **sweep)

    # ---- end-to-end cases (A2, A7-A13) ----
    cases = [
        # name, n_images, kp/img, n_queries, planted, bins
        ("c1_b15", 2, 250, 500, 0.3, 15),
        ("planted_b15", 4, 500, 3000, 0.3, 15),
        ("planted_b12", 6, 400, 2500, 0.4, 12),
    ]
    for name, nimg, kpi, nq, pf, bins in cases:
        db = synthetic.make_database(nimg, kpi, seed=7)
        qs = synthetic.make_queries(nq, seed=8, db_seed=7, kp_per_image=kpi,
                                    planted_frac=pf, n_objects=min(4, nimg))
        idx1, d1, d2 = orc.knn2_match(qs.des, db.des)
        i2, e1, e2 = orc.knn2_match_int(qs.des, db.des)
        assert np.array_equal(idx1, i2) and np.array_equal(d1, e1) and np.array_equal(d2, e2)
        good = orc.ratio_test(d1, d2)
        matches = [(int(q), int(idx1[q])) for q in np.nonzero(good)[0]]
        out = run_reference(ref_main, qs.kp, db.kp, db.img, db.centroid, db.size,
                            matches, qs.shape, bins)
        print(name, "matches", len(matches), "bins", len(out["table_votes"]),
              "valid", len(out["valid_votes"]), "surv", len(out["surv_votes"]))
        save(name, q_des=qs.des, db_des=db.des, db_img=db.img, centroid=db.centroid,
             size=db.size, shape=np.array(qs.shape, np.int32), bins=np.int32(bins),
             idx1=idx1, d1=d1, d2=d2, good=good,
             **kp_arrays("q_", qs.kp), **kp_arrays("db_", db.kp), **out)

    # ---- hand-shaped Hough/affine edge case (matches given directly) ----
    qkp, dbkp, img, cen, size, matches = edge_case(np.random.default_rng(99))
    for bins in (15, 6):
        out = run_reference(ref_main, qkp, dbkp, img, cen, size, matches,
                            (1000, 1200, 3), bins)
        print("edge", bins, "bins", len(out["table_votes"]), "valid",
              len(out["valid_votes"]), "surv", len(out["surv_votes"]))
        save("edge_b%d" % bins, db_img=img, centroid=cen, size=size,
             shape=np.array((1000, 1200, 3), np.int32), bins=np.int32(bins),
             match_q=np.array([q for q, _ in matches], np.int32),
             match_m=np.array([m for _, m in matches], np.int32),
             **kp_arrays("q_", qkp), **kp_arrays("db_", dbkp), **out)

    # ---- post-processing (section 8(f) row 1): reference PostProcessing on PoseBins ----
    import PostProcessing as ref_pp  # noqa: E402
    import PoseBin as ref_pb  # noqa: E402
    prng = np.random.default_rng(77)
    post = {"post_edge": post_edge_case(),
            "post_small": post_case(prng, 40, 6, 1.0, 1.0),
            "post_medium": post_case(prng, 400, 25, 0.8, 0.8, (12000, 9000)),
            "post_chain": post_case(prng, 300, 3, 2.5, 2.0)}
    for name, means in post.items():
        out = run_post(ref_pp, ref_pb, means)
        print(name, "bins", len(means), "position clusters", len(out["final_pose"]),
              "orientation clusters", len(out["ori_off"]) - 1)
        save(name, **out)

    # ---- matcher edge cases (int64 brute force; OpenCV absent: unpinned) ----
    rng = np.random.default_rng(5)
    db = rng.integers(0, 256, (300, 128)).astype(np.uint8)
    db[150] = db[20]          # exact duplicate rows -> tie, lower index wins
    db[151] = db[20]
    q = rng.integers(0, 256, (200, 128)).astype(np.uint8)
    q[:10] = db[20]           # d1 == 0, tie between rows 20/150/151
    q[10:20] = db[:10]        # exact hits
    q[20] = 255               # extremes
    q[21] = 0
    i1, e1, e2 = orc.knn2_match_int(q, db)
    save("matcher_edges", q_des=q, db_des=db, idx1=i1, d1=e1, d2=e2,
         good=orc.ratio_test(e1, e2))


KP_FIELDS = ("x", "y", "size", "angle", "response", "octave", "class_id")


def kp_field_rows(kps):
    """[n, 7] f64 rows (pt x, pt y, size, angle, response, octave, class_id) of KeyPoints."""
    return np.array([[k.pt[0], k.pt[1], k.size, k.angle, k.response, k.octave, k.class_id]
                     for k in kps], np.float64).reshape(-1, 7)


def main_keypoints():
    """The reference's own KeyPoint objects through main.py's stages (the
    drop-in must hand back the reference's objects): for the c1_b15 and planted_b15 inputs
    plus seeded size / response / class_id fields, the DB goes through the reference's
    record format (``make_temp_kp`` tuples per image, main.py:53-66's flattening, ``make_kp``)
    and ``Main.run_matcher`` runs with a stand-in ``cv2.BFMatcher`` whose knnMatch is the
    oracle's exact k=2 (OpenCV is absent); ``matching_keypoints`` and the valid / surviving
    bins' ``keypoint_pairs`` are stored field by field (written to kpfields_<case>.npz)."""
    import sod_pkg
    sod_pkg.load()
    from oracle import oracle as orc
    ref_main, _ = import_reference()
    import SiftHelperFunctions as ref_sh  # noqa: E402

    class _DMatch:
        def __init__(self, q, t, d):
            self.queryIdx, self.trainIdx, self.imgIdx, self.distance = q, t, 0, d

    class _BFMatcher:
        def knnMatch(self, q, d, k=2):
            i1, e1, e2, i2 = orc.knn2_match(np.asarray(q), np.asarray(d), with_idx2=True)
            return [(_DMatch(j, int(i1[j]), float(e1[j])), _DMatch(j, int(i2[j]), float(e2[j])))
                    for j in range(len(i1))]
    sys.modules["cv2"].BFMatcher = _BFMatcher

    for name, seed in (("c1_b15", 601), ("planted_b15", 602)):
        g = dict(np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False))
        rng = np.random.default_rng(seed)
        nd, nq = len(g["db_x"]), len(g["q_x"])
        extra = {}
        for pre, n in (("db_", nd), ("q_", nq)):
            extra[pre + "size"] = rng.uniform(1.5, 40.0, n).astype(np.float32)
            extra[pre + "response"] = rng.uniform(0.005, 0.12, n).astype(np.float32)
            extra[pre + "class_id"] = rng.integers(-1, 6, n).astype(np.int32)

        def objs(pre, n):
            return [KeyPoint(x=float(g[pre + "x"][i]), y=float(g[pre + "y"][i]),
                             _size=float(extra[pre + "size"][i]), _angle=float(g[pre + "angle"][i]),
                             _response=float(extra[pre + "response"][i]),
                             _octave=int(g[pre + "octave"][i]),
                             _class_id=int(extra[pre + "class_id"][i])) for i in range(n)]
        dbk, qk = objs("db_", nd), objs("q_", nq)
        # the pickle's per-image records (GenerateDatabaseInfo.py:35) ...
        records = []
        for im in range(len(g["centroid"])):
            rows = np.nonzero(g["db_img"] == im)[0]
            records.append([ref_sh.make_temp_kp([dbk[r] for r in rows]), g["db_des"][rows],
                            (int(g["size"][im][0]), int(g["size"][im][1])),
                            (float(g["centroid"][im][0]), float(g["centroid"][im][1]))])
        # ... flattened in record order (main.py:53-66), KeyPoints rebuilt by make_kp
        M = ref_main.Main()
        temp_kp, sizes, cents, des = [], [], [], []
        for rec in records:
            temp_kp.extend(rec[0])
            sizes.extend([rec[2]] * len(rec[0]))
            cents.extend([rec[3]] * len(rec[0]))
            des.append(rec[1])
        M.kp = ref_sh.make_kp(temp_kp)
        M.des = np.concatenate(des, axis=0)
        M.img_size_list, M.img_centroid_list = sizes, cents
        M.kp_query, M.des_query = qk, g["q_des"]
        shape = tuple(int(v) for v in g["shape"])
        M.rgb_query = types.SimpleNamespace(shape=shape)
        M.image_query_size = (shape[1], shape[0])
        M.run_matcher()
        mk = M.matching_keypoints
        qpos = {id(k): i for i, k in enumerate(qk)}
        out = dict(extra)
        out["mk_q"] = np.array([qpos[id(t[1])] for t in mk], np.int32)
        out["mk_model"] = kp_field_rows([t[0] for t in mk])
        out["mk_query"] = kp_field_rows([t[1] for t in mk])
        out["mk_img_size"] = np.array([t[2] for t in mk], np.int32).reshape(-1, 2)
        out["mk_centroid"] = np.array([t[3] for t in mk], np.float64).reshape(-1, 2)
        assert np.array_equal(out["mk_q"], np.nonzero(g["good"])[0])
        M.apply_hough_transform(int(g["bins"]))
        M.get_valid_bins(5)
        off, pm, pq = [0], [], []
        for b in M.valid_bins:
            pm.extend(p[0] for p in b.keypoint_pairs)
            pq.extend(p[1] for p in b.keypoint_pairs)
            off.append(len(pm))
        out["valid_off"] = np.array(off, np.int64)
        out["valid_pairs_model"] = kp_field_rows(pm)
        out["valid_pairs_query"] = kp_field_rows(pq)
        assert np.array_equal(out["valid_off"], g["valid_off"])
        M.apply_affine_parameters(4)
        off, pm, pq = [0], [], []
        for b in M.valid_bins:
            pm.extend(p[0] for p in b.keypoint_pairs)
            pq.extend(p[1] for p in b.keypoint_pairs)
            off.append(len(pm))
        out["surv_off"] = np.array(off, np.int64)
        out["surv_pairs_model"] = kp_field_rows(pm)
        out["surv_pairs_query"] = kp_field_rows(pq)
        assert np.array_equal(out["surv_off"], g["surv_off"])
        print(name, "matching_keypoints", len(mk), "valid pairs", len(out["valid_pairs_model"]),
              "surviving pairs", len(out["surv_pairs_model"]))
        save("kpfields_" + name, **out)


def main_repeat():
    """get_valid_bins called twice on the same votes (main.py:121-132): ``valid_bins``
    accumulates (earlier bins kept, new ones appended in insertion order) while
    ``keypoint_pairs`` is rebuilt from the bins at the latest threshold only; then
    apply_affine_parameters(4) on the accumulated list.  The edge_b15 and near_edge_b15
    matches (votes spread over 1..12+); threshold sequences (5, 7), (7, 5) and (9, 3);
    written to repeat_<case>.npz."""
    import sod_pkg
    sod_pkg.load()
    ref_main, _ = import_reference()
    from sift_based_od_amd.database import Keypoints
    for name in ("edge_b15", "near_edge_b15"):
        g = dict(np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False))
        qkp = Keypoints(g["q_x"], g["q_y"], g["q_angle"], g["q_octave"])
        dbkp = Keypoints(g["db_x"], g["db_y"], g["db_angle"], g["db_octave"])
        shape = tuple(int(v) for v in g["shape"])
        bins = int(g["bins"])
        matches = [(int(q), int(m)) for q, m in zip(g["match_q"], g["match_m"])]
        out = {}
        for a, b in ((5, 7), (7, 5), (9, 3)):
            M = ref_main.Main()
            M.rgb_query = types.SimpleNamespace(shape=shape)
            M.image_query_size = (shape[1], shape[0])
            kq, km = kp_objects(qkp), kp_objects(dbkp)
            ident = {}
            for q, m in matches:
                im = int(g["db_img"][m])
                M.matching_keypoints.append(
                    (km[m], kq[q], (int(g["size"][im][0]), int(g["size"][im][1])),
                     (float(g["centroid"][im][0]), float(g["centroid"][im][1]))))
                ident[(id(km[m]), id(kq[q]))] = q
            M.apply_hough_transform(bins)
            tag = "t%d_%d_" % (a, b)
            for step, thr in enumerate((a, b)):
                M.get_valid_bins(thr)
                out[tag + "valid_keys%d" % step] = np.array([x.pose for x in M.valid_bins],
                                                           np.int32).reshape(-1, 4)
                out[tag + "pairs%d" % step] = np.array([ident[(id(p[0]), id(p[1]))]
                                                       for p in M.keypoint_pairs], np.int32)
            M.apply_affine_parameters(4)
            sv = M.valid_bins
            out[tag + "surv_keys"] = np.array([x.pose for x in sv], np.int32).reshape(-1, 4)
            out[tag + "surv_votes"] = np.array([x.votes for x in sv], np.int32)
            out[tag + "surv_params"] = np.array([list(map(float, x.affine_parameters))
                                                 for x in sv], np.float64).reshape(-1, 6)
            out[tag + "surv_pairs"] = np.array([ident[(id(p[0]), id(p[1]))]
                                                for p in M.keypoint_pairs], np.int32)
            print(name, "repeat", a, b, "valid",
                  [len(out[tag + "valid_keys%d" % k]) for k in (0, 1)],
                  "pairs", [len(out[tag + "pairs%d" % k]) for k in (0, 1)], "surv", len(sv))
        save("repeat_" + name, **out)


if __name__ == "__main__":
    if sys.argv[1:] == ["near_edge"]:
        main_near_edge()
    elif sys.argv[1:] == ["keypoints"]:
        main_keypoints()
    elif sys.argv[1:] == ["repeat"]:
        main_repeat()
    else:
        main()
