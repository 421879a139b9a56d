"""The oracle (CPU restatement) pinned against golden vectors produced by the reference's
own Python code (tests/golden/make_golden.py).  CPU only."""
import math

import numpy as np
import pytest

from conftest import golden
from helpers import kp, kp_dict
from oracle import oracle as orc

CASES = ["c1_b15", "planted_b15", "planted_b12"]


def test_pose_sweep_bit_exact():
    g = golden("pose_sweep")
    shape = tuple(int(v) for v in g["shape"])
    n = len(g["mx"])
    for i in range(n):
        p = orc.estimate_object_pose(float(g["mx"][i]), float(g["my"][i]), float(g["ma"][i]),
                                     int(g["mo"][i]), float(g["qx"][i]), float(g["qy"][i]),
                                     float(g["qa"][i]), int(g["qo"][i]), float(g["cx"][i]),
                                     float(g["cy"][i]))
        assert p == tuple(g["poses"][i]), i
        for j, b in enumerate(g["bins"]):
            assert orc.calculate_bin_index(p, int(b), shape) == tuple(g["idx"][j][i])


def test_near_edge_sweep_bit_exact():
    """Poses within a few ulps of an x and a y bin edge (the boundary guard's cases)."""
    g = golden("near_edge_sweep")
    shape = tuple(int(v) for v in g["shape"])
    for b in g["bins"]:
        f = {k: g["b%d_%s" % (b, k)] for k in ("mx", "my", "ma", "mo", "qx", "qy", "qa", "qo",
                                                "cx", "cy", "poses", "idx")}
        for i in range(len(f["mx"])):
            p = orc.estimate_object_pose(float(f["mx"][i]), float(f["my"][i]), float(f["ma"][i]),
                                         int(f["mo"][i]), float(f["qx"][i]), float(f["qy"][i]),
                                         float(f["qa"][i]), int(f["qo"][i]), float(f["cx"][i]),
                                         float(f["cy"][i]))
            assert p == tuple(f["poses"][i]), i
            assert orc.calculate_bin_index(p, int(b), shape) == tuple(f["idx"][i])


def test_per_axis_bins_reduce_to_scalar():
    g = golden("pose_sweep")
    shape = tuple(int(v) for v in g["shape"])
    for i in range(0, 2000):
        p = tuple(g["poses"][i])
        for b in (8, 15):
            assert orc.calculate_bin_index(p, (b, b, b, b), shape) == orc.calculate_bin_index(p, b, shape)


def test_sigma_lut_matches_python():
    for bs in (6, 8, 12, 15, 32, 255):
        for k in range(-255, 256):
            s = 2.0 ** k
            ref = min(max(0, int(math.log(s, 2) / 6.5 * bs)), bs - 1)
            assert orc.sigma_index(s, bs) == ref


def _run_case(g):
    qk, dk = kp(g, "q_"), kp(g, "db_")
    matches = [(int(q), int(g["idx1"][q])) for q in np.nonzero(g["good"])[0]]
    return _run_matches(g, matches, qk, dk)


def _run_matches(g, matches, qk, dk):
    shape = tuple(int(v) for v in g["shape"])
    images = {"centroid": g["centroid"], "size": g["size"]}
    table = orc.hough_vote(matches, kp_dict(qk), kp_dict(dk, g["db_img"]), images,
                           int(g["bins"]), shape)
    assert [k for k in table.keys()] == [tuple(k) for k in g["table_keys"]]
    assert [b.votes for b in table.values()] == list(g["table_votes"])
    vb = orc.valid_bins(table, 5)
    assert [b.pose for b in vb] == [tuple(k) for k in g["valid_keys"]]
    for i, b in enumerate(vb):
        mem = [q for q, _ in b.members]
        assert mem == list(g["valid_members"][g["valid_off"][i]:g["valid_off"][i + 1]])
        assert [b.centroid[0], b.centroid[1], b.angle, b.scale, b.img_size[0],
                b.img_size[1]] == list(g["valid_means"][i])
    aff = orc.affine_verify(vb, kp_dict(qk), kp_dict(dk), (shape[1], shape[0]), 4)
    surv = [i for i, r in enumerate(aff) if r["survived"]]
    assert surv == list(g["surv_index"])
    for k, i in enumerate(surv):
        assert aff[i]["votes"] == g["surv_votes"][k]
        assert aff[i]["params"] == list(g["surv_params"][k])      # same numpy calls: bitwise
        mem = [q for q, _ in aff[i]["members"]]
        assert mem == list(g["surv_members"][g["surv_off"][k]:g["surv_off"][k + 1]])


@pytest.mark.parametrize("name", CASES)
def test_matcher_and_pipeline_golden(name):
    g = golden(name)
    idx1, d1, d2 = orc.knn2_match(g["q_des"], g["db_des"])
    assert np.array_equal(idx1, g["idx1"])
    assert np.array_equal(d1, g["d1"]) and np.array_equal(d2, g["d2"])
    assert np.array_equal(orc.ratio_test(d1, d2), g["good"])
    _run_case(g)


@pytest.mark.parametrize("name", ["edge_b15", "edge_b6", "near_edge_b15", "near_edge_b32"])
def test_edges_golden(name):
    g = golden(name)
    matches = list(zip(g["match_q"].tolist(), g["match_m"].tolist()))
    _run_matches(g, matches, kp(g, "q_"), kp(g, "db_"))


def test_matcher_edges_golden():
    g = golden("matcher_edges")
    idx1, d1, d2 = orc.knn2_match(g["q_des"], g["db_des"])
    assert np.array_equal(idx1, g["idx1"])
    assert np.array_equal(d1, g["d1"]) and np.array_equal(d2, g["d2"])
    # ties keep the lowest trainIdx (rows 20, 150, 151 are identical)
    assert (idx1[:10] == 20).all() and (d1[:10] == 0).all() and (d2[:10] == 0).all()
    assert not orc.ratio_test(d1, d2)[:10].any()


def test_matcher_second_index_two_ways():
    """knnMatch's n.trainIdx: the GEMM restatement and the int64 brute force agree on the
    second neighbour's index, ties included (rows 20 / 150 / 151 are identical)."""
    g = golden("matcher_edges")
    a = orc.knn2_match(g["q_des"], g["db_des"], with_idx2=True)
    b = orc.knn2_match_int(g["q_des"], g["db_des"], with_idx2=True)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert (a[3][:10] == 150).all()          # d1 == d2 == 0: the next-lowest equal row


def test_matcher_needs_two_rows():
    with pytest.raises(ValueError):
        orc.knn2_match(np.zeros((3, 128), np.uint8), np.zeros((1, 128), np.uint8))
