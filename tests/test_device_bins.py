"""Main.valid_bins built lazily from a device selection (pipeline._DeviceBins): every list
operation sees exactly the PoseBin objects posebins_from_device makes, in selection order;
len() builds nothing; a subset build (the affine survivors) equals those bins.  CPU only:
the selection arrays are made up."""
import pickle

import numpy as np

from sift_based_od_amd.hough import posebins_from_device
from sift_based_od_amd.pipeline import _DeviceBins, _LazyPairs


def _res(n=7, seed=3):
    rng = np.random.default_rng(seed)
    votes = rng.integers(1, 6, n).astype(np.int32)
    off = np.concatenate([[0], np.cumsum(votes)]).astype(np.int64)
    return {"keys": rng.integers(0, 15, (n, 4)).astype(np.int32), "votes": votes,
            "offsets": off, "members": rng.permutation(int(off[-1])).astype(np.int32),
            "means": rng.normal(0, 100, (n, 6))}


def _pair(q):
    return ("m%d" % q, "q%d" % q)


def _size(q):
    return (640, 480)


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert (x.pose, x.votes, x.centroid, x.angle, x.scale, x.img_size) == \
               (y.pose, y.votes, y.centroid, y.angle, y.scale, y.img_size)
        assert x.keypoint_pairs == y.keypoint_pairs


def test_len_builds_nothing_and_access_builds_all():
    res = _res()
    vb = _DeviceBins(res, _pair, _size, 5)
    assert len(vb) == 7 and vb.unbuilt() and bool(vb)
    ref = posebins_from_device(res, _pair, _size, 5)
    _same(list(vb), ref)
    assert not vb.unbuilt()
    assert vb[2] is vb[2] and vb[-1] is list(vb)[-1]


def test_list_operations():
    res = _res()
    ref = posebins_from_device(res, _pair, _size, 1)
    for op in (lambda v: v[1:4], lambda v: list(reversed(v)), lambda v: v + [],
               lambda v: [b.pose for b in v], lambda v: v.copy()):
        got, exp = op(_DeviceBins(res, _pair, _size, 1)), op(list(ref))
        if got and hasattr(got[0], "pose"):
            _same(got, exp)
        else:
            assert got == exp
    vb = _DeviceBins(res, _pair, _size, 1)
    vb.append("x")
    assert len(vb) == 8 and vb[-1] == "x" and not vb.unbuilt()
    vb = _DeviceBins(res, _pair, _size, 1)
    assert vb != [] and len(pickle.loads(pickle.dumps([b.pose for b in vb]))) == 7


def test_subset_equals_full_build_and_pairs():
    res = _res(12, 9)
    full = posebins_from_device(res, _pair, _size, 2)
    idx = [0, 3, 4, 11]
    _same(posebins_from_device(res, _pair, _size, 2, idx), [full[i] for i in idx])
    vb = _DeviceBins(res, _pair, _size, 2)
    lp = _LazyPairs(vb)
    assert vb.unbuilt()                  # holding the pairs view builds nothing
    assert list(lp) == [p for b in full for p in b.keypoint_pairs]


def test_left_concatenation_sees_the_bins():
    """`a_list + bins` (list's C concatenation reads the right operand's items directly)
    builds the lazy lists first."""
    res = _res()
    ref = posebins_from_device(res, _pair, _size, 4)
    got = ["x"] + _DeviceBins(res, _pair, _size, 4)
    assert got[0] == "x"
    _same(got[1:], ref)
    lp = _LazyPairs(_DeviceBins(res, _pair, _size, 4))
    assert [] + lp == [p for b in ref for p in b.keypoint_pairs]
