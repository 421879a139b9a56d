"""Drop-in for ``cv2.BFMatcher().knnMatch(des_query, des, k=2)`` (call site
``main.py:70-71``) running on the MI355X matcher kernel (int8 MFMA, match_i8.hip; bf16
match.hip selectable), plus the ratio test
of ``main.py:81-86``.

``knnMatch`` returns what OpenCV returns: per query a list of ``DMatch`` sorted by
distance (ties keep the lower ``trainIdx``); ``distance`` is the float32 L2 distance.
The vectorised :func:`knn2` / :func:`ratio_match` return numpy arrays and are what the
pipeline uses.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib

NORM_L2 = 4   # cv2.NORM_L2


@dataclass
class DMatch:
    """Mirror of ``cv2.DMatch`` (fields main.py reads: queryIdx, trainIdx, distance)."""
    queryIdx: int
    trainIdx: int
    imgIdx: int
    distance: float


def knn2(des_query, des_train, ctx=None):
    """(idx1 int32[Nq], d1 f32[Nq], d2 f32[Nq]) of the two nearest train rows.
    ``d2`` is +inf when there is a single train row."""
    ctx = ctx or _lib.default_context()
    q = np.asarray(des_query)
    d = np.asarray(des_train)
    if q.shape[0] == 0:
        return np.zeros(0, np.int32), np.zeros(0, np.float32), np.zeros(0, np.float32)
    ctx.upload_db(d)
    ctx.upload_queries(q)
    ctx.match()
    ctx.ratio(0.75)
    idx1, d1, d2, _ = ctx.match_result()
    if d.shape[0] == 1:
        d2 = np.full_like(d2, np.inf)
    return idx1, d1, d2


def ratio_match(des_query, des_train, ratio=0.75, ctx=None):
    """Match + Lowe ratio test (``m.distance < ratio * n.distance``, main.py:82).
    Returns (idx1, d1, d2, good bool[Nq])."""
    ctx = ctx or _lib.default_context()
    ctx.upload_db(np.asarray(des_train))
    ctx.upload_queries(np.asarray(des_query))
    ctx.match()
    ctx.ratio(ratio)
    return ctx.match_result()


class BFMatcher:
    """``cv2.BFMatcher(normType=NORM_L2, crossCheck=False)``: brute force, L2 only.

    ``knnMatch(k=2)`` returns both DMatch objects complete, the second one's ``trainIdx``
    included (OpenCV fills it; main.py:81-86 reads only its distance): OpenCV orders by the
    float distance with ties to the lower trainIdx, so ``n.trainIdx`` is the lowest row other
    than ``m``'s at the second float distance -- and, for inputs whose distances reach 2048
    (not SIFT: its norms are ~512), where two squared distances can share a float,
    ``m.trainIdx`` is the lowest row at the first.  Those indices come from MFMA passes over
    the DB (``sod_match_knn_indices``, bf16 matcher), so this object runs on a bf16 context
    of its own unless one is given."""

    def __init__(self, normType=NORM_L2, crossCheck=False, ctx=None):
        if normType != NORM_L2:
            raise NotImplementedError("only NORM_L2 (SIFT) is implemented")
        if crossCheck:
            raise NotImplementedError("crossCheck is not used by the reference")
        self._ctx = ctx

    def _context(self):
        if self._ctx is None:
            self._ctx = _lib.Context(0)
            self._ctx.set_impl("bf16")
        return self._ctx

    def knnMatch(self, queryDescriptors, trainDescriptors, k=2):
        if k not in (1, 2):
            raise NotImplementedError("k must be 1 or 2 (main.py uses k=2)")
        q = np.asarray(queryDescriptors)
        d = np.asarray(trainDescriptors)
        ntrain = d.shape[0]
        if ntrain == 0:   # OpenCV: no neighbours for any query
            return [[] for _ in range(q.shape[0])]
        if q.shape[0] == 0:
            return []
        ctx = self._context()
        ctx.set_impl("bf16")
        ctx.upload_db(d)
        ctx.upload_queries(q)
        ctx.match()
        ctx.ratio(0.75)
        idx1, d1, d2, _ = ctx.match_result()
        idx1, idx2 = ctx.knn_indices()
        if k == 1 or ntrain == 1:
            return [[DMatch(i, int(idx1[i]), 0, float(d1[i]))] for i in range(len(idx1))]
        return [[DMatch(i, int(idx1[i]), 0, float(d1[i])),
                 DMatch(i, int(idx2[i]), 0, float(d2[i]))] for i in range(len(idx1))]
