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
    ``m.trainIdx`` is the lowest row at the first.  Those indices come from MFMA row-finding
    passes over the resident DB (``sod_match_knn_indices``) after the int8 matcher.

    The train set stays on the device between calls: ``knnMatch(q, train)`` re-uploads
    only when ``train`` is not the array object of the previous call or is writeable (its
    content could have changed in place; a content hash of a 1M-row DB costs more than the
    upload), and OpenCV's own resident-collection API -- ``add([des])`` + ``train()``, then
    ``knnMatch(q, k=2)`` -- uploads once."""

    def __init__(self, normType=NORM_L2, crossCheck=False, ctx=None):
        if normType != NORM_L2:
            raise NotImplementedError("only NORM_L2 (SIFT) is implemented")
        if crossCheck:
            raise NotImplementedError("crossCheck is not used by the reference")
        self._ctx = ctx
        self._resident = None      # (array, context, its db_gen) of the rows on the device
        self._collection = []      # add() / train(): OpenCV's train descriptor collection
        self._trained = None
        self.uploads = 0           # descriptor uploads so far (a residency check)

    def _context(self):
        if self._ctx is None:
            self._ctx = _lib.Context(0)
        return self._ctx

    # ---- OpenCV DescriptorMatcher collection API ----------------------------------------
    def add(self, descriptors):
        """Append train descriptor sets (a list of [n_i, 128] arrays), as OpenCV's ``add``;
        their rows are numbered consecutively (``imgIdx`` is the set)."""
        self._collection.extend(np.asarray(d) for d in descriptors)
        self._trained = None

    def getTrainDescriptors(self):
        return list(self._collection)

    def clear(self):
        self._collection = []
        self._trained = None
        self._resident = None

    def empty(self):
        return len(self._collection) == 0

    def train(self):
        """Concatenate the collection and upload it once (later knnMatch calls without a
        train argument reuse it)."""
        if not self._collection:
            self._trained = np.zeros((0, 128), np.uint8)
        else:
            self._trained = np.concatenate(self._collection, axis=0)
            self._trained.flags.writeable = False   # ours: never changes once uploaded
        self._starts = np.cumsum([0] + [len(d) for d in self._collection])

    def _upload(self, d, ctx):
        # residency is trusted only for an array that cannot change behind our back -- the
        # trained collection, or a read-only array owning its data (a read-only VIEW of a
        # writeable base can change through the base) -- and only while the context still
        # holds the DB this matcher put there (db_gen counts every upload / share / impl switch)
        fixed = d is self._trained or (not d.flags.writeable and d.flags.owndata)
        if (fixed and self._resident is not None and self._resident[0] is d
                and self._resident[1] is ctx and self._resident[2] == ctx.db_gen):
            return
        ctx.upload_db(d)
        self._resident = (d, ctx, ctx.db_gen)
        self.uploads += 1

    def knnMatch(self, queryDescriptors, trainDescriptors=None, k=2):
        if k not in (1, 2):
            raise NotImplementedError("k must be 1 or 2 (main.py uses k=2)")
        img_of = None
        if trainDescriptors is None:   # the collection (OpenCV: knnMatch(query, k))
            if self._trained is None:
                self.train()
            d = self._trained
            if len(self._collection) > 1:
                starts = self._starts
                img_of = lambda t: int(np.searchsorted(starts, t, side="right") - 1)  # noqa: E731
        elif isinstance(trainDescriptors, (int, np.integer)):   # knnMatch(query, k) form
            return self.knnMatch(queryDescriptors, None, int(trainDescriptors))
        else:
            d = trainDescriptors if isinstance(trainDescriptors, np.ndarray) else \
                np.asarray(trainDescriptors)
        q = np.asarray(queryDescriptors)
        ntrain = d.shape[0]
        if ntrain == 0:   # OpenCV: no neighbours for any query
            return [[] for _ in range(q.shape[0])]
        if q.shape[0] == 0:
            return []
        ctx = self._context()
        self._upload(d, ctx)
        ctx.upload_queries(q)
        ctx.match()
        ctx.ratio(0.75)
        idx1, d1, d2, _ = ctx.match_result()
        idx1, idx2 = ctx.knn_indices()

        def dm(i, t, dist):
            if img_of is None:
                return DMatch(i, int(t), 0, float(dist))
            im = img_of(t)
            return DMatch(i, int(t) - int(self._starts[im]), im, float(dist))
        if k == 1 or ntrain == 1:
            return [[dm(i, idx1[i], d1[i])] for i in range(len(idx1))]
        return [[dm(i, idx1[i], d1[i]), dm(i, idx2[i], d2[i])] for i in range(len(idx1))]
