"""``Main`` -- the stage driver of ``main.py:17-188`` on the device.

Same stage names, order and thresholds as the reference::

    m = Main()
    m.set_database(db)                                   # main.py:48-66 (pickle -> SoA)
    m.get_query_features(des_query, kp_query, shape)     # main.py:36-45 (SIFT output given)
    m.get_query_image(bgr_image)                         # main.py:36-45 (SIFT on the device)
    m.run_matcher()                                      # main.py:68-87
    m.apply_hough_transform(15)                          # main.py:89-119
    m.get_valid_bins(5)                                  # main.py:121-132
    m.apply_affine_parameters(4)                         # main.py:139-157

Every stage runs on the device and leaves its result there; the reference's Python
objects (``matching_keypoints`` tuples, the ``hough_transform`` dict of PoseBins,
``valid_bins``, ``keypoint_pairs``) are materialised lazily, only when read.  ``run()``
enqueues the whole path on one stream (the bench path).  ``get_query_image`` runs SIFT
detection (``main.py:43``) on the device as well; plotting stays
outside.
"""
from __future__ import annotations

import gc

import numpy as np

from . import _lib
from .constants import REFERENCE
from .database import Keypoints, SiftDatabase
from .hough import hough_table_from_tuples, posebins_from_device
from .postprocessing import final_pose_from_arrays
from .sift_helpers import keypoints_from_arrays

POS_FACTOR = REFERENCE.pos_factor   # main.py:141


class _Shape:
    def __init__(self, shape):
        self.shape = tuple(shape)


class Main:

    def __init__(self, ctx=None, device=0):
        self.ctx = ctx or _lib.Context(device)
        self.db = None
        self.kp = _LazyKeypoints(self, "db")
        self.des = None
        self.kp_query = _LazyKeypoints(self, "query")
        self.des_query = None
        self.rgb_query = None
        self.image_query_size = (0, 0)
        self._matching = None          # list of tuples once materialised / assigned
        self._match = None             # (idx1, good) device results
        self._hough_bins = None
        self._table = None
        self.valid_bins = []
        self.keypoint_pairs = []
        self.final_pose = []
        self._stage = None
        self._sel_token = 0            # device selections made (PoseBin.bind_device)
        self._valid_sel = None         # (token, valid_result) of get_valid_bins' selection
        self._tuple_ctx = None         # context of the tuple-given Hough path (reused)
        self._exact = None             # squared-distance order == OpenCV's (per upload)
        self.affine_path = None        # how the last apply_affine_parameters ran

    # ---------------------------------------------------------------- inputs
    def set_database(self, db):
        """The flattened training database (``main.py:53-66``): a :class:`SiftDatabase`
        (e.g. ``SiftDatabase.load`` of a saved file, packed image included), a path to such
        a file, or the reference's pickle payload (list of per-image records)."""
        if isinstance(db, (str, bytes)) or hasattr(db, "__fspath__"):
            db = SiftDatabase.load(db)
        if not isinstance(db, SiftDatabase):
            db = SiftDatabase.from_records(db)
        self.db = db
        self.des = db.des
        db.upload(self.ctx)
        self._exact = None
        self.kp = _LazyKeypoints(self, "db")

    def get_query_features(self, des_query, kp_query, image_shape, database=None):
        """``main.py:36-45`` with the SIFT output given: descriptors [Nq,128] and the
        keypoints (a :class:`Keypoints` SoA or a list of cv2.KeyPoint);
        ``image_shape`` = ``rgb_query.shape``."""
        if database is not None:
            self.set_database(database)
        if not isinstance(kp_query, Keypoints):
            kp_query = Keypoints.from_cv(kp_query)   # keeps the caller's objects (main.py:43)
        self._qkp = kp_query
        self.des_query = np.asarray(des_query)
        self.rgb_query = _Shape(image_shape)
        self.image_query_size = (int(image_shape[1]), int(image_shape[0]))   # (w, h)
        self.kp_query = _LazyKeypoints(self, "query")
        self.ctx.upload_queries(self.des_query, kp_query)
        self._reset_after_match()

    def get_query_image(self, image, database=None):
        """``main.py:36-45`` from the image itself: ``image`` as ``cv2.imread`` returns it
        (8-bit BGR [h, w, 3]) or already gray [h, w].  BGR2GRAY and
        ``SIFT_create().detectAndCompute`` run on the device and the
        features become the query set without leaving it."""
        if database is not None:
            self.set_database(database)
        img = np.asarray(image)
        r = self.ctx.sift_detect(img)
        if len(r["x"]) == 0:
            raise ValueError("the query image has no SIFT keypoints")
        self.ctx.sift_to_queries()
        self._qkp = Keypoints(r["x"], r["y"], r["angle"], r["octave"], r["size"], r["response"])
        self.des_query = r["descriptors"]
        self.sift_query = r
        self.rgb_query = _Shape(img.shape if img.ndim == 3 else img.shape + (3,))
        self.image_query_size = (int(img.shape[1]), int(img.shape[0]))   # (w, h)
        self.kp_query = _LazyKeypoints(self, "query")
        self._reset_after_match()

    def _exact_order(self):
        """sod_match_exact_order of the current uploads (one device read per upload)."""
        if self._exact is None:
            self._exact = self.ctx.exact_order()
        return self._exact

    def _reset_after_match(self):
        self._exact = None
        self._matching = None
        self._match = None
        self._table = None
        self.valid_bins = []
        self.keypoint_pairs = []

    # ---------------------------------------------------------------- stages
    def run_matcher(self, ratio=0.75):
        """``main.py:68-87``: knnMatch(k=2) + ratio test, on the device.  ``m.trainIdx`` is
        OpenCV's: ordered by the float distance, ties to the lower row.  The matcher orders by
        the exact squared distance, which is the same order whenever every distance is below
        2048 (always for SIFT descriptors, norm ~512); otherwise ``float_order`` re-derives
        the index from the float distance on the device (sod_match_float_order)."""
        self.ctx.match()
        self.ctx.ratio(ratio)
        self.ctx.float_order()
        idx1, d1, d2, good = self.ctx.results(parts=("match",))["match"]   # one transfer
        self._match = (idx1, good)
        self._matching = None
        self._stage = "matched"

    @property
    def matching_keypoints(self):
        """(kpM, kpQ, model_img_size, model_centroid) per good match in query order
        (``main.py:85-86``).  Assigning a list makes the next stage use it instead."""
        if self._matching is None:
            if self._match is None:
                self._matching = []
            else:
                idx1, good = self._match
                self._matching = [self._tuple(int(q), int(idx1[q])) for q in np.nonzero(good)[0]]
        return self._matching

    @matching_keypoints.setter
    def matching_keypoints(self, value):
        self._matching = list(value)
        self._match = None
        self._stage = "assigned"

    def _tuple(self, q, m):
        im = int(self.db.img[m])
        return (self.kp[m], self.kp_query[q], (int(self.db.size[im][0]), int(self.db.size[im][1])),
                (float(self.db.centroid[im][0]), float(self.db.centroid[im][1])))

    def apply_hough_transform(self, bins=15):
        """``main.py:89-119`` with ``bins`` an int (reference) or per-axis 4-tuple."""
        shape = self.rgb_query.shape
        self._hough_bins = bins
        self._table = None
        if self._stage == "assigned":
            # tuples set by the caller: vote over them as given (on a second context, kept)
            if self._tuple_ctx is None:
                self._tuple_ctx = _lib.Context(self.ctx.device)
            _, self._tuple_bins = hough_table_from_tuples(self._matching, shape, bins, 1,
                                                          self._tuple_ctx)
            self._table = {b.pose: b for b in self._tuple_bins}
            return
        self.ctx.hough(shape, bins)

    @property
    def hough_transform(self):
        """The {pose: PoseBin} dict in insertion (first-touch) order."""
        if self._table is None:
            if self._hough_bins is None:
                return {}
            res = self._select(1)
            self._table = {b.pose: b for b in posebins_from_device(res, self._pair, self._size_of,
                                                                   self._sel_token)}
            self._selected_thr = 1
        return self._table

    def _pair(self, q):
        return (self.kp[int(self._match[0][q])], self.kp_query[q])

    def _size_of(self, q):
        m = int(self._match[0][q])
        im = int(self.db.img[m])
        return (int(self.db.size[im][0]), int(self.db.size[im][1]))

    def _select(self, threshold):
        self.ctx.select(threshold)
        self._sel_token += 1
        return self.ctx.results(parts=("valid",))["valid"]   # one transfer

    def get_valid_bins(self, threshold=5):
        """``main.py:121-132``: bins with votes >= threshold, insertion order.  The bins'
        members stay on the device (``keypoint_pairs`` is built when first read), and so
        does ``self.keypoint_pairs`` (a lazy concatenation).  As in the reference, a repeated
        call appends only the bins not yet in ``valid_bins`` (which keeps the earlier
        calls' bins), while ``keypoint_pairs`` is rebuilt from the bins at THIS call's
        threshold alone, in hough_transform's insertion order (main.py:123-129)."""
        if self._stage == "assigned":
            vb = [b for b in self._table.values() if b.votes >= threshold]
        else:
            res = self._select(threshold)
            tok = self._sel_token
            off, mem = res["offsets"], res["members"]
            if self._table is not None:
                vb = [self._table[tuple(int(v) for v in k)] for k in res["keys"]]
                for i, b in enumerate(vb):
                    b.bind_device(tok, i, mem[off[i]:off[i + 1]], self._pair)
            elif not self.valid_bins:
                # main.py's case (a fresh list): the bins come straight from the device
                # selection and their PoseBin objects are made on first access -- the
                # device-resident affine pass builds only its survivors
                self._valid_sel = (tok, res)
                self.valid_bins = _DeviceBins(res, self._pair, self._size_of, tok)
                self.keypoint_pairs = _LazyPairs(self.valid_bins)
                self._valid_thr = threshold
                return
            else:
                vb = posebins_from_device(res, self._pair, self._size_of, tok)
            self._valid_sel = (tok, res)
        # main.py:131's `not in` scan, by pose (PoseBin.__eq__) through a set: O(V)
        seen = {b.pose for b in self.valid_bins}
        for b in vb:
            if b.pose not in seen:
                seen.add(b.pose)
                self.valid_bins.append(b)
        self.keypoint_pairs = _LazyPairs(vb)          # main.py:123,129: this threshold's bins
        self._valid_thr = threshold

    def update_keypoint_pairs(self):
        """``main.py:134-137`` (the concatenation is built when first read)."""
        self.keypoint_pairs = _LazyPairs(self.valid_bins)

    def _device_resident(self):
        """True when ``valid_bins`` is exactly the device's current selection, in its order,
        and no bin was edited by the caller (members, votes, pose): the affine stage can then
        run on the members already on the device."""
        if self._valid_sel is None or self._stage == "assigned":
            return False
        tok, res = self._valid_sel
        vb = self.valid_bins
        if isinstance(vb, _DeviceBins) and vb.unbuilt():   # untouched since the selection
            # ... and that selection is still the device's (reading hough_transform selects
            # again, at threshold 1)
            return vb.token == tok == self._sel_token
        if tok != self._sel_token or len(self.valid_bins) != len(res["keys"]):
            return False
        return all(b.device_index(tok) == i for i, b in enumerate(self.valid_bins))

    def apply_affine_parameters(self, threshold=4):
        """``main.py:139-157``: per-bin fixed point of {AffineParameters;
        remove_outliers} with factor pos_factor*4, on the device (all bins at once).  When
        the valid bins are the device's selection, untouched, the kernel runs on the
        members resident there (no host gather / upload); otherwise on the bins' own
        keypoint pairs."""
        if self._device_resident():
            self.ctx.affine(self.image_query_size, POS_FACTOR * 4, POS_FACTOR * 4, threshold)
            a = self.ctx.results(parts=("affine",))["affine"]   # one transfer
            res = self._valid_sel[1]
            offs = np.asarray(res["offsets"])
            alive = a["alive"]
            survived = a["survived"]
            vb = self.valid_bins
            gc_was_on = gc.isenabled()
            gc.disable()          # (no cycles among these; GC passes were a third of the loop)
            try:
                if isinstance(vb, _DeviceBins) and vb.unbuilt():
                    # nobody has seen the bins: build the survivors only, as the loop below
                    # leaves them (the others are dropped unseen); per-survivor slices, not
                    # a pass over every member
                    sidx = np.nonzero(survived)[0].tolist()
                    out = posebins_from_device(res, self._pair, self._size_of, vb.token, sidx)
                    votes = a["votes"][sidx].tolist()
                    params = a["params"][sidx].tolist()
                    mem = np.asarray(res["members"])
                    lo_hi = offs.tolist()
                    for j, (i, b) in enumerate(zip(sidx, out)):
                        lo, hi = lo_hi[i], lo_hi[i + 1]
                        al = alive[lo:hi]
                        b.keep_device_members(al, mem[lo:hi][al])
                        b.votes = votes[j]
                        b.affine_parameters = params[j]
                else:
                    off = offs.tolist()
                    # every bin's surviving members with one mask (per-bin masking was ~1 us a bin)
                    kept = np.asarray(res["members"])[alive]
                    koff = np.concatenate([[0], np.cumsum(np.add.reduceat(
                        alive.astype(np.int64), offs[:-1]))]).tolist() if len(off) > 1 else [0]
                    votes, params = a["votes"].tolist(), a["params"].tolist()   # scalars in bulk
                    surv = survived.tolist()
                    out = []
                    for i, b in enumerate(vb):
                        b.keep_device_members(alive[off[i]:off[i + 1]], kept[koff[i]:koff[i + 1]])
                        b.votes = votes[i]
                        b.affine_parameters = params[i]
                        if surv[i]:
                            out.append(b)
            finally:
                if gc_was_on:
                    gc.enable()
            if out and not self.ctx.trig_exact():
                # the device's cos / sin are not this host's libm (sod_trig_exact): the
                # survivors' centroids as the reference computes them here (the host's cos /
                # sin per member, sod_exact_means), so post_process's <= thresholds and the
                # final pose see main.py's values bit for bit
                sidx = np.nonzero(survived)[0].tolist()
                for b, (x, y) in zip(out, self.ctx.exact_means(sidx).tolist()):
                    b.centroid = (x, y)
            self.valid_bins = out
            self._valid_sel = None
            self.affine_path = "device-resident"
        else:
            from .affine import verify_bins
            self.valid_bins = verify_bins(self.valid_bins, self.image_query_size, threshold,
                                          POS_FACTOR * 4, POS_FACTOR * 4, self.ctx)
            self.affine_path = "host-pairs"
        self.update_keypoint_pairs()

    def post_process(self):
        """``main.py:159-168`` on ``self.valid_bins``: position clusters, orientation
        clusters, dominant orientation, final pose (pairwise relations on the device)."""
        from .postprocessing import (find_max_orientation, get_final_pose, group_orientation,
                                     group_position)
        pose_cluster = group_position(self.valid_bins, self.ctx)
        orientation_cluster = group_orientation(pose_cluster, self.ctx)
        final_orientation_list = find_max_orientation(orientation_cluster)
        self.final_pose = get_final_pose(pose_cluster, final_orientation_list)

    # ---------------------------------------------------------------- fused
    def run(self, bins=15, vote_threshold=5, affine_threshold=4, ratio=0.75, run_affine=True,
            post_process=True):
        """The whole path on one stream, results left on the device; returns a dict of
        arrays (matches, valid bins, members, means, affine survivors/params, and the
        post-processing clusters / final poses).  When OpenCV's float order is not provably
        the squared-distance order (distances reaching 2048: not SIFT input), the stages are
        enqueued one by one with the float-order trainIdx in between (``run_matcher``)."""
        parts = ("match", "valid") + (("affine",) if run_affine else ()) + \
            (("post",) if post_process else ())
        if self._exact_order():
            # results staged right behind the pipeline: the read below only waits
            self.ctx.pipeline(self.rgb_query.shape, bins, ratio, vote_threshold,
                              affine_threshold, POS_FACTOR * 4.0, POS_FACTOR * 4.0, run_affine,
                              stage=parts)
        else:
            self.ctx.match()
            self.ctx.ratio(ratio)
            self.ctx.float_order()
            self.ctx.hough(self.rgb_query.shape, bins)
            self.ctx.select(vote_threshold)
            if run_affine:
                self.ctx.affine(self.image_query_size, POS_FACTOR * 4.0, POS_FACTOR * 4.0,
                                affine_threshold)
        # every result in one device -> host transfer and one wait (sod_results_fetch)
        r = self.ctx.results(parts=parts)
        idx1, d1, d2, good = r["match"]
        out = {"idx1": idx1, "d1": d1, "d2": d2, "good": good, "valid": r["valid"]}
        if run_affine:
            out["affine"] = r["affine"]
        if post_process:
            out["post"] = r["post"]
            self.final_pose = final_pose_from_arrays(out["post"])
        self._match = (idx1, good)
        self._hough_bins = bins
        return out


class _DeviceBins(list):
    """``Main.valid_bins`` straight from a device selection (valid_result's arrays): the
    PoseBin objects are made on the first access through any list operation, all at once
    and in selection order; ``len`` alone builds nothing.  Until then the device-resident
    affine pass builds only the survivors (the others are dropped unseen) -- at C3 52 of
    1 163 bins."""

    def __init__(self, res, pair_of, size_of, token):
        super().__init__()
        self._src = (res, pair_of, size_of)
        self.token = token

    def unbuilt(self):
        return self._src is not None

    def _build(self):
        if self._src is not None:
            (res, pair_of, size_of), self._src = self._src, None
            list.extend(self, posebins_from_device(res, pair_of, size_of, self.token))

    def __len__(self):
        if self._src is not None:
            return len(self._src[0]["votes"])
        return list.__len__(self)

    def __radd__(self, other):
        # `a_list + self`: list's concatenation reads the right operand's item array
        # directly (C level, no method call), which is empty until built; a subclass's
        # reflected method runs first
        self._build()
        return list.__add__(list(other), self)

    for _m in ("__getitem__", "__iter__", "__contains__", "__repr__", "__eq__", "__ne__",
               "__lt__", "__le__", "__gt__", "__ge__", "__reversed__", "index", "count", "copy",
               "__add__", "__mul__", "__rmul__", "__reduce_ex__", "__sizeof__", "append",
               "extend", "insert", "remove", "pop", "clear", "sort", "reverse", "__setitem__",
               "__delitem__", "__iadd__", "__imul__"):
        def _f(self, *a, _m=_m, **k):
            self._build()
            return getattr(list, _m)(self, *a, **k)
        locals()[_m] = _f
    del _m, _f


class _LazyPairs(list):
    """``Main.keypoint_pairs`` (main.py:134-137): the valid bins' pairs concatenated, built
    on first use, so the pairs stay on the device until someone reads them."""

    def __init__(self, bins):
        super().__init__()
        # (an unbuilt device list is held as it is: copying it would build every bin)
        self._bins = bins if isinstance(bins, _DeviceBins) and bins.unbuilt() else list(bins)
        self._built = False

    def _build(self):
        if not self._built:
            self._built = True
            for b in self._bins:
                super().extend(b.keypoint_pairs)

    def __radd__(self, other):   # (see _DeviceBins.__radd__)
        self._build()
        return list.__add__(list(other), self)

    for _m in ("__len__", "__getitem__", "__iter__", "__contains__", "__repr__", "__eq__",
               "__reversed__", "index", "count", "copy", "__add__", "__mul__"):
        def _f(self, *a, _m=_m, **k):
            self._build()
            return getattr(list, _m)(self, *a, **k)
        locals()[_m] = _f
    for _m in ("append", "extend", "insert", "remove", "pop", "clear", "sort", "reverse",
               "__setitem__", "__delitem__", "__iadd__"):
        def _g(self, *a, _m=_m, **k):
            self._build()
            return getattr(list, _m)(self, *a, **k)
        locals()[_m] = _g
    del _m, _f, _g


class _LazyKeypoints:
    """List-like view creating one (cached) KeyPoint object per accessed row, so the
    same keypoint is the same object everywhere, as in the reference."""

    def __init__(self, owner, which):
        self._owner = owner
        self._which = which
        self._cache = {}

    def _src(self):
        return self._owner.db.kp if self._which == "db" else self._owner._qkp

    def __len__(self):
        src = self._src() if (self._owner.db is not None or self._which == "query") else None
        return len(src) if src is not None else 0

    def __getitem__(self, i):
        i = int(i)
        k = self._cache.get(i)
        if k is None:
            k = keypoints_from_arrays(self._src(), i)   # the caller's own object when given
            self._cache[i] = k
        return k
