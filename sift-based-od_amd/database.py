"""Flat structure-of-arrays layout of the reference's descriptor database.

The reference keeps the database as a pickle of per-image records
``[temp_kp, des, img_size, centroid, path]`` (``GenerateDatabaseInfo.py:35``)
and flattens it on every query with an O(T*N) ``np.append`` loop
(``main.py:53-66``), replicating each image's size and centroid per keypoint
(``main.py:54-60``).  Here the flat form is the native one:

* ``des``       uint8 [N,128]   (OpenCV SIFT descriptors are integers 0..255)
* ``kp``        :class:`Keypoints` SoA -- x, y, angle f32; packed octave i32 (device);
                size, response f32, class_id i32 (host only)
* ``img``       int32 [N]       model image of each row
* ``centroid``  float64 [I,2]   per-image keypoint centroid (``get_centroid``)
* ``size``      int32 [I,2]     per-image (width, height)

Row order is the reference's concatenation order, so ``trainIdx`` values are
identical to ``main.py``'s.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

DESC_DIM = 128


@dataclass
class Keypoints:
    """SoA view of a list of ``cv2.KeyPoint``.  ``x``, ``y``, ``angle`` and the packed
    ``octave`` are what the hot path reads (``HoughTransformHelperFunctions.py:10-20``) and go
    to the device; ``size``, ``response`` and ``class_id`` stay on the host so the KeyPoint
    objects handed back (``Main.kp``, ``matching_keypoints``, ``PoseBin.keypoint_pairs``)
    carry every field the reference's do (``SiftHelperFunctions.py:42-49``, ``main.py:43``);
    absent, they take cv2.KeyPoint's defaults (0, 0, -1).  ``objects``: the caller's own
    KeyPoint objects when the table was built from them (``from_cv``), handed back as they
    are, as the reference hands back ``kp_query``'s."""
    x: np.ndarray
    y: np.ndarray
    angle: np.ndarray
    octave: np.ndarray
    size: np.ndarray | None = None
    response: np.ndarray | None = None
    class_id: np.ndarray | None = None
    objects: list | None = field(default=None, repr=False, compare=False)

    def __post_init__(self):
        self.x = np.ascontiguousarray(self.x, np.float32)
        self.y = np.ascontiguousarray(self.y, np.float32)
        self.angle = np.ascontiguousarray(self.angle, np.float32)
        self.octave = np.ascontiguousarray(self.octave, np.int32)
        n = self.x.shape[0]
        self.size = (np.zeros(n, np.float32) if self.size is None
                     else np.ascontiguousarray(self.size, np.float32))
        self.response = (np.zeros(n, np.float32) if self.response is None
                         else np.ascontiguousarray(self.response, np.float32))
        self.class_id = (np.full(n, -1, np.int32) if self.class_id is None
                         else np.ascontiguousarray(self.class_id, np.int32))
        for a in (self.y, self.angle, self.octave, self.size, self.response, self.class_id):
            if a.shape != (n,):
                raise ValueError("keypoint arrays must be 1-D and equally long")
        if self.objects is not None and len(self.objects) != n:
            raise ValueError("keypoint objects and arrays differ in count")

    def __len__(self):
        return int(self.x.shape[0])

    @classmethod
    def from_cv(cls, kps):
        """From cv2.KeyPoint objects (or anything exposing ``pt``, ``size``, ``angle``,
        ``response``, ``octave``, ``class_id``); the objects themselves are kept."""
        kps = list(kps)
        n = len(kps)
        x = np.empty(n, np.float32)
        y = np.empty(n, np.float32)
        a = np.empty(n, np.float32)
        o = np.empty(n, np.int32)
        sz = np.empty(n, np.float32)
        r = np.empty(n, np.float32)
        c = np.empty(n, np.int32)
        for i, k in enumerate(kps):
            x[i], y[i] = k.pt[0], k.pt[1]
            a[i] = k.angle
            o[i] = k.octave
            sz[i] = getattr(k, "size", 0.0)
            r[i] = getattr(k, "response", 0.0)
            c[i] = getattr(k, "class_id", -1)
        return cls(x, y, a, o, sz, r, c, objects=kps)

    @classmethod
    def concat(cls, parts):
        """One table of several (keeps the objects only when every part has them)."""
        parts = list(parts)
        objs = None
        if parts and all(p.objects is not None for p in parts):
            objs = [k for p in parts for k in p.objects]
        cat = [np.concatenate([getattr(p, f) for p in parts]) for f in _KP_FIELDS]
        return cls(*cat, objects=objs)

    def slice(self, lo, hi):
        return Keypoints(*[getattr(self, f)[lo:hi] for f in _KP_FIELDS],
                         objects=None if self.objects is None else self.objects[lo:hi])

    def keypoint(self, i):
        """The KeyPoint object of row ``i``: the caller's own when given, else a new one with
        every field of the row (``make_kp``, ``SiftHelperFunctions.py:42-49``)."""
        if self.objects is not None:
            return self.objects[i]
        from .sift_helpers import new_keypoint
        return new_keypoint(float(self.x[i]), float(self.y[i]), float(self.size[i]),
                            float(self.angle[i]), float(self.response[i]), int(self.octave[i]),
                            int(self.class_id[i]))


_KP_FIELDS = ("x", "y", "angle", "octave", "size", "response", "class_id")


def centroid_of(x, y):
    """``get_centroid`` (``SiftHelperFunctions.py:4-14``): a sequential double
    sum of the float32 coordinates divided by the count (``np.cumsum`` is a
    sequential sum, unlike ``np.sum``'s pairwise one)."""
    n = len(x)
    sx = float(np.cumsum(np.asarray(x, np.float64))[-1])
    sy = float(np.cumsum(np.asarray(y, np.float64))[-1])
    return (sx / n, sy / n)


@dataclass
class SiftDatabase:
    des: np.ndarray
    kp: Keypoints
    img: np.ndarray
    centroid: np.ndarray
    size: np.ndarray
    packed: np.ndarray | None = None   # device image (Context.export_packed), optional

    def __post_init__(self):
        self.img = np.ascontiguousarray(self.img, np.int32)
        self.centroid = np.ascontiguousarray(self.centroid, np.float64).reshape(-1, 2)
        self.size = np.ascontiguousarray(self.size, np.int32).reshape(-1, 2)
        if self.des is None:
            if self.packed is None:
                raise ValueError("need descriptors or a packed image")
        else:
            self.des = np.ascontiguousarray(self.des)
            if self.des.ndim != 2 or self.des.shape[1] != DESC_DIM:
                raise ValueError("descriptors must be [N,128]")
            if self.img.shape[0] != self.des.shape[0]:
                raise ValueError("descriptor / image-id counts differ")
        if len(self.kp) != self.img.shape[0]:
            raise ValueError("keypoint / image-id counts differ")

    def __len__(self):
        return int(self.img.shape[0])

    # ---- on-disk format -------------------------------------------
    def save(self, path, ctx=None, keep_descriptors=True):
        """Write the flat database as one ``.npz`` (plain arrays, no pickle): keypoint SoA,
        image table, and -- when a context is given -- the device-packed descriptor image
        of the whole DB (``Context.export_packed``), so :meth:`upload` is a single copy.
        The reference stores a pickle of per-image records instead
        (``GenerateDatabaseInfo.py:35``)."""
        arrays = dict(x=self.kp.x, y=self.kp.y, angle=self.kp.angle, octave=self.kp.octave,
                      kp_size=self.kp.size, kp_response=self.kp.response,
                      kp_class_id=self.kp.class_id,
                      img=self.img, centroid=self.centroid, size=self.size)
        if keep_descriptors and self.des is not None:
            arrays["des"] = np.asarray(self.des, np.uint8)
        if ctx is not None and self.des is not None:
            ctx.upload_db(self.des)
            arrays["packed"] = ctx.export_packed()
        elif self.packed is not None:
            arrays["packed"] = self.packed
        np.savez(path, **arrays)

    @classmethod
    def load(cls, path):
        """Read a file written by :meth:`save` (``numpy.load``, pickles refused)."""
        with np.load(path, allow_pickle=False) as z:
            extra = [z[k] if k in z.files else None
                     for k in ("kp_size", "kp_response", "kp_class_id")]
            kp = Keypoints(z["x"], z["y"], z["angle"], z["octave"], *extra)
            des = z["des"] if "des" in z.files else None
            packed = z["packed"] if "packed" in z.files else None
            return cls(des, kp, z["img"], z["centroid"], z["size"], packed)

    def upload(self, ctx):
        """Keypoints + image table, then the descriptors: the packed image in one copy when
        present and laid out for the context's matcher, else the upload + pack pass."""
        from ._lib import SodError
        ctx.set_keypoints(self.kp, self.img, self.centroid, self.size)
        if self.packed is not None:
            try:
                ctx.import_packed(self.packed)
                return
            except SodError:   # packed for another matcher impl: pack from descriptors
                if self.des is None:
                    raise
        ctx.upload_db(self.des)

    @property
    def n_images(self):
        return int(self.centroid.shape[0])

    @classmethod
    def from_records(cls, records):
        """From the reference's pickle payload: a list of
        ``[temp_kp, des, img_size, centroid, path]`` where ``temp_kp`` is a list of
        ``(pt, size, angle, response, octave, class_id)`` (``make_temp_kp``,
        ``SiftHelperFunctions.py:16-22``)."""
        parts, imgs, dess, cents, sizes = [], [], [], [], []
        for i, rec in enumerate(records):
            temp_kp, des, img_size, centroid = rec[0], rec[1], rec[2], rec[3]
            n = len(temp_kp)
            # (pt, size, angle, response, octave, class_id) per keypoint (make_temp_kp)
            parts.append(Keypoints(np.array([t[0][0] for t in temp_kp], np.float32),
                                   np.array([t[0][1] for t in temp_kp], np.float32),
                                   np.array([t[2] for t in temp_kp], np.float32),
                                   np.array([t[4] for t in temp_kp], np.int32),
                                   np.array([t[1] for t in temp_kp], np.float32),
                                   np.array([t[3] for t in temp_kp], np.float32),
                                   np.array([t[5] for t in temp_kp], np.int32)))
            imgs.append(np.full(n, i, np.int32))
            dess.append(np.asarray(des))
            cents.append((float(centroid[0]), float(centroid[1])))
            sizes.append((int(img_size[0]), int(img_size[1])))
        return cls(np.concatenate(dess, axis=0), Keypoints.concat(parts), np.concatenate(imgs),
                   np.array(cents, np.float64), np.array(sizes, np.int32))

    @classmethod
    def from_images(cls, images, sift=None):
        """``GenerateDatabaseInfo.py:19-37`` on the device: SIFT of every training image
        (8-bit gray or BGR, already resized as the script's ``cv2.resize`` to width 1500
        does), its keypoints, ``get_centroid`` and ``img_size = (w, h)``."""
        from .sift import SIFT_create
        sift = sift or SIFT_create()
        parts, imgs, dess, cents, sizes = [], [], [], [], []
        images = [np.asarray(im) for im in images]
        for i, (img, r) in enumerate(zip(images, sift.detect_batch(images))):
            n = len(r["x"])
            if n == 0:
                raise ValueError("training image %d has no SIFT keypoints" % i)
            parts.append(Keypoints(r["x"], r["y"], r["angle"], r["octave"], r["size"],
                                   r["response"]))
            imgs.append(np.full(n, i, np.int32))
            dess.append(r["descriptors"])
            cents.append(centroid_of(r["x"], r["y"]))
            sizes.append((int(np.shape(img)[1]), int(np.shape(img)[0])))
        return cls(np.concatenate(dess, axis=0), Keypoints.concat(parts), np.concatenate(imgs),
                   np.array(cents, np.float64), np.array(sizes, np.int32))

    def shard(self, rank, world):
        """Rows ``[rank*N/world, (rank+1)*N/world)`` -- the DB-row split of
        SURVEY.md §8(e).  Returns (row_offset, descriptors) for the shard;
        keypoints and the image table stay replicated (they are ~8 % of the
        descriptor bytes and every rank needs them for the verification)."""
        n = len(self)
        lo = (n * rank) // world
        hi = (n * (rank + 1)) // world
        return lo, hi
