"""Flat structure-of-arrays layout of the reference's descriptor database.

The reference keeps the database as a pickle of per-image records
``[temp_kp, des, img_size, centroid, path]`` (``GenerateDatabaseInfo.py:35``)
and flattens it on every query with an O(T*N) ``np.append`` loop
(``main.py:53-66``), replicating each image's size and centroid per keypoint
(``main.py:54-60``).  Here the flat form is the native one:

* ``des``       uint8 [N,128]   (OpenCV SIFT descriptors are integers 0..255)
* ``kp``        :class:`Keypoints` SoA -- x, y, angle f32; packed octave i32
* ``img``       int32 [N]       model image of each row
* ``centroid``  float64 [I,2]   per-image keypoint centroid (``get_centroid``)
* ``size``      int32 [I,2]     per-image (width, height)

Row order is the reference's concatenation order, so ``trainIdx`` values are
identical to ``main.py``'s.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

DESC_DIM = 128


@dataclass
class Keypoints:
    """SoA view of a list of ``cv2.KeyPoint`` (only the fields the hot path
    reads: ``pt``, ``angle``, ``octave``; ``HoughTransformHelperFunctions.py:10-20``)."""
    x: np.ndarray
    y: np.ndarray
    angle: np.ndarray
    octave: np.ndarray

    def __post_init__(self):
        self.x = np.ascontiguousarray(self.x, np.float32)
        self.y = np.ascontiguousarray(self.y, np.float32)
        self.angle = np.ascontiguousarray(self.angle, np.float32)
        self.octave = np.ascontiguousarray(self.octave, np.int32)
        n = self.x.shape[0]
        for a in (self.y, self.angle, self.octave):
            if a.shape != (n,):
                raise ValueError("keypoint arrays must be 1-D and equally long")

    def __len__(self):
        return int(self.x.shape[0])

    @classmethod
    def from_cv(cls, kps):
        """From objects exposing ``pt``, ``angle`` and ``octave`` (cv2.KeyPoint)."""
        n = len(kps)
        x = np.empty(n, np.float32)
        y = np.empty(n, np.float32)
        a = np.empty(n, np.float32)
        o = np.empty(n, np.int32)
        for i, k in enumerate(kps):
            x[i], y[i] = k.pt[0], k.pt[1]
            a[i] = k.angle
            o[i] = k.octave
        return cls(x, y, a, o)

    def slice(self, lo, hi):
        return Keypoints(self.x[lo:hi], self.y[lo:hi], self.angle[lo:hi], self.octave[lo:hi])


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
            kp = Keypoints(z["x"], z["y"], z["angle"], z["octave"])
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
        xs, ys, angs, octs, imgs, dess, cents, sizes = [], [], [], [], [], [], [], []
        for i, rec in enumerate(records):
            temp_kp, des, img_size, centroid = rec[0], rec[1], rec[2], rec[3]
            n = len(temp_kp)
            xs.append(np.array([t[0][0] for t in temp_kp], np.float32))
            ys.append(np.array([t[0][1] for t in temp_kp], np.float32))
            angs.append(np.array([t[2] for t in temp_kp], np.float32))
            octs.append(np.array([t[4] for t in temp_kp], np.int32))
            imgs.append(np.full(n, i, np.int32))
            dess.append(np.asarray(des))
            cents.append((float(centroid[0]), float(centroid[1])))
            sizes.append((int(img_size[0]), int(img_size[1])))
        kp = Keypoints(np.concatenate(xs), np.concatenate(ys),
                       np.concatenate(angs), np.concatenate(octs))
        return cls(np.concatenate(dess, axis=0), kp, np.concatenate(imgs),
                   np.array(cents, np.float64), np.array(sizes, np.int32))

    @classmethod
    def from_images(cls, images, sift=None):
        """``GenerateDatabaseInfo.py:19-37`` on the device: SIFT of every training image
        (8-bit gray or BGR, already resized as the script's ``cv2.resize`` to width 1500
        does), its keypoints, ``get_centroid`` and ``img_size = (w, h)``."""
        from .sift import SIFT_create
        sift = sift or SIFT_create()
        xs, ys, angs, octs, imgs, dess, cents, sizes = [], [], [], [], [], [], [], []
        images = [np.asarray(im) for im in images]
        for i, (img, r) in enumerate(zip(images, sift.detect_batch(images))):
            n = len(r["x"])
            if n == 0:
                raise ValueError("training image %d has no SIFT keypoints" % i)
            xs.append(r["x"])
            ys.append(r["y"])
            angs.append(r["angle"])
            octs.append(r["octave"])
            imgs.append(np.full(n, i, np.int32))
            dess.append(r["descriptors"])
            cents.append(centroid_of(r["x"], r["y"]))
            sizes.append((int(np.shape(img)[1]), int(np.shape(img)[0])))
        kp = Keypoints(np.concatenate(xs), np.concatenate(ys), np.concatenate(angs),
                       np.concatenate(octs))
        return cls(np.concatenate(dess, axis=0), kp, np.concatenate(imgs),
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
