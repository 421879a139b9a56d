"""Seeded synthetic SIFT-like workloads.

There is no dataset in this environment (the reference reads
``../Data_Set/...``, ``main.py:48,181``), so every benchmark and parity case
uses these generators:

* descriptors: squared normals, L2-normalised, clipped at 0.2, renormalised to
  norm 512 and rounded to uint8 -- OpenCV's own descriptor normalisation, so
  values are integers 0..255 and ||d||^2 ~ 2.6e5;
* DB images of ``kp_per_image`` keypoints, width 1500, height in [800, 1200]
  (``GenerateDatabaseInfo.py:23-25`` resizes to width 1500);
* queries for a 1000x800 query image: a fraction are *planted* -- a noisy copy
  of a DB descriptor whose keypoint is a similarity transform (scale 2**k,
  rotation, translation, N(0, 0.5 px) noise) of the model keypoint for one of
  ``n_objects`` objects -- and the rest are independent.

Every image is generated from ``default_rng([seed, image_id])`` so a DB shard
can be generated on its own rank and is bit-identical to the same rows of the
full DB.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from .database import DESC_DIM, Keypoints, SiftDatabase, centroid_of

DB_WIDTH = 1500
DB_HEIGHT_RANGE = (800, 1200)
QUERY_SHAPE = (800, 1000, 3)   # rgb_query.shape of a 1000x800 query image


def sift_like_descriptors(rng, n):
    g = rng.standard_normal((n, DESC_DIM)) ** 2
    g /= np.linalg.norm(g, axis=1, keepdims=True) + 1e-12
    np.minimum(g, 0.2, out=g)
    g *= 512.0 / (np.linalg.norm(g, axis=1, keepdims=True) + 1e-12)
    return np.clip(np.rint(g), 0, 255).astype(np.uint8)


def pack_octave(octave, layer, xi=None):
    """OpenCV SIFT packing: byte0 = octave (signed), byte1 = layer, byte2 = xi."""
    o = np.asarray(octave, np.int64) & 0xFF
    p = o | ((np.asarray(layer, np.int64) & 0xFF) << 8)
    if xi is not None:
        p |= (np.asarray(xi, np.int64) & 0xFF) << 16
    return p.astype(np.int32)


def _image(seed, image_id, kp_per_image, descriptors=True):
    rng = np.random.default_rng([seed, image_id, 1])        # geometry stream
    w = DB_WIDTH
    h = int(rng.integers(DB_HEIGHT_RANGE[0], DB_HEIGHT_RANGE[1] + 1))
    des = (sift_like_descriptors(np.random.default_rng([seed, image_id, 0]), kp_per_image)
           if descriptors else None)
    x = rng.uniform(0, w, kp_per_image).astype(np.float32)
    y = rng.uniform(0, h, kp_per_image).astype(np.float32)
    ang = rng.uniform(0, 360, kp_per_image).astype(np.float32)
    octv = rng.integers(-1, 4, kp_per_image)
    layer = rng.integers(1, 4, kp_per_image)
    xi = rng.integers(0, 256, kp_per_image)
    return des, x, y, ang, pack_octave(octv, layer, xi), (w, h)


def make_database(n_images, kp_per_image=1000, seed=0, first_image=0, descriptors=True,
                  workers=1):
    """Images ``[first_image, first_image + n_images)`` of the seeded DB.  With
    ``descriptors=False`` only the keypoints / image table are generated (the other ranks'
    part of the replicated keypoint table); ``des`` is then an empty [0,128] array.
    ``workers`` > 1 generates images on that many threads (numpy releases the GIL in the
    per-image generators and ufuncs); every image has its own seed, so the result is the
    same bit for bit."""
    ids = range(first_image, first_image + n_images)
    if workers > 1 and n_images > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(workers) as ex:
            parts = list(ex.map(lambda i: _image(seed, i, kp_per_image, descriptors), ids))
    else:
        parts = [_image(seed, i, kp_per_image, descriptors) for i in ids]
    des, xs, ys, angs, octs, imgs, cents, sizes = [], [], [], [], [], [], [], []
    for i, (d, x, y, a, o, wh) in zip(ids, parts):
        des.append(d); xs.append(x); ys.append(y); angs.append(a); octs.append(o)
        imgs.append(np.full(kp_per_image, i - first_image, np.int32))
        cents.append(centroid_of(x, y))
        sizes.append(wh)
    kp = Keypoints(np.concatenate(xs), np.concatenate(ys), np.concatenate(angs),
                   np.concatenate(octs))
    if not descriptors:
        return kp, np.concatenate(imgs), np.array(cents, np.float64), np.array(sizes, np.int32)
    return SiftDatabase(np.concatenate(des), kp, np.concatenate(imgs),
                        np.array(cents, np.float64), np.array(sizes, np.int32))


@dataclass
class QuerySet:
    des: np.ndarray          # uint8 [Nq,128]
    kp: Keypoints
    shape: tuple             # rgb_query.shape
    planted_db_row: np.ndarray   # int64 [Nq], -1 if independent
    planted_object: np.ndarray   # int32 [Nq], -1 if independent

    def __len__(self):
        return int(self.des.shape[0])


def make_queries(n_queries, seed=1, db_seed=0, kp_per_image=1000, planted_frac=0.2,
                 n_objects=4, shape=QUERY_SHAPE, decoy_frac=0.05):
    """Queries against the DB of ``make_database(seed=db_seed, ...)``; the
    planted ones copy rows of DB images ``0..n_objects-1`` (regenerated here,
    so the full DB is not needed).  ``decoy_frac`` of the queries copy a DB
    row of those images but keep a random keypoint: they pass the ratio test
    and scatter votes over the pose space, like real SIFT mismatches."""
    rng = np.random.default_rng(seed)
    h, w = shape[0], shape[1]
    objs = [_image(db_seed, j, kp_per_image) for j in range(n_objects)]
    cents = [centroid_of(o[1], o[2]) for o in objs]
    obj_k = rng.integers(0, 2, n_objects)                   # scale 2**k
    obj_theta = rng.uniform(0, 360, n_objects)
    obj_t = np.stack([rng.uniform(0.15 * w, 0.85 * w, n_objects),
                      rng.uniform(0.15 * h, 0.85 * h, n_objects)], 1)

    n_pl = int(round(planted_frac * n_queries))
    des = sift_like_descriptors(rng, n_queries)
    x = rng.uniform(0, w, n_queries).astype(np.float32)
    y = rng.uniform(0, h, n_queries).astype(np.float32)
    ang = rng.uniform(0, 360, n_queries).astype(np.float32)
    octv = rng.integers(-1, 4, n_queries)
    layer = rng.integers(1, 4, n_queries)
    octave = pack_octave(octv, layer, rng.integers(0, 256, n_queries))
    row = np.full(n_queries, -1, np.int64)
    objid = np.full(n_queries, -1, np.int32)

    n_dec = int(round(decoy_frac * n_queries))
    perm = rng.permutation(n_queries)
    slots = perm[:n_pl]
    for s in perm[n_pl:n_pl + n_dec]:
        j = int(rng.integers(0, n_objects))
        m = int(rng.integers(0, kp_per_image))
        noise = rng.integers(-3, 4, DESC_DIM)
        des[s] = np.clip(objs[j][0][m].astype(np.int64) + noise, 0, 255).astype(np.uint8)
        row[s] = j * kp_per_image + m
    for s in slots:
        j = int(rng.integers(0, n_objects))
        m = int(rng.integers(0, kp_per_image))
        d, mx, my, ma, mo, _ = objs[j]
        noise = rng.integers(-3, 4, DESC_DIM)
        des[s] = np.clip(d[m].astype(np.int64) + noise, 0, 255).astype(np.uint8)
        k = int(obj_k[j])
        th = math.radians(obj_theta[j])
        sig = 2.0 ** k
        dx, dy = float(mx[m]) - cents[j][0], float(my[m]) - cents[j][1]
        px = obj_t[j, 0] + sig * (math.cos(th) * dx - math.sin(th) * dy) + rng.normal(0, 0.5)
        py = obj_t[j, 1] + sig * (math.sin(th) * dx + math.cos(th) * dy) + rng.normal(0, 0.5)
        x[s], y[s] = px, py
        ang[s] = np.float32((float(ma[m]) + obj_theta[j]) % 360.0)
        mo_i = int(mo[m])
        o_m = mo_i & 0xFF
        o_m = o_m - 256 if o_m >= 128 else o_m
        octave[s] = (mo_i & ~0xFF) | ((o_m + k) & 0xFF)
        row[s] = j * kp_per_image + m
        objid[s] = j
    return QuerySet(des, Keypoints(x, y, ang, octave), tuple(shape), row, objid)


def textured_image(h, w, seed=0, n_blobs=None, n_rects=None):
    """Seeded 8-bit gray test image with SIFT structure at several scales: a smooth
    gradient, random rectangles (corners, edges), Gaussian blobs of radii 1.5-24 px and
    mild noise.  For the SIFT row: no image files are needed."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    img = 60.0 + 40.0 * (xx / max(w, 1)) + 30.0 * (yy / max(h, 1))
    n_rects = n_rects if n_rects is not None else max(4, (h * w) // 6000)
    for _ in range(n_rects):
        x0, y0 = rng.integers(0, w), rng.integers(0, h)
        rw, rh = rng.integers(4, max(5, w // 6)), rng.integers(4, max(5, h // 6))
        img[y0:y0 + rh, x0:x0 + rw] += rng.uniform(-50, 50)
    n_blobs = n_blobs if n_blobs is not None else max(8, (h * w) // 300)
    cx = rng.uniform(0, w, n_blobs)
    cy = rng.uniform(0, h, n_blobs)
    rad = np.exp(rng.uniform(np.log(1.5), np.log(24.0), n_blobs))
    amp = rng.uniform(-90, 90, n_blobs)
    for x0, y0, r, a in zip(cx, cy, rad, amp):
        k = int(3 * r) + 1
        xa, xb = max(0, int(x0) - k), min(w, int(x0) + k + 1)
        ya, yb = max(0, int(y0) - k), min(h, int(y0) + k + 1)
        if xa >= xb or ya >= yb:
            continue
        gx = np.exp(-((np.arange(xa, xb) - x0) ** 2) / (2 * r * r))
        gy = np.exp(-((np.arange(ya, yb) - y0) ** 2) / (2 * r * r))
        img[ya:yb, xa:xb] += a * np.outer(gy, gx)
    img += rng.normal(0, 2.0, img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)
