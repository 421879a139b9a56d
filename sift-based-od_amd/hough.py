"""Drop-in for ``HoughTransformHelperFunctions.py`` (and the per-axis signature of the
old ``HoughTransform.py:8``), evaluated by the device pose kernel (hough.hip).

The per-item functions keep the reference signatures; each call is one small device
launch, so loops over matches should use the ``*_batch`` forms or the fused pipeline
(:class:`~.pipeline.Main`), which computes every match's pose and all 16 votes on the
device without a host round trip.
"""
from __future__ import annotations

import gc

import numpy as np

from . import _lib
from .posebin import PoseBin
from .sift_helpers import unpack_sift_octave  # noqa: F401  (re-export, reference module API)


def _kp_arrays(kps):
    x = np.array([k.pt[0] for k in kps], np.float32)
    y = np.array([k.pt[1] for k in kps], np.float32)
    a = np.array([k.angle for k in kps], np.float32)
    o = np.array([k.octave for k in kps], np.int32)
    return x, y, a, o


def estimate_object_pose_batch(mx, my, mangle, moctave, qx, qy, qangle, qoctave, cx, cy,
                               ctx=None):
    """Poses (x, y, alpha, scale_factor) f64[n,4] for arrays of matched keypoints."""
    ctx = ctx or _lib.default_context()
    pose, _ = ctx.pose_batch(mx, my, mangle, moctave, qx, qy, qangle, qoctave, cx, cy,
                             (1, 1), 1)
    return pose


def estimate_object_pose(data, ctx=None):
    """``HoughTransformHelperFunctions.py:4-37``: ``data`` = (kpM, kpQ, model_size,
    model_centroid) as in ``Main.matching_keypoints``; returns (x, y, alpha, scale)."""
    kpM, kpQ, _, cen = data[0], data[1], data[2], data[3]
    mx, my, ma, mo = _kp_arrays([kpM])
    qx, qy, qa, qo = _kp_arrays([kpQ])
    p = estimate_object_pose_batch(mx, my, ma, mo, qx, qy, qa, qo, [float(cen[0])],
                                   [float(cen[1])], ctx)[0]
    return (float(p[0]), float(p[1]), float(p[2]), float(p[3]))


def calculate_bin_index_batch(poses, bins, query_image_shape, ctx=None):
    """Bin indices int32[n,4] for poses f64[n,4]; ``bins`` int or per-axis 4-tuple."""
    ctx = ctx or _lib.default_context()
    return ctx.bin_index_batch(poses, query_image_shape, bins)


def calculate_bin_index(object_pose, bins, query_image_shape, ctx=None):
    """``HoughTransformHelperFunctions.py:39-72``."""
    idx = calculate_bin_index_batch(np.asarray(object_pose, np.float64).reshape(1, 4), bins,
                                    query_image_shape, ctx)[0]
    return int(idx[0]), int(idx[1]), int(idx[2]), int(idx[3])


def posebins_from_device(res, pair_of, size_of=None, token=None, idx=None):
    """PoseBin objects from a device selection (``Context.valid_result()``): ``pair_of(q)``
    returns the (kpM, kpQ) pair of member query ``q``, called only when a bin's
    ``keypoint_pairs`` is first read (the members stay device arrays until then);
    ``size_of(q)`` the model image size (ints) used when a bin has a single vote (the
    reference keeps the int tuple then).  ``token`` names the device selection the bins
    are bound to (``PoseBin.bind_device``).  ``idx``: only those valid bins (indices into
    the selection, in the given order)."""
    # no cyclic-GC passes while ~10^4 containers are made (they were half the time at C3;
    # none of these objects forms a cycle)
    gc_was_on = gc.isenabled()
    gc.disable()
    try:
        return _posebins(res, pair_of, size_of, token, idx)
    finally:
        if gc_was_on:
            gc.enable()


def _posebins(res, pair_of, size_of, token, idx=None):
    mem = res["members"]
    # Python scalars in bulk (tolist): per-element numpy indexing was ~2 us per bin, 3 ms of
    # main.py's get_valid_bins at C3 (1 163 bins)
    if idx is None:
        sel = range(len(res["votes"]))
        keys = [tuple(k) for k in np.asarray(res["keys"]).tolist()]
        votes = np.asarray(res["votes"]).tolist()
        means = np.asarray(res["means"]).tolist()
    else:
        sel = [int(i) for i in idx]
        keys = [tuple(k) for k in np.asarray(res["keys"])[sel].tolist()]
        votes = np.asarray(res["votes"])[sel].tolist()
        means = np.asarray(res["means"])[sel].tolist()
    off = np.asarray(res["offsets"]).tolist()
    # each bin is PoseBin(key, size, votes, None, mean) + bind_device(token, i, members,
    # pair_of), its attributes set in one dict (the two calls cost ~1 us per bin on the host;
    # tests/test_keypoints.py checks the two constructions give equal objects)
    new = object.__new__
    out = []
    for j, (i, key) in enumerate(zip(sel, keys)):
        a, e = off[i], off[i + 1]
        m = mem[a:e]
        mu = means[j]
        v = votes[j]
        size = size_of(int(mem[a])) if v == 1 and size_of is not None else (mu[4], mu[5])
        b = new(PoseBin)
        b.__dict__ = {"_pairs": [], "_lazy": (pair_of, m), "_dev": (token, i, m, None),
                      "pose": key, "img_size": size, "votes": v, "centroid": (mu[0], mu[1]),
                      "angle": mu[2], "scale": mu[3], "affine_parameters": [],
                      "_dev_pose": key, "_dev_votes": e - a}
        out.append(b)
    return out


def hough_table_from_tuples(matching_keypoints, query_image_shape, bins, vote_threshold=1,
                            ctx=None):
    """Device Hough voting over ``Main.matching_keypoints``-style tuples
    (kpM, kpQ, model_size, model_centroid): each match becomes its own model row and image
    so the tuples' own centroids and sizes are used.  Returns (ctx, [PoseBin]) for the bins
    with >= vote_threshold votes in first-touch order."""
    from .database import Keypoints
    ctx = ctx or _lib.default_context()
    n = len(matching_keypoints)
    mx, my, ma, mo = _kp_arrays([t[0] for t in matching_keypoints])
    qx, qy, qa, qo = _kp_arrays([t[1] for t in matching_keypoints])
    cen = np.array([[float(t[3][0]), float(t[3][1])] for t in matching_keypoints], np.float64)
    size = np.array([[int(t[2][0]), int(t[2][1])] for t in matching_keypoints], np.int32)
    ctx.set_keypoints(Keypoints(mx, my, ma, mo), np.arange(n, dtype=np.int32), cen, size)
    ctx.upload_queries(None, Keypoints(qx, qy, qa, qo))
    ctx.set_matches(np.arange(n, dtype=np.int32), np.ones(n, bool))
    ctx.hough(query_image_shape, bins)
    ctx.select(vote_threshold)
    res = ctx.valid_result()
    bins_ = posebins_from_device(
        res, lambda q: (matching_keypoints[q][0], matching_keypoints[q][1]),
        lambda q: tuple(matching_keypoints[q][2]))
    return ctx, bins_


def perform_hough_transform(matching_keypoints, image_query, bin_x=15, bin_y=15,
                            bin_theta=15, bin_sigma=15, ctx=None):
    """Per-axis Hough transform with the signature of ``HoughTransform.py:8``.  (The
    reference body of that function is dead code that raises; this one computes what the
    live path, ``main.py:89-119``, computes, with one bin count per axis.)  Returns the
    dict {pose: PoseBin} in first-touch order; voting runs on the device."""
    if len(matching_keypoints) == 0:
        return {}
    _, table = hough_table_from_tuples(matching_keypoints, image_query.shape,
                                       (bin_x, bin_y, bin_theta, bin_sigma), 1, ctx)
    return {b.pose: b for b in table}
