"""Drop-in for ``AffineParameters.py``: per-bin affine least squares and outlier removal,
evaluated by the device kernel (hough.hip ``affine_kernel``).

``AffineParameters(posebin)`` solves x = pinv(A^T A) A^T b (``AffineParameters.py:49-55``)
as two decoupled 3x3 normal-equation systems with the same pseudo-inverse cutoff as
numpy (rcond 1e-15 of the largest singular value) -- A^T A of the reference is exactly
block-diagonal with two copies of G = sum [x y 1]^T [x y 1].  ``remove_outliers``
applies the reference's tolerance (image size x scale-bin INDEX / factor,
``AffineParameters.py:120-121``).  ``Gen_A``/``Gen_b``/``Ext_Params`` are the reference's
list builders, kept for API compatibility.
"""
from __future__ import annotations

import numpy as np

from . import _lib


def Gen_A(x, y, votes):
    """``AffineParameters.py:11-20``."""
    A = []
    for k in range(0, votes):
        A.append([x[k], y[k], 0, 0, 1, 0])
        A.append([0, 0, x[k], y[k], 0, 1])
    return A


def Gen_b(b_x, b_y, votes):
    """``AffineParameters.py:31-39``."""
    b = []
    for k in range(0, votes):
        b.append(b_x[k])
        b.append(b_y[k])
    return b


def Ext_Params(x):
    """``AffineParameters.py:69-76``."""
    return x[0], x[1], x[2], x[3], x[4], x[5]


def Calc_x(A, b, ctx=None):
    """``AffineParameters.py:49-55`` for an A built by :func:`Gen_A` (rows
    [x, y, 0, 0, 1, 0] / [0, 0, x, y, 0, 1]): solved on the device."""
    A = np.asarray(A, np.float64).reshape(-1, 6)
    b = np.asarray(b, np.float64).reshape(-1)
    if len(A) % 2 or not (np.all(A[0::2, 2:4] == 0) and np.all(A[0::2, 4] == 1)
                          and np.all(A[1::2, 0:2] == 0) and np.all(A[1::2, 5] == 1)
                          and np.array_equal(A[0::2, 0:2], A[1::2, 2:4])):
        raise ValueError("Calc_x expects the A matrix of Gen_A")
    mx, my = A[0::2, 0], A[0::2, 1]
    r = _solve([(mx, my, b[0::2], b[1::2])], [0], (1, 1), 1.0, 1.0, 0, 0, None, ctx)
    return np.array(r["params"][0])


def _solve(bins_pts, i_sigma, query_size, xf, yf, thr, max_iter, params_in, ctx):
    ctx = ctx or _lib.default_context()
    off = np.zeros(len(bins_pts) + 1, np.int64)
    for i, p in enumerate(bins_pts):
        off[i + 1] = off[i] + len(p[0])
    cat = [np.concatenate([np.asarray(p[j], np.float64) for p in bins_pts]).astype(np.float32)
           if len(bins_pts) else np.zeros(0, np.float32) for j in range(4)]
    return ctx.affine_batch(off, cat[0], cat[1], cat[2], cat[3], np.asarray(i_sigma, np.int32),
                            query_size, xf, yf, thr, max_iter, params_in)


def _points(posebin):
    kp = posebin.keypoint_pairs[:posebin.votes]
    mx = [p[0].pt[0] for p in kp]
    my = [p[0].pt[1] for p in kp]
    qx = [p[1].pt[0] for p in kp]
    qy = [p[1].pt[1] for p in kp]
    return mx, my, qx, qy


def AffineParameters(posebin, ctx=None):
    """``AffineParameters.py:89-113``: sets ``posebin.affine_parameters``; no-op when
    the bin has no votes."""
    if posebin.votes <= 0:
        return
    r = _solve([_points(posebin)], [posebin.pose[3]], (1, 1), 1.0, 1.0, 0, 0, None, ctx)
    posebin.affine_parameters = [float(v) for v in r["params"][0]]


def remove_outliers(posebin, image_query_size, x_factor=8, y_factor=8, ctx=None):
    """``AffineParameters.py:116-160``: drops keypoint pairs whose affine prediction is
    off by more than image_size * pose[3] / factor; returns (posebin, changed)."""
    n = len(posebin.keypoint_pairs)
    if n == 0:
        return posebin, False
    prm = np.asarray(posebin.affine_parameters, np.float64).reshape(1, 6)
    kp = posebin.keypoint_pairs
    pts = ([p[0].pt[0] for p in kp], [p[0].pt[1] for p in kp],
           [p[1].pt[0] for p in kp], [p[1].pt[1] for p in kp])
    r = _solve([pts], [posebin.pose[3]], image_query_size, float(x_factor), float(y_factor),
               0, 1, prm, ctx)
    keep = r["alive"]
    posebin.keypoint_pairs = [v for v, k in zip(kp, keep) if k]
    posebin.votes = len(posebin.keypoint_pairs)
    return posebin, bool((~keep).any())


def verify_bins(posebins, image_query_size, threshold=4, x_factor=128, y_factor=128, ctx=None):
    """Batched ``Main.apply_affine_parameters`` (main.py:139-157) over a list of PoseBins:
    the per-bin fixed point of {AffineParameters; remove_outliers} on the device, all bins
    in one launch.  Mutates the bins like the reference and returns the survivors."""
    if not posebins:
        return []
    pts = [(
        [p[0].pt[0] for p in b.keypoint_pairs], [p[0].pt[1] for p in b.keypoint_pairs],
        [p[1].pt[0] for p in b.keypoint_pairs], [p[1].pt[1] for p in b.keypoint_pairs])
        for b in posebins]
    r = _solve(pts, [b.pose[3] for b in posebins], image_query_size, float(x_factor),
               float(y_factor), int(threshold), 1 << 30, None, ctx)
    out = []
    pos = 0
    for i, b in enumerate(posebins):
        n = len(b.keypoint_pairs)
        keep = r["alive"][pos:pos + n]
        pos += n
        b.keypoint_pairs = [v for v, k in zip(b.keypoint_pairs, keep) if k]
        b.votes = len(b.keypoint_pairs)
        b.affine_parameters = [float(v) for v in r["params"][i]]
        if r["survived"][i]:
            out.append(b)
    return out
