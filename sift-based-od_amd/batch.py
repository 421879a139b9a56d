"""Query batching: several query images share ONE matcher pass
over the DB, then each image runs its own Hough / valid-bin / affine / post-processing
stages on its query range (``sod_query_window``).  The reference processes one query
image per ``Main`` run (``main.py:178-188``); matching dominates and a small image leaves
most of the chip idle, so batching amortises the DB stream."""
from __future__ import annotations

import numpy as np

from .database import Keypoints

POS_FACTOR = 32    # main.py:141


def run_query_batch(ctx, images, bins=15, ratio=0.75, vote_threshold=5, affine_threshold=4,
                    post_process=True, results=True):
    """``images``: list of ``(descriptors [n,128], Keypoints, rgb_query.shape)``.  Returns a
    list of per-image dicts (matches, valid bins, affine survivors, post-processing) with
    image-local query indices; ``results=False`` leaves them on the device (timing)."""
    des = np.concatenate([np.asarray(d) for d, _, _ in images], axis=0)
    kps = [k for _, k, _ in images]
    kp = Keypoints(np.concatenate([k.x for k in kps]), np.concatenate([k.y for k in kps]),
                   np.concatenate([k.angle for k in kps]), np.concatenate([k.octave for k in kps]))
    ctx.upload_queries(des, kp)
    ctx.match()
    ctx.ratio(ratio)
    out = []
    lo = 0
    for d, _, shape in images:
        n = len(d)
        ctx.query_window(lo, n)
        ctx.hough(shape, bins)
        ctx.select(vote_threshold)
        ctx.affine((shape[1], shape[0]), POS_FACTOR * 4.0, POS_FACTOR * 4.0, affine_threshold)
        if results:
            r = {"valid": ctx.valid_result(), "affine": ctx.affine_result()}
            if post_process:
                r["post"] = ctx.postprocess()
            out.append(r)
        lo += n
    if results:
        idx1, d1, d2, good = ctx.match_result()
        lo = 0
        for (d, _, _), r in zip(images, out):
            n = len(d)
            r.update(idx1=idx1[lo:lo + n], d1=d1[lo:lo + n], d2=d2[lo:lo + n],
                     good=good[lo:lo + n])
            lo += n
    ctx.query_window()
    return out
