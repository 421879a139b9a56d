"""Query batching: several query images share ONE matcher pass
over the DB, then each image runs its own Hough / valid-bin / affine / post-processing
stages on its query range (``sod_query_window``).  The reference processes one query
image per ``Main`` run (``main.py:178-188``); matching dominates and a small image leaves
most of the chip idle, so batching amortises the DB stream."""
from __future__ import annotations

import numpy as np

from .database import Keypoints
from .constants import REFERENCE

POS_FACTOR = REFERENCE.pos_factor   # main.py:141


def run_query_batch(ctx, images, bins=15, ratio=0.75, vote_threshold=5, affine_threshold=4,
                    post_process=True, results=True, fused=True):
    """``images``: list of ``(descriptors [n,128], Keypoints, rgb_query.shape)``.  Returns a
    list of per-image dicts (matches, valid bins, affine survivors, post-processing) with
    image-local query indices; ``results=False`` leaves them on the device (timing).

    ``fused``: one launch per stage for the whole batch (``sod_query_images``: image-major
    bin keys); otherwise the stages run image by image on query windows."""
    des = np.concatenate([np.asarray(d) for d, _, _ in images], axis=0)
    kps = [k for _, k, _ in images]
    kp = Keypoints.concat(kps)
    ctx.upload_queries(des, kp)
    ctx.match()
    ctx.ratio(ratio)
    if fused:
        return _fused(ctx, images, bins, vote_threshold, affine_threshold, post_process, results)
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


def sift_query_batch(ctx, images, bins=15, ratio=0.75, vote_threshold=5, affine_threshold=4,
                     post_process=True, results=True):
    """Query IMAGES end to end on the device (SURVEY 8(f) rows 3 + 4): SIFT of every image
    (``main.py:36-45``, four in flight), ONE matcher pass over the DB for all their
    features, then the fused per-image Hough / valid-bin / affine / post-processing stages.
    ``images``: 8-bit gray [h, w] or BGR [h, w, 3] arrays (``cv2.imread`` output).  Returns
    the per-image dicts of :func:`run_query_batch` plus each image's keypoint count."""
    counts = ctx.sift_detect_batch(images, results=False)
    if int(np.sum(counts)) == 0:
        raise ValueError("no SIFT keypoints in the batch")
    ctx.sift_to_queries()          # also declares the images (offsets, shapes) when > 1
    ctx.match()
    ctx.ratio(ratio)
    shapes = [tuple(np.shape(im)[:2]) + (3,) for im in images]
    out = _fused_sizes(ctx, [int(c) for c in counts], shapes, bins, vote_threshold,
                       affine_threshold, post_process, results)
    for r, c in zip(out, counts):
        r["n_keypoints"] = int(c)
    return out


def _fused(ctx, images, bins, vote_threshold, affine_threshold, post_process, results):
    return _fused_sizes(ctx, [len(d) for d, _, _ in images], [s for _, _, s in images], bins,
                        vote_threshold, affine_threshold, post_process, results)


def _fused_sizes(ctx, sizes, shapes, bins, vote_threshold, affine_threshold, post_process,
                 results):
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    ctx.query_images(off, shapes)
    ctx.hough((1, 1), bins)
    ctx.select(vote_threshold)
    ctx.affine((1, 1), POS_FACTOR * 4.0, POS_FACTOR * 4.0, affine_threshold)
    out = []
    if results:
        res = ctx.results(post=post_process)   # one transfer, one wait (sod_results_fetch)
        v, a = res["valid"], res["affine"]
        img = ctx.valid_images()
        post = res.get("post")
        idx1, d1, d2, good = res["match"]
        for b in range(len(sizes)):
            lo, hi = int(off[b]), int(off[b + 1])
            sel = np.nonzero(img == b)[0]
            vo = v["offsets"]
            mem = [v["members"][vo[i]:vo[i + 1]] - lo for i in sel]
            counts = np.array([len(m) for m in mem], np.int64)
            r = {"idx1": idx1[lo:hi], "d1": d1[lo:hi], "d2": d2[lo:hi], "good": good[lo:hi],
                 "valid": {"keys": v["keys"][sel], "votes": v["votes"][sel],
                           "offsets": np.concatenate([[0], np.cumsum(counts)]).astype(np.int64),
                           "members": (np.concatenate(mem) if mem else np.zeros(0)).astype(np.int32),
                           "means": v["means"][sel]}}
            am = [a["alive"][vo[i]:vo[i + 1]] for i in sel]
            r["affine"] = {"survived": a["survived"][sel], "votes": a["votes"][sel],
                           "params": a["params"][sel],
                           "alive": np.concatenate(am) if am else np.zeros(0, bool)}
            if post is not None:
                r["post"] = _post_for_image(post, img, b, sel)
            out.append(r)
    ctx.query_images([], [])
    return out


def _post_for_image(post, img, b, sel):
    """The fused post-processing result restricted to image b, with bin indices relative to
    the image's own valid-bin list (clusters never span images)."""
    local = {int(v): i for i, v in enumerate(sel)}
    bi = post["bin_index"]
    keep_bins = [k for k in range(len(bi)) if img[bi[k]] == b]
    pos_off, pos_mem, pose, orient = [0], [], [], []
    ori_pos_off, ori_off, ori_mem = [0], [0], []
    kb = {k: j for j, k in enumerate(keep_bins)}
    for c in range(len(post["pos_off"]) - 1):
        members = post["pos_members"][post["pos_off"][c]:post["pos_off"][c + 1]]
        if img[bi[members[0]]] != b:
            continue
        pos_mem.extend(kb[int(m)] for m in members)
        pos_off.append(len(pos_mem))
        for o in range(post["ori_pos_off"][c], post["ori_pos_off"][c + 1]):
            ori_mem.extend(kb[int(m)] for m in post["ori_members"][post["ori_off"][o]:post["ori_off"][o + 1]])
            ori_off.append(len(ori_mem))
        ori_pos_off.append(len(ori_off) - 1)
        pose.append(post["final_pose"][c])
        orient.append(post["final_orientation"][c])
    return {"bin_index": np.array([local[int(bi[k])] for k in keep_bins], np.int32),
            "pos_off": np.array(pos_off, np.int32), "pos_members": np.array(pos_mem, np.int32),
            "ori_pos_off": np.array(ori_pos_off, np.int32), "ori_off": np.array(ori_off, np.int32),
            "ori_members": np.array(ori_mem, np.int32),
            "final_orientation": np.array(orient, np.float64),
            "final_pose": np.array(pose, np.float64).reshape(-1, 6)}
