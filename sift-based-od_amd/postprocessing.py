"""Post-processing of the verified pose bins, drop-in for
``PostProcessing.py`` (functions at :4-112) as driven by ``main.py:159-168``.

The pairwise position / orientation relations (the O(n^2) part) are one device kernel
(``post_adjacency_kernel``, ``csrc/post.hip``); the clusters keep the reference's
recursive-DFS visit order, so every later sum and tie matches it.  The functions take
and return PoseBin-like objects (``centroid``, ``angle``, ``scale``, ``img_size``)."""
from __future__ import annotations

import numpy as np

from . import _lib


def _means(bins):
    return np.array([[float(b.centroid[0]), float(b.centroid[1]), float(b.angle),
                      float(b.scale), float(b.img_size[0]), float(b.img_size[1])]
                     for b in bins], np.float64).reshape(-1, 6)


def _ctx(ctx):
    return ctx if ctx is not None else _lib.default_context()


def dfs(i, set, dict, pose_set, valid_bins):  # noqa: A002 -- reference signature
    """``PostProcessing.py:4-11``: depth-first collection of the component of ``i``
    (iterative, same visit order as the reference's recursion)."""
    stack = [(i, 0)]
    if i in set:
        return pose_set
    set.add(i)
    pose_set.append(valid_bins[i])
    while stack:
        node, k = stack[-1]
        nbrs = dict[node]
        while k < len(nbrs) and nbrs[k] in set:
            k += 1
        if k == len(nbrs):
            stack.pop()
            continue
        stack[-1] = (node, k + 1)
        nb = nbrs[k]
        set.add(nb)
        pose_set.append(valid_bins[nb])
        stack.append((nb, 0))
    return pose_set


def _split(objs, off, members):
    return [[objs[k] for k in members[off[c]:off[c + 1]]] for c in range(len(off) - 1)]


def group_position(valid_bins, ctx=None):
    """``PostProcessing.py:14-37``: position clusters (lists of bins, DFS order)."""
    if not len(valid_bins):
        return []
    r = _ctx(ctx).post_batch(_means(valid_bins))
    return _split(list(valid_bins), r["pos_off"], r["pos_members"])


def group_orientation(pose_cluster, ctx=None):
    """``PostProcessing.py:39-62``: per position cluster, its orientation clusters.  The
    clusters are laid out far apart with identical positions inside each, so the device
    pass reproduces each cluster in its given order and groups only by angle."""
    flat, rows = [], []
    for c, cl in enumerate(pose_cluster):
        for b in cl:
            flat.append(b)
            rows.append((c * 1.0e9, 0.0, float(b.angle), 1.0, 1.0, 1.0))
    if not flat:
        return [[] for _ in pose_cluster]
    r = _ctx(ctx).post_batch(np.array(rows, np.float64))
    out = []
    for c in range(len(r["pos_off"]) - 1):
        lo, hi = r["ori_pos_off"][c], r["ori_pos_off"][c + 1]
        out.append([[flat[k] for k in r["ori_members"][r["ori_off"][o]:r["ori_off"][o + 1]]]
                    for o in range(lo, hi)])
    return out


def find_max_orientation(orientation_cluster):
    """``PostProcessing.py:64-81``: mean angle of the last largest orientation cluster."""
    res = []
    for clusters in orientation_cluster:
        max_vote, final = 0, 0
        for comp in clusters:
            if len(comp) >= max_vote:
                max_vote = len(comp)
                final = 0
                for b in comp:
                    final += b.angle
                final = final / len(comp)
        res.append(final)
    return res


def get_final_pose(pose_cluster, final_orientation_list):
    """``PostProcessing.py:85-112``: ((mean x, mean y), orientation, mean scale, img_size
    of the first minimum-area bin) per position cluster."""
    out = []
    for i, cl in enumerate(pose_cluster):
        mx = my = msc = 0
        min_area = float("inf")
        min_shape = 0, 0
        for b in cl:
            mx += b.centroid[0]
            my += b.centroid[1]
            msc += b.scale
            area = (b.img_size[0] * b.scale) * (b.img_size[1] * b.scale)
            if area < min_area:
                min_area = area
                min_shape = b.img_size
        n = len(cl)
        out.append(((mx / n, my / n), final_orientation_list[i], msc / n, min_shape))
    return out


def final_pose_from_arrays(r):
    """The device result's ``final_pose`` rows as main.py's tuples."""
    return [((p[0], p[1]), p[2], p[3], (p[4], p[5])) for p in r["final_pose"].tolist()]
