"""Drop-in for ``PoseBin.py``: the state of one Hough pose bin.

The attribute names and the method names are the reference's (``PoseBin.py:4-85``) because
the post-processing and visualisation code read them (``PostProcessing.py:22-28,48-49,
98-106``, ``VisualHelperFunctions.py:7-11``).  The device pipeline computes every bin's
votes, members and running means in one pass (hough.hip: ``hist_kernel``, ``member_*``,
``means_kernel``) and builds these objects only when a caller asks for them
(``pipeline.Main``); the update methods here are for callers that drive a bin by hand.

Arithmetic contract (what the device's ``means_kernel`` reproduces bit for bit): each
quantity q of a bin with n votes moves to ``(q * n + new) / (n + 1)`` -- one f64 multiply,
one add, one correctly rounded divide, in that order (``PoseBin.py:19-43``).
"""
from __future__ import annotations

import numpy as np


def _running_mean(old, new, n):
    """One step of the reference's running mean: ``(old*n + new)/(n+1)`` (not fused)."""
    return (old * n + new) / (n + 1)


def _pair_mean(old, new, n):
    return (_running_mean(old[0], new[0], n), _running_mean(old[1], new[1], n))


class PoseBin:
    """One (i_x, i_y, i_theta, i_sigma) bin.

    ``centroid``/``angle``/``scale`` are the running means of the object poses voted into
    the bin, ``img_size`` the running mean of the voting model images' (w, h);
    ``keypoint_pairs`` the voting (model kp, query kp, ...) tuples in vote order;
    ``affine_parameters`` is filled by ``affine.AffineParameters``.
    """

    __hash__ = None   # the reference defines __eq__ only, which makes bins unhashable

    def __init__(self, pose, img_size=(100, 100), votes=0, keypoint_pairs=None,
                 mean=(0, 0, 0, 0)):
        # the reference's default `keypoint_pairs=[]` is one list shared by every bin
        # built without pairs; main.py always passes its own list, so a fresh one is kept
        self._lazy = None       # (pair_of, member query indices): pairs built on first read
        self._dev = None        # device binding, see bind_device
        self.keypoint_pairs = [] if keypoint_pairs is None else keypoint_pairs
        self.pose, self.img_size, self.votes = pose, img_size, votes
        self.centroid = (mean[0], mean[1])
        self.angle, self.scale = mean[2], mean[3]
        self.affine_parameters = []

    # ---- members resident on the device (pipeline.Main) ---------------------------------
    @property
    def keypoint_pairs(self):
        if self._lazy is not None:
            pair_of, members = self._lazy
            self._lazy = None
            self._pairs = [pair_of(int(q)) for q in members]
            if self._dev is not None:          # what the device holds, to detect edits
                self._dev = self._dev[:3] + (list(self._pairs),)
        return self._pairs

    @keypoint_pairs.setter
    def keypoint_pairs(self, pairs):
        self._pairs = pairs
        self._lazy = None
        self._dev = None        # the caller's own list: the device copy no longer applies

    def bind_device(self, token, index, members, pair_of):
        """The bin is valid bin ``index`` of the device selection ``token`` with member
        queries ``members``; its keypoint pairs are built from them on first read."""
        if self._dev is None and self._lazy is None and self._pairs:
            snap = list(self._pairs)           # already built: keep the objects
        else:
            snap = None
            self._pairs = []
            self._lazy = (pair_of, members)
        self._dev = (token, index, members, snap)
        self._dev_pose, self._dev_votes = self.pose, len(members)

    def device_index(self, token):
        """The bin's index in device selection ``token`` when the device copy still equals
        the bin (members, votes, pose unchanged by the caller), else None."""
        d = self._dev
        if d is None or d[0] != token or self.pose != self._dev_pose or self.votes != self._dev_votes:
            return None
        if self._lazy is None:                 # built: still exactly those objects?
            snap = d[3]
            if snap is None or len(snap) != len(self._pairs) or any(
                    a is not b for a, b in zip(snap, self._pairs)):
                return None
        return d[1]

    def keep_device_members(self, alive, kept=None):
        """After a device step on the bound members (the affine outlier removal): keep the
        members where ``alive`` (bool, member order) -- built objects stay the same objects,
        unbuilt ones stay lazy.  ``kept``: the surviving members, when the caller selected
        them for many bins at once."""
        _, _, members, snap = self._dev
        if self._lazy is None:
            self._pairs = [p for p, k in zip(self._pairs, np.asarray(alive, bool)) if k]
        else:
            if kept is None:
                kept = np.asarray(members)[np.asarray(alive, bool)]
            self._lazy = (self._lazy[0], kept)
        self._dev = None

    # ---- per-vote updates (PoseBin.py:19-54) --------------------------------------------
    def update_centroid(self, center):
        self.centroid = _pair_mean(self.centroid, center, self.votes)

    def update_angle(self, alpha):
        self.angle = _running_mean(self.angle, alpha, self.votes)

    def update_scale(self, scale):
        self.scale = _running_mean(self.scale, scale, self.votes)

    def update_img_size(self, img_size):
        self.img_size = _pair_mean(self.img_size, img_size, self.votes)

    def update_posebin(self, object_pose, img_size, keypoint_pair):
        """One vote: every mean moves with the OLD count, then the pair is appended and the
        count incremented (the reference's order, ``PoseBin.py:45-51``)."""
        x, y, alpha, s = object_pose[:4]
        self.update_centroid((x, y))
        self.update_angle(alpha)
        self.update_scale(s)
        self.update_img_size(img_size)
        self.add_keypoint_pair(keypoint_pair)
        self.add_vote()

    def add_vote(self, new_votes=1):
        self.votes += new_votes

    # ---- members ------------------------------------------------------------------------
    def add_keypoint_pair(self, pair):
        self.keypoint_pairs.append(pair)

    def remove_keypoint_pair(self, pair):
        self.keypoint_pairs.remove(pair)

    def get_pts(self):
        """(query x, query y, model x, model y) as f64 arrays in member order."""
        n = len(self.keypoint_pairs)
        pts = np.empty((4, n), np.float64)
        for j, pair in enumerate(self.keypoint_pairs):
            pts[0:2, j] = pair[1].pt
            pts[2:4, j] = pair[0].pt
        return pts[0], pts[1], pts[2], pts[3]

    # ---- identity -----------------------------------------------------------------------
    def is_same_pose(self, pose):
        return self.pose == pose

    def __eq__(self, other):
        return isinstance(other, PoseBin) and self.pose == other.pose

    def __repr__(self):
        return f"[{self.pose}, {self.votes}, {self.img_size}]"

    def __str__(self):
        return f"Pose: {self.pose}"
