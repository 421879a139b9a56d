"""Drop-in for ``PoseBin.py``: the state of one Hough pose bin.

Same attributes and methods as the reference (``PoseBin.py:4-85``) because the
post-processing and visualisation code read them (``PostProcessing.py:22-28,48-49,98-106``,
``VisualHelperFunctions.py:7-11``).  The device pipeline computes the bins' votes, members
and running means in one pass (hough.hip) and materialises PoseBin objects only when
they are asked for; the per-vote update methods below are the reference's arithmetic for
callers that drive a PoseBin by hand.
"""
from __future__ import annotations

import numpy as np


class PoseBin:

    def __init__(self, pose, img_size=(100, 100), votes=0, keypoint_pairs=None,
                 mean=(0, 0, 0, 0)):
        self.pose = pose                  # (i_x, i_y, i_theta, i_sigma)
        self.img_size = img_size          # (width, height) running mean
        self.votes = votes
        self.keypoint_pairs = [] if keypoint_pairs is None else keypoint_pairs
        self.centroid = mean[0], mean[1]
        self.angle = mean[2]
        self.scale = mean[3]
        self.affine_parameters = []

    def add_keypoint_pair(self, pair):
        self.keypoint_pairs.append(pair)

    def update_centroid(self, center):                    # PoseBin.py:19-25
        n = self.votes
        self.centroid = ((self.centroid[0] * n + center[0]) / (n + 1),
                         (self.centroid[1] * n + center[1]) / (n + 1))

    def update_angle(self, alpha):                        # PoseBin.py:27-30
        self.angle = (self.angle * self.votes + alpha) / (self.votes + 1)

    def update_scale(self, scale):                        # PoseBin.py:32-35
        self.scale = (self.scale * self.votes + scale) / (self.votes + 1)

    def update_img_size(self, img_size):                  # PoseBin.py:37-43
        n = self.votes
        self.img_size = ((self.img_size[0] * n + img_size[0]) / (n + 1),
                         (self.img_size[1] * n + img_size[1]) / (n + 1))

    def update_posebin(self, object_pose, img_size, keypoint_pair):   # PoseBin.py:45-51
        self.update_centroid((object_pose[0], object_pose[1]))
        self.update_angle(object_pose[2])
        self.update_scale(object_pose[3])
        self.update_img_size(img_size)
        self.add_keypoint_pair(keypoint_pair)
        self.add_vote()

    def add_vote(self, new_votes=1):
        self.votes += new_votes

    def get_pts(self):                                    # PoseBin.py:56-67
        if not self.keypoint_pairs:
            e = np.array([])
            return e, e.copy(), e.copy(), e.copy()
        q = np.array([p[1].pt for p in self.keypoint_pairs], np.float64)
        m = np.array([p[0].pt for p in self.keypoint_pairs], np.float64)
        return q[:, 0], q[:, 1], m[:, 0], m[:, 1]

    def remove_keypoint_pair(self, pair):
        self.keypoint_pairs.remove(pair)

    def is_same_pose(self, pose):
        return pose == self.pose

    def __eq__(self, other):
        if isinstance(other, PoseBin):
            return other.pose == self.pose
        return False

    __hash__ = None   # like the reference (defines __eq__ only)

    def __repr__(self):
        return "[" + str(self.pose) + ", " + str(self.votes) + ", " + str(self.img_size) + "]"

    def __str__(self):
        return "Pose: " + str(self.pose)
