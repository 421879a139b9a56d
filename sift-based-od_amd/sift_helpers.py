"""Drop-in for ``SiftHelperFunctions.py`` (keypoint helpers).

These are data-format helpers around ``cv2.KeyPoint`` (they run once per image when a
database is built, not on the per-query hot path), so they stay host-side Python.
``unpack_sift_octave`` is also evaluated on the device inside the pose kernel
(hough.hip ``unpack_octave``); this is the same arithmetic for single keypoints.

OpenCV is not required: when ``cv2`` is importable its ``KeyPoint`` is used, otherwise
the minimal :class:`KeyPoint` below (same attribute names and float32 storage).
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - cv2 is absent in this environment
    import cv2 as _cv2
    _CvKeyPoint = _cv2.KeyPoint
except Exception:  # noqa: BLE001
    _cv2 = None
    _CvKeyPoint = None


class KeyPoint:
    """Stand-in for ``cv2.KeyPoint``: ``pt``/``size``/``angle``/``response`` are float32
    fields (cv::Point2f, float) exposed as Python floats; ``octave``/``class_id`` ints."""

    __slots__ = ("pt", "size", "angle", "response", "octave", "class_id")

    def __init__(self, x=0.0, y=0.0, _size=0.0, _angle=-1.0, _response=0.0, _octave=0,
                 _class_id=-1):
        self.pt = (float(np.float32(x)), float(np.float32(y)))
        self.size = float(np.float32(_size))
        self.angle = float(np.float32(_angle))
        self.response = float(np.float32(_response))
        self.octave = int(_octave)
        self.class_id = int(_class_id)

    def __repr__(self):
        return "KeyPoint(pt=%r, angle=%r, octave=%#x)" % (self.pt, self.angle, self.octave)


def new_keypoint(x, y, size=0.0, angle=-1.0, response=0.0, octave=0, class_id=-1):
    if _CvKeyPoint is not None:  # pragma: no cover
        return _CvKeyPoint(x=float(x), y=float(y), size=float(size), angle=float(angle),
                           response=float(response), octave=int(octave),
                           class_id=int(class_id))
    return KeyPoint(x, y, size, angle, response, octave, class_id)


def get_centroid(kp):
    """``SiftHelperFunctions.py:4-14``: sequential double sum / count."""
    x_centroid = 0
    y_centroid = 0
    total = len(kp)
    for point in kp:
        x_centroid = x_centroid + point.pt[0]
        y_centroid = y_centroid + point.pt[1]
    return x_centroid / total, y_centroid / total


def make_temp_kp(kp):
    """``SiftHelperFunctions.py:16-22``: KeyPoint -> picklable tuple."""
    return [(point.pt, point.size, point.angle, point.response, point.octave, point.class_id)
            for point in kp]


def unpack_sift_octave(kpt):
    """``SiftHelperFunctions.py:25-40``: packed octave -> (octave, layer, scale)."""
    _octave = kpt.octave
    octave = _octave & 0xFF
    layer = (_octave >> 8) & 0xFF
    if octave >= 128:
        octave |= -128
    if octave >= 0:
        scale = float(1 / (1 << octave))
    else:
        scale = float(1 << -octave)
    return (octave, layer, scale)


def make_kp(temp_kp):
    """``SiftHelperFunctions.py:42-49``: tuples -> KeyPoint objects."""
    return [new_keypoint(p[0][0], p[0][1], p[1], p[2], p[3], p[4], p[5]) for p in temp_kp]


def keypoints_from_arrays(kp, i):
    """KeyPoint object for row ``i`` of a :class:`~.database.Keypoints` SoA: the caller's own
    object when the table was built from objects, else a new one carrying every field
    (pt, size, angle, response, octave, class_id) as ``make_kp`` builds it."""
    return kp.keypoint(int(i))
