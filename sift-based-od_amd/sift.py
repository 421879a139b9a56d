"""SIFT detect + describe on the device, drop-in for the OpenCV
calls the reference makes:

    sift = cv2.SIFT_create()                                  # main.py:179, GenerateDatabaseInfo.py:16
    kp, des = sift.detectAndCompute(gray, None)               # main.py:43, GenerateDatabaseInfo.py:32

``SIFT_create(...)`` returns an object whose ``detectAndCompute`` returns a tuple of
``KeyPoint`` objects (``pt``, ``size``, ``angle``, ``response``, ``octave``, ``class_id``
-- the fields ``make_temp_kp`` / ``unpack_sift_octave`` read, SiftHelperFunctions.py:16-40)
and a float32 [n, 128] descriptor array (integer-valued, as OpenCV's), or ``None`` when
the image has no keypoints.  The whole pipeline runs in libsod (``csrc/sift.hip``); the
arrays form (``detect_arrays``) skips the per-keypoint Python objects, and
``Context.sift_to_queries`` hands the result to the matcher without leaving the device.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .sift_helpers import KeyPoint


def keypoints_from_arrays(r):
    return tuple(KeyPoint(x, y, s, a, resp, o) for x, y, s, a, resp, o in zip(
        r["x"].tolist(), r["y"].tolist(), r["size"].tolist(), r["angle"].tolist(),
        r["response"].tolist(), r["octave"].tolist()))


def _retain_best(r, n_points):
    """KeyPointsFilter::retainBest: keep every keypoint whose response reaches the
    n-th largest (OpenCV keeps the same set; its order after nth_element is unspecified,
    here the detection order is kept)."""
    n = len(r["x"])
    if n_points <= 0 or n <= n_points:
        return r
    thr = np.sort(r["response"])[::-1][n_points - 1]
    keep = r["response"] >= thr
    return {k: v[keep] for k, v in r.items()}


class SIFT:
    """``cv2.SIFT`` on the device.  One libsod context (GPU) per instance unless ``ctx``
    is given."""

    def __init__(self, nfeatures=0, nOctaveLayers=3, contrastThreshold=0.04,  # noqa: N803
                 edgeThreshold=10.0, sigma=1.6, ctx=None):
        self.nfeatures = int(nfeatures)
        self._ctx = ctx if ctx is not None else _lib.default_context()
        self._ctx.sift_params(nOctaveLayers, contrastThreshold, edgeThreshold, sigma)
        self._params = (nOctaveLayers, contrastThreshold, edgeThreshold, sigma)

    @property
    def context(self):
        return self._ctx

    def detect_arrays(self, image, descriptors=True):
        """SoA keypoints (x, y, size, angle, response, octave) + ``descriptors``."""
        self._ctx.sift_params(*self._params)   # the context may be shared
        r = self._ctx.sift_detect(image, descriptors=descriptors)
        return _retain_best(r, self.nfeatures)

    def detect_batch(self, images, descriptors=True):
        """detect_arrays of several images (four in flight on the device)."""
        self._ctx.sift_params(*self._params)
        return [_retain_best(r, self.nfeatures)
                for r in self._ctx.sift_detect_batch(images, descriptors=descriptors)]

    def detectAndCompute(self, image, mask, descriptors=None,   # noqa: N802
                         useProvidedKeypoints=False):           # noqa: N803
        if mask is not None:
            raise NotImplementedError("SIFT masks are not supported (the reference passes None)")
        if useProvidedKeypoints:
            raise NotImplementedError("useProvidedKeypoints is not supported")
        r = self.detect_arrays(image, descriptors=True)
        kp = keypoints_from_arrays(r)
        return kp, (r["descriptors"] if len(kp) else None)

    def detect(self, image, mask=None):
        if mask is not None:
            raise NotImplementedError("SIFT masks are not supported (the reference passes None)")
        return keypoints_from_arrays(self.detect_arrays(image, descriptors=False))

    def descriptorSize(self):  # noqa: N802
        return 128


def SIFT_create(nfeatures=0, nOctaveLayers=3, contrastThreshold=0.04,  # noqa: N802,N803
                edgeThreshold=10.0, sigma=1.6, ctx=None):
    return SIFT(nfeatures, nOctaveLayers, contrastThreshold, edgeThreshold, sigma, ctx)


def bgr_to_gray(bgr):
    """cv2.cvtColor(img, COLOR_BGR2GRAY) for 8-bit images (main.py:41), on the host:
    (B*1868 + G*9617 + R*4899 + 2^13) >> 14."""
    b = np.asarray(bgr, np.uint8)[..., :3].astype(np.int32)
    return ((b[..., 0] * 1868 + b[..., 1] * 9617 + b[..., 2] * 4899 + (1 << 13)) >> 14).astype(
        np.uint8)
