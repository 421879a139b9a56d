"""sift_based_od_amd -- MI355X-native hot path of torn8to/sift-based-OD.

Brute-force SIFT matching (k=2, Lowe ratio) -> generalized-Hough pose-bin
voting -> per-bin affine least-squares verification, as hand-written HIP
kernels for gfx950 behind a C ABI (``include/sod.h``, ``libsod.so``) that this
package drives through ctypes.  Import through ``sod_pkg.load()`` (the
directory name has hyphens).

Drop-in surface (reference names, reference semantics):

* ``BFMatcher().knnMatch(des_query, des, k=2)``           (``main.py:70-71``)
* ``unpack_sift_octave``, ``get_centroid``, ``make_temp_kp``, ``make_kp``
                                                          (``SiftHelperFunctions.py``)
* ``estimate_object_pose``, ``calculate_bin_index``        (``HoughTransformHelperFunctions.py``)
* ``PoseBin``                                              (``PoseBin.py``)
* ``AffineParameters``, ``remove_outliers``                 (``AffineParameters.py``)
* ``Main`` with ``run_matcher`` / ``apply_hough_transform`` / ``get_valid_bins`` /
  ``apply_affine_parameters``                              (``main.py:17-157``)

The native library is loaded lazily on first use and its absence is an error
(there is no CPU fallback anywhere in this package).
"""
from .database import Keypoints, SiftDatabase, centroid_of  # noqa: F401

__all__ = ["Keypoints", "SiftDatabase", "centroid_of"]
