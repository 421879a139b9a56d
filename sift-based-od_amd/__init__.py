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
  ``apply_affine_parameters`` / ``post_process``            (``main.py:17-168``)
* ``SIFT_create().detectAndCompute(gray, None)`` on the device (``main.py:43,179``)
* ``group_position``, ``group_orientation``, ``find_max_orientation``, ``get_final_pose``,
  ``dfs``                                                  (``PostProcessing.py``)

The native library is loaded lazily on first use and its absence is an error
(there is no CPU fallback anywhere in this package).
"""
from .database import Keypoints, SiftDatabase, centroid_of  # noqa: F401
from .sift_helpers import (KeyPoint, get_centroid, make_kp, make_temp_kp,  # noqa: F401
                           unpack_sift_octave)
from .posebin import PoseBin  # noqa: F401
from .matcher import BFMatcher, DMatch, knn2, ratio_match  # noqa: F401
from .hough import (calculate_bin_index, calculate_bin_index_batch,  # noqa: F401
                    estimate_object_pose, estimate_object_pose_batch, perform_hough_transform)
from .affine import (AffineParameters, Calc_x, Ext_Params, Gen_A, Gen_b,  # noqa: F401
                     remove_outliers, verify_bins)
from .pipeline import Main  # noqa: F401
from .postprocessing import (dfs, find_max_orientation, get_final_pose,  # noqa: F401
                             group_orientation, group_position)
from .sharded import FileHostComm, FileStore, HostComm, RcclComm, run_sharded, shard_range  # noqa: F401
from .batch import run_query_batch, sift_query_batch  # noqa: F401
from .sift import SIFT, SIFT_create, bgr_to_gray  # noqa: F401
from .constants import REFERENCE, ReferenceConstants  # noqa: F401

__all__ = ["Keypoints", "SiftDatabase", "centroid_of", "KeyPoint", "get_centroid", "make_kp",
           "make_temp_kp", "unpack_sift_octave", "PoseBin", "BFMatcher", "DMatch", "knn2",
           "ratio_match", "calculate_bin_index", "calculate_bin_index_batch",
           "estimate_object_pose", "estimate_object_pose_batch", "perform_hough_transform",
           "AffineParameters", "Calc_x", "Ext_Params", "Gen_A", "Gen_b", "remove_outliers",
           "verify_bins", "Main", "dfs", "group_position", "group_orientation",
           "find_max_orientation", "get_final_pose", "run_query_batch", "sift_query_batch", "HostComm", "RcclComm", "FileHostComm", "FileStore", "run_sharded",
           "shard_range", "SIFT", "SIFT_create", "bgr_to_gray", "REFERENCE", "ReferenceConstants"]

