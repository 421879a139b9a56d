"""The reference's hard-coded constants in one frozen record (SURVEY.md §5 "Config/flags"),
with the defaults main.py runs with.  The Python layer's defaults come from here; the device
kernels bake in the ones that shape their arithmetic (noted per field)."""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class ReferenceConstants:
    ratio: float = 0.75            # Lowe's ratio test, main.py:82 (strict <)
    bins: int = 15                 # Hough bins per axis, main.py:183
    vote_threshold: int = 5        # get_valid_bins, main.py:184 (>=)
    affine_threshold: int = 4      # apply_affine_parameters, main.py:185 (>=)
    pos_factor: int = 32           # main.py:141; remove_outliers divides by pos_factor * 4
    n_oct: int = 4                 # HoughTransformHelperFunctions.py:66; the scale bin divides
    #                                log2(s) by 2 * (n_oct - 1) + 0.5 = 6.5 (hough.hip's LUT)
    max_dim: int = 1500            # DB image width after resize, GenerateDatabaseInfo.py:23
    cluster_div: int = 4           # pose clusters: |dx| <= w * scale / 4, PostProcessing.py:27-28
    orientation_tol_deg: float = 1.0   # orientation clusters, PostProcessing.py:52 (<=)

    @property
    def outlier_factor(self) -> float:
        """remove_outliers' x_factor = y_factor (main.py:150: pos_factor * 4)."""
        return float(self.pos_factor * 4)


REFERENCE = ReferenceConstants()
