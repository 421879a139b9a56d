"""The reference's hard-coded constants in one frozen record, and the Python
layer's defaults taken from it."""
import dataclasses
import inspect

import pytest

from sift_based_od_amd import REFERENCE, Main, ReferenceConstants, _lib
from sift_based_od_amd import batch, pipeline, sharded


def test_reference_values():
    # main.py:82,141,150,183-185; HoughTransformHelperFunctions.py:66;
    # GenerateDatabaseInfo.py:23; PostProcessing.py:27-28,52
    assert (REFERENCE.ratio, REFERENCE.bins, REFERENCE.vote_threshold,
            REFERENCE.affine_threshold) == (0.75, 15, 5, 4)
    assert REFERENCE.pos_factor == 32 and REFERENCE.outlier_factor == 128.0
    assert 2 * (REFERENCE.n_oct - 1) + 0.5 == 6.5
    assert (REFERENCE.max_dim, REFERENCE.cluster_div, REFERENCE.orientation_tol_deg) == \
        (1500, 4, 1.0)
    with pytest.raises(dataclasses.FrozenInstanceError):
        REFERENCE.ratio = 0.8
    assert ReferenceConstants() == REFERENCE


def test_defaults_follow_the_record():
    want = {"ratio": REFERENCE.ratio, "bins": REFERENCE.bins,
            "vote_threshold": REFERENCE.vote_threshold,
            "affine_threshold": REFERENCE.affine_threshold}
    for fn in (Main.run, _lib.Context.pipeline, batch.run_query_batch, batch.sift_query_batch,
               sharded.run_sharded):
        params = inspect.signature(fn).parameters
        for k, v in want.items():
            if k in params and params[k].default is not inspect.Parameter.empty:
                assert params[k].default == v, (fn.__qualname__, k)
    assert pipeline.POS_FACTOR == batch.POS_FACTOR == REFERENCE.pos_factor
