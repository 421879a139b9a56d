"""Operand bytes for tools/probes/mfma_power: SIFT-like descriptors (synthetic.py, the bench's
generator) shifted by -128 as the int8 matcher packs them, 64 KiB."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import synthetic  # noqa: E402

d = synthetic.sift_like_descriptors(np.random.default_rng(0), 512)
((d.astype(np.int16) - 128).astype(np.int8)).tofile(sys.argv[1])
