"""Operand bytes for tools/probes/mfma_power: SIFT-like descriptors (synthetic.py, the bench's
generator) shifted by -SHIFT as the int8 matcher packs them (SHIFT 128 = the kernel's; a
smaller shift keeps small values small: values beyond 127 + SHIFT are clamped -- power
measurement only), 64 KiB.
    python tools/probes/sift_operand_bytes.py OUT [SHIFT]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import sod_pkg  # noqa: E402

sod_pkg.load()
from sift_based_od_amd import synthetic  # noqa: E402

shift = int(sys.argv[2]) if len(sys.argv) > 2 else 128
d = synthetic.sift_like_descriptors(np.random.default_rng(0), 512).astype(np.int16) - shift
np.clip(d, -128, 127).astype(np.int8).tofile(sys.argv[1])
