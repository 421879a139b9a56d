"""Natural-image inputs for the SIFT parity tests -- run here only.

The reference holds no SIFT fixture (its outputs come from OpenCV, absent here), but it
does hold images: `Capture.PNG` and the result plots under `results/`.  Two of them are
converted to 8-bit gray with OpenCV's BGR2GRAY formula ((B*1868 + G*9617 + R*4899 +
2^13) >> 14, the conversion main.py:41 applies) and stored as data; the expected
keypoints/descriptors are recomputed by oracle/sift_oracle.c in the tests.

    python tests/golden/make_sift_images.py      # needs /root/reference and PIL
"""
import os

import numpy as np
from PIL import Image

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sift_images.npz")
SOURCES = {"capture": "Capture.PNG",
           "rotated": "results/before affine/standing/rotated/rotated_1.png"}


def gray(path):
    rgb = np.array(Image.open(path).convert("RGB")).astype(np.int32)
    r, g, b = rgb[..., 0], rgb[..., 1], rgb[..., 2]
    return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)


if __name__ == "__main__":
    arrs = {k: gray(os.path.join(REF, v)) for k, v in SOURCES.items()}
    np.savez_compressed(OUT, **arrs)
    for k, v in arrs.items():
        print(k, v.shape)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")
