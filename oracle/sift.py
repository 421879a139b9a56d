"""ctypes binding of oracle/sift_oracle.c -- TEST INFRASTRUCTURE ONLY.

The C file restates OpenCV's SIFT (`cv2.SIFT_create().detectAndCompute`, the call at
main.py:43 / GenerateDatabaseInfo.py:32); see its header for the algorithm, the fixed
arithmetic and why parity against OpenCV itself is unpinned.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline use this module."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libsift_oracle.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        L.sift_oracle_detect.restype = ctypes.c_int
        L.sift_oracle_detect.argtypes = [
            _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
            ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.sift_oracle_layer.restype = ctypes.c_int
        L.sift_oracle_layer.argtypes = [
            _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
            ctypes.POINTER(ctypes.c_int)]
        L.sift_num_octaves.restype = ctypes.c_int
        L.sift_num_octaves.argtypes = [ctypes.c_int, ctypes.c_int]
        L.sift_gauss_kernel.restype = ctypes.c_int
        L.sift_gauss_kernel.argtypes = [ctypes.c_double, _f32p, ctypes.c_int]
        L.sift_fast_atan2.restype = ctypes.c_float
        L.sift_fast_atan2.argtypes = [ctypes.c_float, ctypes.c_float]
        L.sift_oracle_bgr2gray.restype = None
        L.sift_oracle_bgr2gray.argtypes = [_u8p, ctypes.c_int64, _u8p]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def detect_and_compute(gray, n_octave_layers=3, contrast_threshold=0.04, edge_threshold=10.0,
                       sigma=1.6, descriptors=True):
    """SoA keypoints (x, y, size, angle, response, octave) in OpenCV's output order and,
    if asked, the float32 [n, 128] descriptors."""
    g = np.ascontiguousarray(gray, np.uint8)
    h, w = g.shape
    L = lib()
    n = L.sift_oracle_detect(g, w, h, n_octave_layers, contrast_threshold, edge_threshold,
                             sigma, 0, None, None, None, None, None, None, None)
    if n < 0:
        raise ValueError("sift_oracle_detect: bad arguments")
    out = {k: np.zeros(n, np.float32) for k in ("x", "y", "size", "angle", "response")}
    out["octave"] = np.zeros(n, np.int32)
    desc = np.zeros((n, 128), np.float32) if descriptors else None
    m = L.sift_oracle_detect(g, w, h, n_octave_layers, contrast_threshold, edge_threshold,
                             sigma, n, _ptr(out["x"]), _ptr(out["y"]), _ptr(out["size"]),
                             _ptr(out["angle"]), _ptr(out["response"]), _ptr(out["octave"]),
                             _ptr(desc) if descriptors else None)
    assert m == n
    if descriptors:
        out["descriptors"] = desc
    return out


def layer(gray, kind, octave, index, n_octave_layers=3, sigma=1.6):
    """Gaussian (kind 0) or DoG (kind 1) pyramid layer as a float32 [h, w] array."""
    g = np.ascontiguousarray(gray, np.uint8)
    h, w = g.shape
    ow, oh = ctypes.c_int(), ctypes.c_int()
    L = lib()
    n = L.sift_oracle_layer(g, w, h, n_octave_layers, sigma, kind, octave, index, None,
                            ctypes.byref(ow), ctypes.byref(oh))
    if n < 0:
        raise IndexError("no such layer")
    out = np.zeros((oh.value, ow.value), np.float32)
    L.sift_oracle_layer(g, w, h, n_octave_layers, sigma, kind, octave, index, _ptr(out), None,
                        None)
    return out


def num_octaves(w, h):
    return lib().sift_num_octaves(w, h)


def gauss_kernel(sigma):
    k = np.zeros(64, np.float32)
    r = lib().sift_gauss_kernel(sigma, k, 64)
    return k[: r + 1]


def bgr2gray(bgr):
    b = np.ascontiguousarray(bgr, np.uint8)
    out = np.zeros(b.shape[:-1], np.uint8)
    lib().sift_oracle_bgr2gray(b.reshape(-1), b.size // 3, out.reshape(-1))
    return out
