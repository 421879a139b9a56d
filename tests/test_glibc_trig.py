"""glibc's sin / cos restated for the device (sift-based-od_amd/csrc/glibc_trig.h).

estimate_object_pose rotates each match's model offset with math.cos / math.sin
(/root/reference/HoughTransformHelperFunctions.py:31-35), i.e. the host's glibc, whose results
are not correctly rounded; the restatement reproduces glibc 2.35's x86_64 FMA-variant s_sin.c
(the ifunc target on CPUs with FMA / AVX2) with the library's own constants and table.

* CPU: tools/glibc_trig_check.cpp (the header compiled for the host) against this host's
  libm on several ranges, the s_sin.c branch edges and the table points -- bit for bit.
* GPU: the device's values of the same function (sod_glibc_sincos) against the host's libm
  called through ctypes (not numpy: np.sin is numpy's own SIMD code, not glibc).
"""
import ctypes
import math
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_restatement_equals_host_libm(tmp_path):
    exe = tmp_path / "gtc"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-mfma",
                    os.path.join(REPO, "tools", "glibc_trig_check.cpp"), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe), "300000"], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0 and out.stdout.strip().endswith("OK"), out.stdout


def test_table_generator_refuses_other_libm(tmp_path):
    """tools/gen_glibc_trig.py reads fixed file offsets of ONE libm build: it regenerates the
    committed glibc_trig_tab.h exactly from the library whose sha256 the header records, and
    refuses (no output) any other file."""
    import hashlib
    gen = os.path.join(REPO, "tools", "gen_glibc_trig.py")
    tab = open(os.path.join(REPO, "sift-based-od_amd", "csrc", "glibc_trig_tab.h")).read()
    libm = "/lib/x86_64-linux-gnu/libm.so.6"
    recorded = tab.split('#define GT_LIBM_SHA256 "')[1].split('"')[0]
    if not os.path.exists(libm) or hashlib.sha256(open(libm, "rb").read()).hexdigest() != recorded:
        pytest.skip("this host's libm is not the recorded build (the device path's probe, "
                    "sod_trig_exact, then arms the host-libm fallback)")
    r = subprocess.run([sys.executable, gen, "--check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # any other file: refused before a byte is emitted
    other = tmp_path / "libm.so.6"
    other.write_bytes(open(libm, "rb").read()[:-1] + b"\x01")
    code = ("import runpy, sys; sys.argv = ['gen']; g = runpy.run_path(%r, run_name='x'); "
            "g['load'](%r)" % (gen, str(other)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    assert r.returncode != 0 and "refusing" in (r.stderr + r.stdout)


def _libm_sincos(x):
    libm = ctypes.CDLL("libm.so.6")
    libm.sin.restype = libm.cos.restype = ctypes.c_double
    libm.sin.argtypes = libm.cos.argtypes = [ctypes.c_double]
    s = np.array([libm.sin(float(v)) for v in x])
    c = np.array([libm.cos(float(v)) for v in x])
    return s, c


def _angles(n):
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(0.0, 2 * math.pi, n),
                        rng.uniform(-0.126, 0.126, n // 8),
                        rng.uniform(0.855, 2.43, n // 8),
                        rng.uniform(-100.0, 100.0, n // 8)])
    # the pose angles main.py makes: radians of a float difference of OpenCV angles, +2pi, % 2pi
    d = rng.uniform(-360.0, 360.0, n // 4).astype(np.float32).astype(np.float64)
    x = np.concatenate([x, np.fmod(d * (math.pi / 180.0) + 2 * math.pi, 2 * math.pi)])
    return x


def test_python_math_is_libm():
    """What the reference calls (math.cos / math.sin) is the libm the tests compare with."""
    x = _angles(2000)
    s, c = _libm_sincos(x)
    assert all(math.sin(v) == a and math.cos(v) == b for v, a, b in zip(x, s, c))


@pytest.mark.gpu
def test_device_glibc_sincos_equals_host_libm(ctx):
    x = _angles(40000)
    s, c = ctx.glibc_sincos(x)
    hs, hc = _libm_sincos(x)
    if not ctx.trig_exact():
        pytest.skip("this host's libm is not glibc's FMA variant (the guard stays armed)")
    assert np.array_equal(s.view(np.uint64), hs.view(np.uint64)), int((s != hs).sum())
    assert np.array_equal(c.view(np.uint64), hc.view(np.uint64)), int((c != hc).sum())
