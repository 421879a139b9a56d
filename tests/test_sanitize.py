"""SURVEY.md §5's sanitizer build of the host code (CPU, no GPU): the C restatement of
OpenCV's SIFT (oracle/sift_oracle.c), post.hip's host walk (post_walk.h: the reference's DFS
visit order, PostProcessing.py:4-112) and glibc_trig.h's host compile are built with
AddressSanitizer + UndefinedBehaviorSanitizer (-fno-sanitize-recover: any report fails the
run) and run on the committed fixtures; their outputs must also equal the regular builds'
(SIFT) or the reference's goldens (post-processing) bit for bit."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import golden

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SAN = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
       "-fno-sanitize-recover=all", "-ffp-contract=off"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=86",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None,
                                reason="needs gcc / g++")


def _run(cmd, **kw):
    r = subprocess.run(cmd, capture_output=True, text=True, env=ENV, timeout=600, **kw)
    report = r.stderr + r.stdout
    assert "Sanitizer" not in report and "runtime error" not in report, report[-4000:]
    assert r.returncode == 0, (r.returncode, report[-4000:])
    return r


def _records(path, kinds):
    raw = open(path, "rb").read()
    out, off = [], 0
    for dt in kinds:
        n = int(np.frombuffer(raw, np.int64, 1, off)[0])
        off += 8
        a = np.frombuffer(raw, dt, n, off)
        off += a.nbytes
        out.append(a)
    assert off == len(raw)
    return out


def test_post_walk_sanitized(tmp_path):
    exe = tmp_path / "post_san"
    subprocess.run(["g++", "-std=c++17", *SAN, os.path.join(HERE, "sanitize", "post_main.cpp"),
                    "-o", str(exe)], check=True)
    for name in ("post_edge", "post_small", "post_medium", "post_chain"):
        g = golden(name)
        m = np.ascontiguousarray(g["means"], np.float64)
        src, dst = tmp_path / (name + ".in"), tmp_path / (name + ".out")
        with open(src, "wb") as f:
            f.write(np.int64(len(m)).tobytes() + m.tobytes())
        _run([str(exe), str(src), str(dst)])
        pos_off, pos_mem, ori_pos_off, ori_off, ori_mem, orient, pose = _records(
            dst, [np.int32] * 5 + [np.float64] * 2)
        for k, v in (("pos_off", pos_off), ("pos_members", pos_mem),
                     ("ori_pos_off", ori_pos_off), ("ori_off", ori_off),
                     ("ori_members", ori_mem)):
            assert np.array_equal(v, g[k]), (name, k)
        assert np.array_equal(orient.view(np.uint64), g["final_orientation"].view(np.uint64))
        assert np.array_equal(pose.reshape(-1, 6).view(np.uint64),
                              np.asarray(g["final_pose"]).reshape(-1, 6).view(np.uint64))


def test_sift_oracle_sanitized(tmp_path):
    from oracle import sift as osift
    exe = tmp_path / "sift_san"
    subprocess.run(["gcc", "-std=c11", *SAN, os.path.join(REPO, "oracle", "sift_oracle.c"),
                    os.path.join(HERE, "sanitize", "sift_main.c"), "-o", str(exe), "-lm"],
                   check=True)
    imgs = golden("sift_images")
    for name in ("rotated", "capture"):
        img = np.ascontiguousarray(imgs[name], np.uint8)
        h, w = img.shape
        src, dst = tmp_path / (name + ".in"), tmp_path / (name + ".out")
        with open(src, "wb") as f:
            f.write(np.array([w, h], np.int32).tobytes() + img.tobytes())
        _run([str(exe), str(src), str(dst)])
        raw = open(dst, "rb").read()
        n = int(np.frombuffer(raw, np.int32, 1)[0])
        f32 = np.frombuffer(raw, np.float32, n * 5, 4).reshape(5, n)
        oc = np.frombuffer(raw, np.int32, n, 4 + 20 * n)
        desc = np.frombuffer(raw, np.float32, n * 128, 4 + 24 * n).reshape(n, 128)
        ref = osift.detect_and_compute(img)           # the regular -O2 build (libsift_oracle.so)
        assert n == len(ref["x"]) and n > 100
        for i, k in enumerate(("x", "y", "size", "angle", "response")):
            assert np.array_equal(f32[i].view(np.uint32), ref[k].view(np.uint32)), (name, k)
        assert np.array_equal(oc, ref["octave"])
        assert np.array_equal(desc.view(np.uint32), ref["descriptors"].view(np.uint32))


def test_glibc_trig_host_sanitized(tmp_path):
    exe = tmp_path / "gtc_san"
    subprocess.run(["g++", "-std=c++17", *SAN, "-mfma",
                    os.path.join(REPO, "tools", "glibc_trig_check.cpp"), "-o", str(exe)],
                   check=True)
    r = _run([str(exe), "20000"])
    assert r.stdout.strip().endswith("OK"), r.stdout[-2000:]
