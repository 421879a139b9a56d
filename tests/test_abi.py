"""The C ABI: libsod.so loads without a GPU and exports exactly what include/sod.h
declares; the ctypes signature table mirrors the header.  No compute calls (CPU only)."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

from conftest import REPO
from sift_based_od_amd import _lib

HEADER = os.path.join(REPO, "include", "sod.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sod_[a-z0-9_]+)\s*\(", src)))


def test_header_parses():
    names = declared()
    assert "sod_create" in names and "sod_pipeline_enqueue" in names
    assert len(names) >= 25


def test_library_exports_every_declared_symbol():
    L = _lib.lib()                      # loads libamdhip64 / librccl, no device needed
    for n in declared():
        assert hasattr(L, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = sorted(set(re.findall(r" T (sod_[a-z0-9_]+)", out)))
    assert exported == declared()


def test_ctypes_table_mirrors_header():
    assert sorted(_lib.SIGNATURES) == declared()


def test_abi_version_without_gpu():
    assert _lib.lib().sod_abi_version() == 1


def test_pipeline_args_layout():
    # sod_pipeline_args in sod.h: double, 2 x i32, i32[4], 2 x i32, 2 x double, 2 x i32
    a = _lib.PipelineArgs
    assert a.ratio.offset == 0
    assert a.query_h.offset == 8 and a.bins.offset == 16
    assert a.vote_threshold.offset == 32 and a.x_factor.offset == 40
    assert a.run_affine.offset == 56 and a.stage_parts.offset == 60 and ctypes.sizeof(a) == 64


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "libsod.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.lib()


def test_bins4():
    assert _lib.bins4(15) == (15, 15, 15, 15)
    assert _lib.bins4((32, 32, 8, 12)) == (32, 32, 8, 12)
    with pytest.raises(ValueError):
        _lib.bins4((1, 2, 3))


def test_host_trig_is_glibc_sin_and_cos_not_sincos():
    """The boundary guard and the exact PoseBin means redo pose x / y with the host's glibc
    sin / cos, the calls math.sin / math.cos make.  glibc's sincos differs from them in ~0.1 %
    of arguments (checked here: 23 667 of 2e7 angles), so a compiler folding the pair into
    sincos would break their bit-exactness: the library must import sin and cos only."""
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    imported = set(re.findall(r" U (\w+)(?:@\S+)?", out))
    assert {"sin", "cos"} <= imported
    assert not imported & {"sincos", "__sincos", "sincosf"}


@pytest.mark.skipif(not shutil.which("gcc"), reason="needs gcc")
def test_results_struct_layout(tmp_path):
    """sod_results (sod.h) as the C compiler lays it out == the ctypes mirror (_lib.Results)."""
    fields = [f[0] for f in _lib.Results._fields_]
    src = tmp_path / "lay.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "sod.h"\nint main(void) {\n'
                   '  printf("%zu\\n", sizeof(sod_results));\n' +
                   "".join('  printf("%%zu\\n", offsetof(sod_results, %s));\n' % f for f in fields) +
                   "  return 0;\n}\n")
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    assert got[0] == ctypes.sizeof(_lib.Results)
    assert got[1:] == [getattr(_lib.Results, f).offset for f in fields]


def test_numpy_matmul_probe():
    """The Python layer's probe of how this host's numpy rounds remove_outliers' 2x2 product
    (AffineParameters.py:145) on BOTH output rows: 1 = fma(m_r0, x, m_r1*y), 2 =
    fma(m_r1, y, m_r0*x), 0 = two roundings; a second, independent sample (other matrices,
    both rows) is rounded exactly as the mode says."""
    from fractions import Fraction
    import numpy as np

    def fma(a, b, c):
        return float(Fraction(a) * Fraction(b) + Fraction(c))
    got = _lib.numpy_matmul_fma()
    assert got in (0, 1, 2)
    assert _lib.MATMUL_FMA_CONSISTENT
    rng = np.random.default_rng(99)
    for a, b, c, d, x, y in rng.uniform(-3, 3, (200, 6)) * [1, 1, 1, 1, 500, 500]:
        r = np.matmul([[a, b], [c, d]], [x, y]).tolist()
        for m0, m1, v in ((a, b, r[0]), (c, d, r[1])):
            want = (fma(m0, x, m1 * y) if got == 1 else fma(m1, y, m0 * x) if got == 2
                    else m0 * x + m1 * y)
            assert v == want


def test_results_gather_views():
    """_lib._gather (sod_results_fetch's host read): arrays at host addresses, merged into
    runs copied once, come back equal to their sources -- runs of adjacent arrays, a far
    one, empty and null entries, 2-D rows, records that step back inside or before a run."""
    import numpy as np
    a = np.arange(40, dtype=np.int32)
    b = np.arange(12, dtype=np.float64).reshape(2, 6) * 0.5
    far = np.array([True, False, True])
    base = a.ctypes.data
    i4, f8, b1 = np.dtype("<i4"), np.dtype("<f8"), np.dtype("|b1")
    spec = [("x", base, 10, i4, 0), ("y", base + 40, 5, i4, 4), ("b", b.ctypes.data, 2, f8, 6),
            ("f", far.ctypes.data, 3, b1, 0), ("e", base, 0, i4, 0), ("n", 0, 0, f8, 6),
            ("back", base + 8, 3, i4, 0), ("x2", base + 4, 2, i4, 0)]   # (before the run)
    out = _lib._gather(spec)
    assert np.array_equal(out["x"], a[:10])
    assert list(out["back"]) == [2, 3, 4] and list(out["x2"]) == [1, 2]
    assert np.array_equal(out["y"], a[10:30].reshape(5, 4))
    assert np.array_equal(out["b"], b) and np.array_equal(out["f"], far)
    assert out["e"].shape == (0,) and out["n"].shape == (0, 6)
    a[:] = -1                                   # copies, not views of the source memory
    assert out["x"][0] == 0


def _fake_results(rng, nq, V, M, nb, npos, nori, selected, affined, post, nulls=()):
    """A sod_results pointing into one random host buffer (kept alive by the caller)."""
    import numpy as np
    buf = rng.integers(0, 256, 1 << 18, dtype=np.uint8)
    buf[1::7] &= 1     # (bool arrays read 0/1 bytes from the device; any byte here is fine)
    o = [buf.ctypes.data]

    def take(n):
        a = o[0]
        o[0] += (n + 15) & ~15
        return a
    rs = _lib.Results()
    arr = np.frombuffer(rs, _lib._RES_DTYPE).copy()
    for k, v in {"nq": nq, "selected": selected, "n_valid": V, "n_members": M,
                 "affined": affined, "post": post, "n_bins": nb, "n_pos": npos,
                 "n_ori": nori}.items():
        arr[0][k] = v
    sizes = {"idx1": nq * 4, "d1": nq * 4, "d2": nq * 4, "good": nq, "keys": V * 16,
             "votes": V * 4, "offsets": (V + 1) * 8, "members": M * 4, "means": V * 48,
             "survived": V, "affine_votes": V * 4, "params": V * 48, "alive": M,
             "bin_index": nb * 4, "pos_off": (npos + 1) * 4, "pos_members": nb * 4,
             "ori_pos_off": (npos + 1) * 4, "ori_off": (nori + 1) * 4, "ori_members": nb * 4,
             "final_orientation": npos * 8, "final_pose": npos * 48}
    for k, s in sizes.items():
        arr[0][k] = 0 if k in nulls else take(s)
    ctypes.memmove(ctypes.addressof(rs), arr.ctypes.data, ctypes.sizeof(rs))
    return rs, buf


def test_resparse_equals_python_reader():
    """The C results reader (csrc/resparse.c) returns what _results_from_struct returns: the
    same dict / tuple structure, dtypes, shapes and values, as copies -- over every part mask,
    empty parts, null pointers and zero counts."""
    import numpy as np
    assert _lib._RESPARSE is not None, "_resparse not built (make -C sift-based-od_amd/csrc)"
    rng = np.random.default_rng(5)

    def same(a, b):
        assert type(a) is type(b)
        if isinstance(a, dict):
            assert list(a) == list(b)
            for k in a:
                same(a[k], b[k])
        elif isinstance(a, tuple):
            assert len(a) == len(b)
            for x, y in zip(a, b):
                same(x, y)
        else:
            assert a.dtype == b.dtype and a.shape == b.shape, (a.dtype, b.dtype, a.shape, b.shape)
            assert a.tobytes() == b.tobytes()
    cases = [(500, 40, 400, 12, 5, 7, 1, 1, 1, ()), (500, 40, 400, 12, 5, 7, 1, 0, 0, ()),
             (500, 0, 0, 0, 0, 0, 1, 1, 1, ()), (0, 3, 5, 3, 1, 1, 1, 1, 1, ()),
             (17, 9, 20, 4, 2, 3, 1, 1, 1, ("members", "final_pose", "d2")),
             (1, 1, 1, 1, 1, 1, 0, 0, 0, ())]
    for case in cases:
        rs, buf = _fake_results(rng, *case)
        for mask in (1, 2, 3, 7, 15):
            want = _lib._results_from_struct(rs, mask)
            got = _lib._RESPARSE.results(ctypes.addressof(rs), mask)
            same(got, want)
        got = _lib._RESPARSE.results(ctypes.addressof(rs), 15)
        before = {k: v.copy() for k, v in got.get("valid", {}).items()}
        buf[:] = 0                                   # copies, not views of the source
        for k, v in before.items():
            assert np.array_equal(got["valid"][k], v)
    with pytest.raises(ValueError):
        _lib._RESPARSE.results(0, 15)


def test_pipeline_args_reused_only_when_equal():
    """Context.pipeline reuses its argument struct when every argument equals the last
    call's, and rebuilds it when any differs (a stub library records what the C side gets)."""
    seen = []

    class Stub:
        def sod_pipeline_enqueue(self, h, a):
            seen.append(bytes(a._obj))
            return 0
    c = object.__new__(_lib.Context)
    c._L, c._h = Stub(), None
    bins = [32, 32, 8, 12]
    calls = [((480, 640), bins, 0.75, ("match",)), ((480, 640), bins, 0.75, ("match",)),
             ((480, 640), bins, 0.8, ("match",)), ((480, 640), 15, 0.8, ("match", "post")),
             ((481, 640), 15, 0.8, ("match", "post")), ((481, 640), bins, 0.8, ("match", "post"))]
    for shape, b, r, st in calls:
        c.pipeline(shape, b, r, stage=st)
    snap = [(shape, _lib.bins4(b), r, st) for shape, b, r, st in calls]
    bins[3] = 6                                   # the caller's list mutated in place
    c.pipeline((481, 640), bins, 0.8, stage=("match", "post"))
    want = []
    for shape, b, r, st in snap + [((481, 640), (32, 32, 8, 6), 0.8, ("match", "post"))]:
        a = _lib.PipelineArgs()
        for p in st:
            a.stage_parts |= c.RES[p]
        a.ratio, a.query_h, a.query_w = r, shape[0], shape[1]
        for i, v in enumerate(_lib.bins4(b)):
            a.bins[i] = v
        a.vote_threshold, a.affine_threshold, a.x_factor, a.y_factor = 5, 4, 128.0, 128.0
        a.run_affine = 1
        want.append(bytes(a))
    assert seen == want
    assert c.bins == (32, 32, 8, 6)
