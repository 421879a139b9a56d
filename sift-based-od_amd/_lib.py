"""ctypes binding of libsod.so (C ABI declared in include/sod.h).

Loading fails loudly: there is no CPU fallback anywhere in this package.  Build the
library with ``__graft_entry__.build()`` (or ``make -C sift-based-od_amd/csrc``).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

# SOD_LIB_PATH: load an alternative build (A/B experiments of kernel variants only)
LIB_PATH = os.environ.get("SOD_LIB_PATH") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "libsod.so")

SOD_OK, SOD_EINVAL, SOD_EHIP, SOD_ENOMEM, SOD_ESTATE, SOD_ECOMM = range(6)
DTYPE_U8, DTYPE_F32 = 0, 1
UNIQUE_ID_BYTES = 128

_ERRNAMES = {SOD_EINVAL: "EINVAL", SOD_EHIP: "EHIP", SOD_ENOMEM: "ENOMEM",
             SOD_ESTATE: "ESTATE", SOD_ECOMM: "ECOMM"}

c_f32p = C.POINTER(C.c_float)
c_f64p = C.POINTER(C.c_double)
c_i32p = C.POINTER(C.c_int32)
c_i64p = C.POINTER(C.c_int64)
c_u8p = C.POINTER(C.c_uint8)
c_vp = C.c_void_p
c_ctx = C.c_void_p


class PipelineArgs(C.Structure):
    _fields_ = [("ratio", C.c_double), ("query_h", C.c_int32), ("query_w", C.c_int32),
                ("bins", C.c_int32 * 4), ("vote_threshold", C.c_int32),
                ("affine_threshold", C.c_int32), ("x_factor", C.c_double),
                ("y_factor", C.c_double), ("run_affine", C.c_int32), ("stage_parts", C.c_int32)]


_MATMUL_FMA = None


def numpy_matmul_fma():
    """How this host's numpy rounds remove_outliers' 2x2 product np.matmul(M, X)
    (AffineParameters.py:145), both output rows, probed once per process against exact
    rational arithmetic: 1 when every row is fma(m_r0, x, m_r1*y) (OpenBLAS's dgemv on an FMA
    CPU), 2 when fma(m_r1, y, m_r0*x) (the other contraction order), 0 when m_r0*x + m_r1*y
    (two roundings).  The affine kernel follows the mode given (option affine_fma).  A host
    matching none of the three on every probe gets 0 (and ``MATMUL_FMA_CONSISTENT`` False):
    its rare boundary cases are then parity-unpinned."""
    global _MATMUL_FMA, MATMUL_FMA_CONSISTENT
    if _MATMUL_FMA is None:
        from fractions import Fraction

        def fma(a, b, c):
            return float(Fraction(a) * Fraction(b) + Fraction(c))
        rng = np.random.default_rng(12345)
        ok = {0: True, 1: True, 2: True}
        seen = {0: False, 1: False, 2: False}   # the mode is told apart from the others
        for row in rng.uniform(-2, 2, (256, 6)):
            a, b, c, d = (float(v) for v in row[:4])
            x, y = float(row[4] * 750 + 750), float(row[5] * 500 + 500)
            r = np.matmul([[a, b], [c, d]], [x, y]).tolist()
            for m0, m1, got in ((a, b, r[0]), (c, d, r[1])):
                cand = {0: m0 * x + m1 * y, 1: fma(m0, x, m1 * y), 2: fma(m1, y, m0 * x)}
                for k, v in cand.items():
                    ok[k] &= got == v
                    seen[k] |= any(v != w for w in cand.values())
        modes = [k for k in (1, 2, 0) if ok[k]]
        MATMUL_FMA_CONSISTENT = bool(modes)
        # ties (a probe set where two modes never differ) resolve to the listed order
        _MATMUL_FMA = next((k for k in modes if seen[k]), modes[0] if modes else 0)
    return _MATMUL_FMA


MATMUL_FMA_CONSISTENT = True


class Results(C.Structure):
    """sod_results (sod.h): pointers into the context's page-locked staging buffer."""
    _fields_ = [("nq", C.c_int64), ("idx1", C.POINTER(C.c_int32)), ("d1", C.POINTER(C.c_float)),
                ("d2", C.POINTER(C.c_float)), ("good", C.POINTER(C.c_uint8)),
                ("selected", C.c_int32), ("n_valid", C.c_int64), ("n_members", C.c_int64),
                ("keys", C.POINTER(C.c_int32)), ("votes", C.POINTER(C.c_int32)),
                ("offsets", C.POINTER(C.c_int64)), ("members", C.POINTER(C.c_int32)),
                ("means", C.POINTER(C.c_double)), ("affined", C.c_int32),
                ("survived", C.POINTER(C.c_uint8)), ("affine_votes", C.POINTER(C.c_int32)),
                ("params", C.POINTER(C.c_double)), ("alive", C.POINTER(C.c_uint8)),
                ("post", C.c_int32), ("n_bins", C.c_int32),
                ("bin_index", C.POINTER(C.c_int32)), ("n_pos", C.c_int32), ("n_ori", C.c_int32),
                ("pos_off", C.POINTER(C.c_int32)), ("pos_members", C.POINTER(C.c_int32)),
                ("ori_pos_off", C.POINTER(C.c_int32)), ("ori_off", C.POINTER(C.c_int32)),
                ("ori_members", C.POINTER(C.c_int32)),
                ("final_orientation", C.POINTER(C.c_double)),
                ("final_pose", C.POINTER(C.c_double))]


_I4, _I8, _F4, _F8, _B1 = (np.dtype(t) for t in ("<i4", "<i8", "<f4", "<f8", "|b1"))


def _gather(spec):
    """{name: numpy array} for (name, address, rows, dtype, width) records of host memory:
    consecutive records whose byte ranges ascend with gaps under a page (the staging buffer
    holds most arrays back to back, 16-byte aligned) form one run, each run is copied ONCE and
    its arrays are views of that copy.  (A gap under 4 096 bytes between two mapped ranges
    touches no page outside them, so reading it is safe.)"""
    out, runs, run = {}, [], None
    for name, addr, n, dt, width in spec:
        if n <= 0 or not addr:
            out[name] = np.zeros((n, width) if width else (max(n, 0),), dt)
            continue
        cnt = n * width if width else n
        end = addr + cnt * dt.itemsize
        if run is None or addr < run[0] or addr - run[1] >= 4096:
            run = [addr, end]
            runs.append(run)
        elif end > run[1]:
            run[1] = end
        run.append((name, addr - run[0], dt, cnt, (n, width) if width else None))
    fb = np.frombuffer
    for run in runs:
        raw = fb((C.c_uint8 * (run[1] - run[0])).from_address(run[0]), np.uint8).copy()
        for name, off, dt, cnt, shape in run[2:]:
            v = fb(raw, dt, cnt, off)
            out[name] = v.reshape(shape) if shape else v
    return out


# sod_results read in one go: every field as a plain number (pointers as addresses)
_RES_DTYPE = np.dtype({"names": [f for f, _ in Results._fields_],
                       "formats": ["<u8" if issubclass(t, C._Pointer) else
                                   ("<i8" if t is C.c_int64 else "<i4") for _, t in Results._fields_],
                       "offsets": [getattr(Results, f).offset for f, _ in Results._fields_],
                       "itemsize": C.sizeof(Results)})
_RF = {f: i for i, f in enumerate(_RES_DTYPE.names)}


def _res_table(rows):
    # (output name, pointer field, count field, count + k, dtype, width) -> field positions
    return tuple((name, _RF[ptr], _RF[cnt], k, dt, w) for name, ptr, cnt, k, dt, w in rows)


# the staging buffer's arrays first, in its order, then the host-decoded ones (keys, votes
# and the post-processing vectors live in separate host allocations)
_RES_MATCH = _res_table([("idx1", "idx1", "nq", 0, _I4, 0), ("d1", "d1", "nq", 0, _F4, 0),
                         ("d2", "d2", "nq", 0, _F4, 0), ("good", "good", "nq", 0, _B1, 0)])
_RES_VALID = _res_table([("offsets", "offsets", "n_valid", 1, _I8, 0),
                         ("members", "members", "n_members", 0, _I4, 0),
                         ("means", "means", "n_valid", 0, _F8, 6)])
_RES_AFFINE = _res_table([("survived", "survived", "n_valid", 0, _B1, 0),
                          ("affine_votes", "affine_votes", "n_valid", 0, _I4, 0),
                          ("params", "params", "n_valid", 0, _F8, 6),
                          ("alive", "alive", "n_members", 0, _B1, 0)])
_RES_KEYS = _res_table([("keys", "keys", "n_valid", 0, _I4, 4),
                        ("votes", "votes", "n_valid", 0, _I4, 0)])
_RES_POST = _res_table([("bin_index", "bin_index", "n_bins", 0, _I4, 0),
                        ("pos_off", "pos_off", "n_pos", 1, _I4, 0),
                        ("pos_members", "pos_members", "n_bins", 0, _I4, 0),
                        ("ori_pos_off", "ori_pos_off", "n_pos", 1, _I4, 0),
                        ("ori_off", "ori_off", "n_ori", 1, _I4, 0),
                        ("ori_members", "ori_members", "n_bins", 0, _I4, 0),
                        ("final_orientation", "final_orientation", "n_pos", 0, _F8, 0),
                        ("final_pose", "final_pose", "n_pos", 0, _F8, 6)])
_SEL, _AFF, _POST = _RF["selected"], _RF["affined"], _RF["post"]


def _results_from_struct(rs, mask):
    """sod_results (the parts in ``mask``) as Context.results' dict of numpy arrays."""
    r = np.frombuffer(rs, _RES_DTYPE)[0].tolist()   # (values in field order)
    sel, aff, post = r[_SEL], r[_AFF], r[_POST]
    tables = (_RES_MATCH if mask & 1 else ()) + (_RES_VALID if sel else ()) + \
        (_RES_AFFINE if aff else ()) + (_RES_KEYS if sel else ()) + (_RES_POST if post else ())
    a = _gather([(name, r[p], r[c] + k, dt, w) for name, p, c, k, dt, w in tables])
    out = {}
    if mask & 1:
        out["match"] = (a["idx1"], a["d1"], a["d2"], a["good"])
    if sel:
        out["valid"] = {"keys": a["keys"], "votes": a["votes"], "offsets": a["offsets"],
                        "members": a["members"], "means": a["means"]}
    if aff:
        out["affine"] = {"survived": a["survived"], "votes": a["affine_votes"],
                         "params": a["params"], "alive": a["alive"]}
    if post:
        out["post"] = {k: a[k] for k in ("bin_index", "pos_off", "pos_members", "ori_pos_off",
                                         "ori_off", "ori_members", "final_orientation",
                                         "final_pose")}
    return out


def _load_resparse():
    """The C results reader (csrc/resparse.c, built beside libsod.so), or None: then
    _results_from_struct reads them (same dict; SOD_RESPARSE=0 forces the Python reader)."""
    if os.environ.get("SOD_RESPARSE", "1") == "0":
        return None
    import importlib.util
    import sysconfig
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "_resparse" + sysconfig.get_config_var("EXT_SUFFIX"))
    if not os.path.exists(path):
        return None
    spec = importlib.util.spec_from_file_location("_resparse", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


_RESPARSE = _load_resparse()


# name -> (restype, argtypes); must mirror include/sod.h exactly (tests check the symbols)
SIGNATURES = {
    "sod_abi_version": (C.c_int, []),
    "sod_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "sod_create": (C.c_int, [C.c_int, C.POINTER(c_ctx)]),
    "sod_destroy": (None, [c_ctx]),
    "sod_last_error": (C.c_char_p, [c_ctx]),
    "sod_synchronize": (C.c_int, [c_ctx]),
    "sod_last_match_ms": (C.c_int, [c_ctx, c_f32p]),
    "sod_match_times": (C.c_int, [c_ctx, C.c_int, c_f32p]),
    "sod_last_stage_ms": (C.c_int, [c_ctx, c_f32p, C.c_int]),
    "sod_set_stage_timing": (C.c_int, [c_ctx, C.c_int]),
    "sod_set_match_timing": (C.c_int, [c_ctx, C.c_int]),
    "sod_set_matcher_streams": (C.c_int, [c_ctx, C.c_int]),
    "sod_set_post_exact": (C.c_int, [c_ctx, C.c_int]),
    "sod_exact_means": (C.c_int, [c_ctx, C.c_int32, c_i32p, c_f64p]),
    "sod_db_set_keypoints": (C.c_int, [c_ctx, C.c_int64, c_f32p, c_f32p, c_f32p, c_i32p, c_i32p,
                                       C.c_int32, c_f64p, c_i32p]),
    "sod_db_upload_descriptors": (C.c_int, [c_ctx, c_vp, C.c_int, C.c_int64, C.c_int64]),
    "sod_db_share": (C.c_int, [c_ctx, c_ctx]),
    "sod_db_packed_size": (C.c_int, [c_ctx, c_i64p]),
    "sod_db_export_packed": (C.c_int, [c_ctx, c_vp, C.c_int64]),
    "sod_db_import_packed": (C.c_int, [c_ctx, c_vp, C.c_int64]),
    "sod_query_upload": (C.c_int, [c_ctx, c_vp, C.c_int, C.c_int32, c_f32p, c_f32p, c_f32p,
                                   c_i32p]),
    "sod_query_window": (C.c_int, [c_ctx, C.c_int32, C.c_int32]),
    "sod_query_images": (C.c_int, [c_ctx, C.c_int32, c_i32p, c_i32p]),
    "sod_valid_images_get": (C.c_int, [c_ctx, c_i32p]),
    "sod_match_enqueue": (C.c_int, [c_ctx]),
    "sod_match_set_impl": (C.c_int, [c_ctx, C.c_int]),
    "sod_match_set_kernel": (C.c_int, [c_ctx, C.c_int]),
    "sod_trig_exact": (C.c_int, [c_ctx]),
    "sod_host_wait_ns": (C.c_int, [c_ctx, c_i64p, C.c_int]),
    "sod_glibc_sincos": (C.c_int, [c_ctx, C.c_int64, c_vp, c_vp, c_vp]),
    "sod_results_fetch": (C.c_int, [c_ctx, C.c_int, C.POINTER(Results)]),
    "sod_set_option": (C.c_int, [c_ctx, C.c_char_p, C.c_int64]),
    "sod_get_option": (C.c_int, [c_ctx, C.c_char_p, C.POINTER(C.c_int64)]),
    "sod_match_set_overlap": (C.c_int, [c_ctx, C.c_int]),
    "sod_set_cu_reserve": (C.c_int, [c_ctx, C.c_int]),
    "sod_match_allgather_enqueue": (C.c_int, [c_ctx]),
    "sod_ratio_enqueue": (C.c_int, [c_ctx, C.c_double]),
    "sod_match_get": (C.c_int, [c_ctx, c_i32p, c_f32p, c_f32p, c_u8p]),
    "sod_matches_set": (C.c_int, [c_ctx, C.c_int32, c_i32p, c_u8p]),
    "sod_match_exact_order": (C.c_int, [c_ctx, C.POINTER(C.c_int)]),
    "sod_match_knn_indices": (C.c_int, [c_ctx, c_i32p, c_i32p]),
    "sod_match_float_order": (C.c_int, [c_ctx]),
    "sod_hough_enqueue": (C.c_int, [c_ctx, C.c_int32, C.c_int32, c_i32p, C.c_int64, C.c_int64]),
    "sod_hough_allreduce_enqueue": (C.c_int, [c_ctx]),
    "sod_select_enqueue": (C.c_int, [c_ctx, C.c_int32]),
    "sod_hough_select_enqueue": (C.c_int, [c_ctx, C.c_int32, C.c_int32, c_i32p, C.c_int32]),
    "sod_valid_counts": (C.c_int, [c_ctx, c_i64p, c_i64p]),
    "sod_valid_get": (C.c_int, [c_ctx, c_i32p, c_i32p, c_i64p, c_i32p, c_f64p]),
    "sod_bins_count": (C.c_int, [c_ctx, c_i64p]),
    "sod_bins_get": (C.c_int, [c_ctx, c_i32p, c_i32p]),
    "sod_hough_guard_stats": (C.c_int, [c_ctx, c_i64p, c_i64p, c_i64p, c_i64p]),
    "sod_affine_enqueue": (C.c_int, [c_ctx, C.c_int32, C.c_int32, C.c_double, C.c_double,
                                     C.c_int32]),
    "sod_affine_get": (C.c_int, [c_ctx, c_u8p, c_i32p, c_f64p, c_u8p]),
    "sod_pipeline_enqueue": (C.c_int, [c_ctx, C.POINTER(PipelineArgs)]),
    "sod_postprocess": (C.c_int, [c_ctx, c_i32p, c_i32p, c_i32p, c_i32p, c_i32p, c_i32p, c_i32p,
                                  c_i32p, c_i32p, c_f64p, c_f64p]),
    "sod_post_batch": (C.c_int, [c_ctx, C.c_int32, c_f64p, c_i32p, c_i32p, c_i32p, c_i32p, c_i32p,
                                 c_i32p, c_i32p, c_f64p, c_f64p]),
    "sod_pose_batch": (C.c_int, [c_ctx, C.c_int64, c_f32p, c_f32p, c_f32p, c_i32p, c_f32p, c_f32p,
                                 c_f32p, c_i32p, c_f64p, c_f64p, C.c_int32, C.c_int32, c_i32p,
                                 c_f64p, c_i32p]),
    "sod_bin_index_batch": (C.c_int, [c_ctx, C.c_int64, c_f64p, C.c_int32, C.c_int32, c_i32p,
                                      c_i32p]),
    "sod_affine_batch": (C.c_int, [c_ctx, C.c_int64, c_i64p, c_f32p, c_f32p, c_f32p, c_f32p,
                                   c_i32p, C.c_int32, C.c_int32, C.c_double, C.c_double,
                                   C.c_int32, C.c_int32, c_f64p, c_u8p, c_i32p, c_f64p, c_u8p]),
    "sod_match_candidates_get": (C.c_int, [c_ctx, c_f32p, c_i32p, c_f32p]),
    "sod_match_candidates_merge": (C.c_int, [c_ctx, C.c_int32, c_f32p, c_i32p, c_f32p]),
    "sod_hough_partial_get": (C.c_int, [c_ctx, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "sod_hough_partial_set": (C.c_int, [c_ctx, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "sod_sift_set_params": (C.c_int, [c_ctx, C.c_int32, C.c_double, C.c_double, C.c_double]),
    "sod_sift_set_lane_order": (C.c_int, [c_ctx, C.c_int]),
    "sod_sift_lane_order": (C.c_int, [c_ctx, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "sod_sift_detect": (C.c_int, [c_ctx, c_u8p, C.c_int32, C.c_int32, c_i32p]),
    "sod_sift_detect_bgr": (C.c_int, [c_ctx, c_u8p, C.c_int32, C.c_int32, c_i32p]),
    "sod_sift_detect_batch": (C.c_int, [c_ctx, C.c_int32, C.POINTER(c_u8p), c_i32p, c_i32p,
                                        c_i32p, c_i32p]),
    "sod_sift_get": (C.c_int, [c_ctx, C.c_int64, c_f32p, c_f32p, c_f32p, c_f32p, c_f32p, c_i32p,
                               c_f32p]),
    "sod_sift_to_queries": (C.c_int, [c_ctx]),
    "sod_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8 * UNIQUE_ID_BYTES)]),
    "sod_comm_init": (C.c_int, [c_ctx, C.c_int32, C.c_int32, C.POINTER(C.c_uint8 * UNIQUE_ID_BYTES)]),
    "sod_comm_info": (C.c_int, [c_ctx, c_i32p, c_i32p]),
}

_lib = None
_lock = threading.Lock()


class SodError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("libsod %s (%d): %s" % (_ERRNAMES.get(code, "?"), code, msg))
        self.code = code


def lib():
    """The loaded libsod.so; raises if it is missing (no fallback)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    "libsod.so not found at %s -- build it with __graft_entry__.build() "
                    "(hipcc --offload-arch=gfx950); this package has no CPU fallback" % LIB_PATH)
            L = C.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            _lib = L
        return _lib


def ptr(a, ctype):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ctype))


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def unique_id():
    buf = (C.c_uint8 * UNIQUE_ID_BYTES)()
    rc = lib().sod_comm_unique_id(C.byref(buf))
    if rc != SOD_OK:
        raise SodError(rc, lib().sod_last_error(None).decode())
    return bytes(buf)


class Context:
    """One libsod context = one GPU (HIP device ``device``) driven by this thread."""

    _pargs_key = _pargs = None   # (Context.pipeline's last argument struct)

    def __init__(self, device=0):
        self._L = lib()
        h = c_ctx()
        rc = self._L.sod_create(int(device), C.byref(h))
        if rc != SOD_OK:
            raise SodError(rc, self._L.sod_last_error(None).decode())
        self._h = h
        self.device = device
        self.nq = 0
        self.n_total = 0
        self.bins = None
        self.db_gen = 0      # counts DB uploads / shares / impl switches (residency checks)
        # the outlier test's M.X rounding of the reference on this host (AffineParameters.py:145)
        self._chk(self._L.sod_set_option(self._h, b"affine_fma", numpy_matmul_fma()))

    # -- plumbing --
    def _chk(self, rc):
        if rc != SOD_OK:
            raise SodError(rc, self._L.sod_last_error(self._h).decode())

    def close(self):
        if getattr(self, "_h", None):
            self._L.sod_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def synchronize(self):
        self._chk(self._L.sod_synchronize(self._h))

    # -- data --
    def set_keypoints(self, kp, img, centroid, size):
        self._kp_keep = (_c(kp.x, np.float32), _c(kp.y, np.float32), _c(kp.angle, np.float32),
                         _c(kp.octave, np.int32), _c(img, np.int32),
                         _c(centroid, np.float64).reshape(-1), _c(size, np.int32).reshape(-1))
        x, y, a, o, im, ce, sz = self._kp_keep
        self._chk(self._L.sod_db_set_keypoints(
            self._h, len(x), ptr(x, C.c_float), ptr(y, C.c_float), ptr(a, C.c_float),
            ptr(o, C.c_int32), ptr(im, C.c_int32), len(ce) // 2, ptr(ce, C.c_double),
            ptr(sz, C.c_int32)))
        self.n_total = len(x)
        del self._kp_keep

    @staticmethod
    def _des(des):
        des = np.asarray(des)
        if des.ndim != 2 or des.shape[1] != 128:
            raise ValueError("descriptors must be [N,128]")
        if des.dtype == np.uint8:
            return np.ascontiguousarray(des), DTYPE_U8
        return np.ascontiguousarray(des, dtype=np.float32), DTYPE_F32

    def upload_db(self, des, row_offset=0):
        d, dt = self._des(des)
        self._chk(self._L.sod_db_upload_descriptors(self._h, d.ctypes.data_as(c_vp), dt,
                                                     d.shape[0], int(row_offset)))
        self.db_gen += 1
        self.n_shard = d.shape[0]
        self.row_offset = int(row_offset)

    def upload_queries(self, des, kp=None):
        if des is None:
            if kp is None:
                raise ValueError("need descriptors or keypoints")
            d, dt, n = None, DTYPE_U8, len(kp)
        else:
            d, dt = self._des(des)
            n = d.shape[0]
        if kp is not None:
            x, y, a, o = (_c(kp.x, np.float32), _c(kp.y, np.float32), _c(kp.angle, np.float32),
                          _c(kp.octave, np.int32))
            if len(x) != n:
                raise ValueError("query keypoints and descriptors differ in count")
            args = (ptr(x, C.c_float), ptr(y, C.c_float), ptr(a, C.c_float), ptr(o, C.c_int32))
        else:
            args = (None, None, None, None)
        self._chk(self._L.sod_query_upload(self._h, None if d is None else d.ctypes.data_as(c_vp),
                                           dt, n, *args))
        self.nq = n

    def set_matches(self, idx1, good):
        i = _c(idx1, np.int32)
        g = _c(np.asarray(good).astype(np.uint8), np.uint8)
        self._chk(self._L.sod_matches_set(self._h, len(i), ptr(i, C.c_int32), ptr(g, C.c_uint8)))

    IMPLS = {"bf16": 0, "i8": 1, "i8w": 2}

    def set_impl(self, impl):
        """Matcher implementation "i8" (int8 16x16x64, default), "bf16" or "i8w" (int8
        32x32x32); call before uploads."""
        self._chk(self._L.sod_match_set_impl(self._h, self.IMPLS[impl] if isinstance(impl, str)
                                             else int(impl)))
        self.db_gen += 1

    def host_wait_ms(self, reset=True):
        """Host time (ms) enqueue calls spent blocked on the device (the partial-result slot
        wait) since the last reset (sod_host_wait_ns)."""
        v = C.c_int64()
        self._chk(self._L.sod_host_wait_ns(self._h, C.byref(v), 1 if reset else 0))
        return v.value / 1e6

    def trig_exact(self):
        """True when the device's cos / sin are this host's libm bit for bit (then poses,
        bins and PoseBin means equal the reference's without any host redo)."""
        return self._L.sod_trig_exact(self._h) == 1

    def glibc_sincos(self, x):
        """The device's glibc sin / cos of the angles x (test hook)."""
        x = np.ascontiguousarray(x, np.float64)
        s, c = np.empty_like(x), np.empty_like(x)
        self._chk(self._L.sod_glibc_sincos(self._h, len(x), x.ctypes.data_as(C.c_void_p),
                                           s.ctypes.data_as(C.c_void_p), c.ctypes.data_as(C.c_void_p)))
        return s, c

    KERNELS = {"auto": 0, "ring": 1}

    OPTIONS = ("match_qt", "match_pf", "match_pair", "hough_fused", "select_multi", "sift_stream_mask",
               "sift_sort_max", "sift_desc_range_max", "sift_layer_split", "sift_side_mask",
               "sift_fork2", "sift_early_desc", "sift_direct", "sift_eager_rank", "debug_sync",
               "affine_fma", "trig_exact")

    def set_option(self, name, value):
        """A tuning / test switch of this context by name (sod.h sod_set_option); returns the
        previous value.  None of them changes results."""
        old = self.get_option(name)
        self._chk(self._L.sod_set_option(self._h, name.encode(), int(value)))
        return old

    def get_option(self, name):
        v = C.c_int64()
        self._chk(self._L.sod_get_option(self._h, name.encode(), C.byref(v)))
        return v.value

    def set_match_kernel(self, kernel):
        """Kernel shape of the int8 matcher: "auto" (by query count, default) or "ring" (the LDS
        ring kernel, the only shape since round 6); results are identical."""
        self._chk(self._L.sod_match_set_kernel(self._h, self.KERNELS[kernel] if isinstance(kernel, str)
                                               else int(kernel)))

    def set_overlap(self, on=True):
        """Matcher kernel on a stream of its own: the next query's matcher overlaps this
        one's Hough / select / affine stages (sod_match_set_overlap); results unchanged."""
        self._chk(self._L.sod_match_set_overlap(self._h, 1 if on else 0))

    def set_cu_reserve(self, per_xcd=1):
        """Run the matcher on all but `per_xcd` CUs of every XCD and the other stages (and
        RCCL exchanges) on those, so a query's tail overlaps the next matcher instead of
        being starved by it (sod_set_cu_reserve; implies set_overlap).  0 undoes it."""
        self._chk(self._L.sod_set_cu_reserve(self._h, int(per_xcd)))

    # -- stages --
    def match(self):
        self._chk(self._L.sod_match_enqueue(self._h))

    def match_allgather(self):
        self._chk(self._L.sod_match_allgather_enqueue(self._h))

    def ratio(self, ratio=0.75):
        self._chk(self._L.sod_ratio_enqueue(self._h, float(ratio)))

    def match_result(self):
        n = self.nq
        idx1 = np.empty(n, np.int32)
        d1 = np.empty(n, np.float32)
        d2 = np.empty(n, np.float32)
        good = np.empty(n, np.uint8)
        self._chk(self._L.sod_match_get(self._h, ptr(idx1, C.c_int32), ptr(d1, C.c_float),
                                        ptr(d2, C.c_float), ptr(good, C.c_uint8)))
        return idx1, d1, d2, good.astype(bool)

    def knn_indices(self):
        """knnMatch's (m.trainIdx, n.trainIdx) per query, OpenCV's float-distance order
        (sod_match_knn_indices; int8 16x16x64 or bf16 matcher)."""
        i1 = np.empty(self.nq, np.int32)
        i2 = np.empty(self.nq, np.int32)
        self._chk(self._L.sod_match_knn_indices(self._h, ptr(i1, C.c_int32), ptr(i2, C.c_int32)))
        return i1, i2

    def float_order(self):
        """The device's trainIdx becomes OpenCV's float-order one (sod_match_float_order; a
        no-op when exact_order() holds)."""
        self._chk(self._L.sod_match_float_order(self._h))

    def exact_order(self):
        v = C.c_int()
        self._chk(self._L.sod_match_exact_order(self._h, C.byref(v)))
        return bool(v.value)

    def hough(self, query_shape, bins, own=None):
        b = np.ascontiguousarray(bins4(bins), np.int32)
        lo, hi = own if own is not None else (0, self.n_total)
        self._chk(self._L.sod_hough_enqueue(self._h, int(query_shape[0]), int(query_shape[1]),
                                            ptr(b, C.c_int32), int(lo), int(hi)))
        self.bins = tuple(int(v) for v in b)

    def hough_allreduce(self):
        self._chk(self._L.sod_hough_allreduce_enqueue(self._h))

    def select(self, vote_threshold=5):
        self._chk(self._L.sod_select_enqueue(self._h, int(vote_threshold)))

    def hough_select(self, query_shape, bins, vote_threshold=5):
        """Hough + select in one call (sod_hough_select_enqueue): one fused launch for one image
        of <= 1024 queries (kFusedQ) on one rank, else hough() + select()."""
        b = np.ascontiguousarray(bins4(bins), np.int32)
        self._chk(self._L.sod_hough_select_enqueue(self._h, int(query_shape[0]),
                                                   int(query_shape[1]), ptr(b, C.c_int32),
                                                   int(vote_threshold)))
        self.bins = tuple(int(v) for v in b)

    def valid_counts(self):
        v, m = C.c_int64(), C.c_int64()
        self._chk(self._L.sod_valid_counts(self._h, C.byref(v), C.byref(m)))
        return v.value, m.value

    def valid_result(self):
        V, M = self.valid_counts()
        keys = np.empty((V, 4), np.int32)
        votes = np.empty(V, np.int32)
        off = np.empty(V + 1, np.int64)
        mem = np.empty(M, np.int32)
        means = np.empty((V, 6), np.float64)
        self._chk(self._L.sod_valid_get(self._h, ptr(keys, C.c_int32), ptr(votes, C.c_int32),
                                        ptr(off, C.c_int64), ptr(mem, C.c_int32),
                                        ptr(means, C.c_double)))
        return {"keys": keys, "votes": votes, "offsets": off, "members": mem, "means": means}

    def all_bins(self):
        n = C.c_int64()
        self._chk(self._L.sod_bins_count(self._h, C.byref(n)))
        keys = np.empty((n.value, 4), np.int32)
        votes = np.empty(n.value, np.int32)
        self._chk(self._L.sod_bins_get(self._h, ptr(keys, C.c_int32), ptr(votes, C.c_int32)))
        return keys, votes

    def guard_stats(self):
        """Boundary guard of the last Hough launch / pose batch (sod_hough_guard_stats):
        (listed matches, changed bins, listed total, changed total)."""
        v = [C.c_int64() for _ in range(4)]
        self._chk(self._L.sod_hough_guard_stats(self._h, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def affine(self, query_size, x_factor=128.0, y_factor=128.0, threshold=4):
        self._chk(self._L.sod_affine_enqueue(self._h, int(query_size[0]), int(query_size[1]),
                                             float(x_factor), float(y_factor), int(threshold)))

    def affine_result(self):
        V, M = self.valid_counts()
        surv = np.empty(V, np.uint8)
        votes = np.empty(V, np.int32)
        params = np.empty((V, 6), np.float64)
        alive = np.empty(M, np.uint8)
        self._chk(self._L.sod_affine_get(self._h, ptr(surv, C.c_uint8), ptr(votes, C.c_int32),
                                         ptr(params, C.c_double), ptr(alive, C.c_uint8)))
        return {"survived": surv.astype(bool), "votes": votes, "params": params,
                "alive": alive.astype(bool)}

    RES = {"match": 1, "valid": 2, "affine": 4, "post": 8}

    def results(self, post=True, parts=None):
        """Results of the last pipeline in one device -> host transfer (sod_results_fetch):
        {"match": (idx1, d1, d2, good), "valid": valid_result()'s dict, "affine":
        affine_result()'s dict, "post": postprocess()'s dict} -- of ``parts`` (names; default
        all, without "post" when post is False) that were enqueued; the same values as those
        getters."""
        if parts is None:
            parts = ("match", "valid", "affine") + (("post",) if post else ())
        mask = 0
        for p in parts:
            mask |= self.RES[p]
        rs = Results()
        self._chk(self._L.sod_results_fetch(self._h, mask, C.byref(rs)))
        if _RESPARSE is not None:
            return _RESPARSE.results(C.addressof(rs), mask)
        return _results_from_struct(rs, mask)

    def pipeline(self, query_shape, bins=15, ratio=0.75, vote_threshold=5, affine_threshold=4,
                 x_factor=128.0, y_factor=128.0, run_affine=True, stage=()):
        """The whole path in one enqueue (sod_pipeline_enqueue); ``stage``: result parts
        ("match", "valid", "affine", "post") staged right behind it, so that the next
        ``results()`` of those parts only waits."""
        # the argument struct of the last call is reused when every argument is equal (a run
        # of images: its ~15 field writes sit before the matcher launch); the key holds
        # immutable values (bins4's tuple, the stage tuple), never a caller's mutable object
        b4 = bins4(bins)
        key = (query_shape[0], query_shape[1], b4, ratio, vote_threshold, affine_threshold,
               x_factor, y_factor, run_affine, tuple(stage))
        if key == self._pargs_key:
            a = self._pargs
        else:
            a = PipelineArgs()
            for p in stage:
                a.stage_parts |= self.RES[p]
            a.ratio = float(ratio)
            a.query_h, a.query_w = int(query_shape[0]), int(query_shape[1])
            for i, v in enumerate(b4):
                a.bins[i] = v
            a.vote_threshold = int(vote_threshold)
            a.affine_threshold = int(affine_threshold)
            a.x_factor, a.y_factor = float(x_factor), float(y_factor)
            a.run_affine = 1 if run_affine else 0
            self._pargs_key, self._pargs = key, a
        self._chk(self._L.sod_pipeline_enqueue(self._h, C.byref(a)))
        self.bins = b4

    def last_match_ms(self):
        v = C.c_float()
        self._chk(self._L.sod_last_match_ms(self._h, C.byref(v)))
        return v.value

    def match_times(self, n):
        """Kernel times (ms) of the last n matcher launches, oldest first (n <= 64)."""
        out = np.zeros(int(n), np.float32)
        self._chk(self._L.sod_match_times(self._h, int(n), ptr(out, C.c_float)))
        return out

    def set_match_timing(self, on):
        """Matcher launch events (sod_set_match_timing; default off): True = every launch, False / 0
        records none, an int s every s-th launch from now on."""
        stride = int(on) if not isinstance(on, bool) else (1 if on else 0)
        self._chk(self._L.sod_set_match_timing(self._h, stride))

    def exact_means(self, vbin):
        """(len(vbin), 2) x / y PoseBin means of those valid bins as the reference computes
        them (sod_exact_means)."""
        vb = np.ascontiguousarray(vbin, np.int32)
        out = np.zeros((len(vb), 2), np.float64)
        self._chk(self._L.sod_exact_means(self._h, len(vb), ptr(vb, C.c_int32), ptr(out, C.c_double)))
        return out

    def set_post_exact(self, on):
        """postprocess() on the survivors' x / y means redone with glibc (default True)."""
        self._chk(self._L.sod_set_post_exact(self._h, 1 if on else 0))

    def set_matcher_streams(self, n):
        """1 (default) or 2 matcher streams (sod_set_matcher_streams)."""
        self._chk(self._L.sod_set_matcher_streams(self._h, int(n)))

    def set_stage_timing(self, on):
        """Record the per-stage events read by stage_ms (default off: each event delays the
        stream's next kernel)."""
        self._chk(self._L.sod_set_stage_timing(self._h, 1 if on else 0))

    STAGES = ("match_kernel", "merge_ratio", "hough_vote", "select", "affine", "allreduce",
              "allgather")

    def stage_ms(self):
        """Device time (ms) of each stage's own launches in the last step, in STAGES order
        (sod_last_stage_ms): host work and waits between the calls are not counted."""
        out = np.zeros(len(self.STAGES), np.float32)
        self._chk(self._L.sod_last_stage_ms(self._h, ptr(out, C.c_float), len(out)))
        return out

    # -- stateless batch forms --
    def pose_batch(self, mx, my, mang, moct, qx, qy, qang, qoct, cx, cy, query_shape, bins):
        arr = [_c(mx, np.float32), _c(my, np.float32), _c(mang, np.float32), _c(moct, np.int32),
               _c(qx, np.float32), _c(qy, np.float32), _c(qang, np.float32), _c(qoct, np.int32),
               _c(cx, np.float64), _c(cy, np.float64)]
        n = len(arr[0])
        if any(len(a) != n for a in arr):
            raise ValueError("pose_batch arrays differ in length")
        b = np.ascontiguousarray(bins4(bins), np.int32)
        pose = np.empty((n, 4), np.float64)
        idx = np.empty((n, 4), np.int32)
        ct = [C.c_float, C.c_float, C.c_float, C.c_int32, C.c_float, C.c_float, C.c_float,
              C.c_int32, C.c_double, C.c_double]
        self._chk(self._L.sod_pose_batch(self._h, n, *[ptr(a, t) for a, t in zip(arr, ct)],
                                         int(query_shape[0]), int(query_shape[1]),
                                         ptr(b, C.c_int32), ptr(pose, C.c_double),
                                         ptr(idx, C.c_int32)))
        return pose, idx

    def bin_index_batch(self, pose, query_shape, bins):
        p = _c(pose, np.float64).reshape(-1, 4)
        b = np.ascontiguousarray(bins4(bins), np.int32)
        idx = np.empty((len(p), 4), np.int32)
        self._chk(self._L.sod_bin_index_batch(self._h, len(p), ptr(p, C.c_double),
                                              int(query_shape[0]), int(query_shape[1]),
                                              ptr(b, C.c_int32), ptr(idx, C.c_int32)))
        return idx

    # -- host-side exchange (multi-rank without RCCL) --
    def candidates(self):
        n = self.nq
        d1 = np.empty(n, np.float32)
        idx = np.empty(n, np.int32)
        d2 = np.empty(n, np.float32)
        self._chk(self._L.sod_match_candidates_get(self._h, ptr(d1, C.c_float),
                                                   ptr(idx, C.c_int32), ptr(d2, C.c_float)))
        return d1, idx, d2

    def merge_candidates(self, d1, idx, d2):
        d1 = _c(d1, np.float32)
        idx = _c(idx, np.int32)
        d2 = _c(d2, np.float32)
        nparts = d1.size // self.nq
        self._chk(self._L.sod_match_candidates_merge(self._h, nparts, ptr(d1, C.c_float),
                                                     ptr(idx, C.c_int32), ptr(d2, C.c_float)))

    def hough_partial(self):
        n = int(np.prod(self.bins))
        cnt = np.empty(n, np.uint32)
        fst = np.empty(n, np.uint32)
        self._chk(self._L.sod_hough_partial_get(self._h, ptr(cnt, C.c_uint32), ptr(fst, C.c_uint32)))
        return cnt, fst

    def set_hough_partial(self, counts, first):
        cnt = _c(counts, np.uint32)
        fst = _c(first, np.uint32)
        self._chk(self._L.sod_hough_partial_set(self._h, ptr(cnt, C.c_uint32), ptr(fst, C.c_uint32)))

    def affine_batch(self, offsets, mx, my, qx, qy, i_sigma, query_size, x_factor=128.0,
                     y_factor=128.0, threshold=4, max_iter=1 << 30, params_in=None):
        off = _c(offsets, np.int64)
        nb = len(off) - 1
        pts = [_c(v, np.float32) for v in (mx, my, qx, qy)]
        isg = _c(i_sigma, np.int32)
        M = int(off[-1]) if nb >= 0 else 0
        surv = np.empty(nb, np.uint8)
        votes = np.empty(nb, np.int32)
        params = np.empty((nb, 6), np.float64)
        alive = np.empty(M, np.uint8)
        pin = None if params_in is None else _c(params_in, np.float64).reshape(-1)
        self._chk(self._L.sod_affine_batch(
            self._h, nb, ptr(off, C.c_int64), *[ptr(p, C.c_float) for p in pts],
            ptr(isg, C.c_int32), int(query_size[0]), int(query_size[1]), float(x_factor),
            float(y_factor), int(threshold), int(max_iter), ptr(pin, C.c_double),
            ptr(surv, C.c_uint8),
            ptr(votes, C.c_int32), ptr(params, C.c_double), ptr(alive, C.c_uint8)))
        return {"survived": surv.astype(bool), "votes": votes, "params": params,
                "alive": alive.astype(bool)}

    def _post_arrays(self, n):
        return dict(n_pos=C.c_int32(0), n_ori=C.c_int32(0),
                    pos_off=np.empty(n + 1, np.int32), pos_members=np.empty(max(n, 1), np.int32),
                    ori_pos_off=np.empty(n + 1, np.int32), ori_off=np.empty(n + 1, np.int32),
                    ori_members=np.empty(max(n, 1), np.int32),
                    orient=np.empty(max(n, 1), np.float64), pose=np.empty((max(n, 1), 6), np.float64))

    @staticmethod
    def _post_result(a, n):
        npos, nori = a["n_pos"].value, a["n_ori"].value
        return {"pos_off": a["pos_off"][:npos + 1].copy(), "pos_members": a["pos_members"][:n].copy(),
                "ori_pos_off": a["ori_pos_off"][:npos + 1].copy(),
                "ori_off": a["ori_off"][:nori + 1].copy(), "ori_members": a["ori_members"][:n].copy(),
                "final_orientation": a["orient"][:npos].copy(), "final_pose": a["pose"][:npos].copy()}

    def _post_call(self, fn, *head, n, a):
        self._chk(fn(self._h, *head, C.byref(a["n_pos"]), ptr(a["pos_off"], C.c_int32),
                     ptr(a["pos_members"], C.c_int32), C.byref(a["n_ori"]),
                     ptr(a["ori_pos_off"], C.c_int32), ptr(a["ori_off"], C.c_int32),
                     ptr(a["ori_members"], C.c_int32), ptr(a["orient"], C.c_double),
                     ptr(a["pose"], C.c_double)))
        return self._post_result(a, n)

    # -- SIFT on the device --
    def sift_params(self, n_octave_layers=3, contrast_threshold=0.04, edge_threshold=10.0,
                    sigma=1.6):
        self._chk(self._L.sod_sift_set_params(self._h, int(n_octave_layers),
                                              float(contrast_threshold), float(edge_threshold),
                                              float(sigma)))

    def sift_set_lane_order(self, mode=-1):
        """Histogram adds: -1 = wave adds when the device self-check holds, 0 = ordered
        single-lane adds (sod_sift_set_lane_order)."""
        self._chk(self._L.sod_sift_set_lane_order(self._h, int(mode)))

    def sift_lane_order(self):
        """(active path: 1 wave adds / 0 ordered, self-check: 1 held / 0 failed / -1 not run)."""
        a, p = C.c_int(), C.c_int()
        self._chk(self._L.sod_sift_lane_order(self._h, C.byref(a), C.byref(p)))
        return a.value, p.value

    def sift_detect(self, image, descriptors=True):
        """detectAndCompute on an 8-bit gray [h, w] or BGR [h, w, 3|4] image: SoA keypoints
        (x, y, size, angle, response, octave) in OpenCV's order (+ float32 [n, 128])."""
        img = np.asarray(image)
        if img.dtype != np.uint8:
            raise TypeError("SIFT input must be an 8-bit image")
        n = C.c_int32()
        if img.ndim == 2:
            g = _c(img, np.uint8)
            self._chk(self._L.sod_sift_detect(self._h, ptr(g, C.c_uint8), g.shape[1], g.shape[0],
                                              C.byref(n)))
        elif img.ndim == 3 and img.shape[2] in (3, 4):
            b = _c(img[:, :, :3], np.uint8)
            self._chk(self._L.sod_sift_detect_bgr(self._h, ptr(b, C.c_uint8), b.shape[1],
                                                  b.shape[0], C.byref(n)))
        else:
            raise ValueError("SIFT input must be [h, w] or [h, w, 3|4]")
        self._sift_n = n.value
        return self._sift_get(n.value, descriptors)

    def _sift_get(self, n, descriptors):
        out = {k: np.zeros(n, np.float32) for k in ("x", "y", "size", "angle", "response")}
        out["octave"] = np.zeros(n, np.int32)
        desc = np.zeros((n, 128), np.float32) if descriptors else None
        self._chk(self._L.sod_sift_get(
            self._h, n, ptr(out["x"], C.c_float), ptr(out["y"], C.c_float),
            ptr(out["size"], C.c_float), ptr(out["angle"], C.c_float),
            ptr(out["response"], C.c_float), ptr(out["octave"], C.c_int32),
            ptr(desc, C.c_float)))
        if descriptors:
            out["descriptors"] = desc
        return out

    def sift_detect_batch(self, images, descriptors=True, results=True):
        """detectAndCompute on several 8-bit images (gray [h, w] or BGR [h, w, 3|4]), four
        in flight at once.  Returns one SoA dict per image (``results=False``: only the
        counts; the features stay on the device for ``sift_to_queries``)."""
        imgs = []
        for im in images:
            a = np.asarray(im)
            if a.dtype != np.uint8 or a.ndim not in (2, 3) or (a.ndim == 3 and a.shape[2] not in (3, 4)):
                raise ValueError("SIFT inputs must be 8-bit [h, w] or [h, w, 3|4] images")
            imgs.append(_c(a if a.ndim == 2 else a[:, :, :3], np.uint8))
        n = len(imgs)
        ptrs = (c_u8p * n)(*[ptr(a, C.c_uint8) for a in imgs])
        w = np.array([a.shape[1] for a in imgs], np.int32)
        h = np.array([a.shape[0] for a in imgs], np.int32)
        ch = np.array([1 if a.ndim == 2 else 3 for a in imgs], np.int32)
        counts = np.zeros(n, np.int32)
        self._chk(self._L.sod_sift_detect_batch(self._h, n, ptrs, ptr(w, C.c_int32),
                                                ptr(h, C.c_int32), ptr(ch, C.c_int32),
                                                ptr(counts, C.c_int32)))
        self._sift_n = int(counts.sum())
        self._sift_counts = counts
        if not results:
            return counts
        allr = self._sift_get(self._sift_n, descriptors)
        off = np.concatenate([[0], np.cumsum(counts)])
        return [{k: v[off[i]:off[i + 1]] for k, v in allr.items()} for i in range(n)]

    def sift_to_queries(self):
        """The last SIFT detection becomes the query set (device to device)."""
        self._chk(self._L.sod_sift_to_queries(self._h))
        self.nq = self._sift_n

    def post_batch(self, means):
        """PostProcessing.py:4-112 on PoseBin means [n, 6] = (x, y, angle, scale, w, h)."""
        m = _c(means, np.float64).reshape(-1, 6)
        n = len(m)
        a = self._post_arrays(n)
        return self._post_call(self._L.sod_post_batch, n, ptr(m, C.c_double), n=n, a=a)

    def postprocess(self):
        """main.py:159-168 on the pipeline's surviving (or valid) bins; ``bin_index`` maps
        the post-processed list to valid-bin indices.  One device -> host transfer
        (sod_results_fetch, SOD_RES_POST); ``postprocess_getter`` is the sod_postprocess
        form (the same outputs)."""
        return self.results(parts=("post",))["post"]

    def postprocess_getter(self):
        V, _ = self.valid_counts()
        a = self._post_arrays(V)
        nb = C.c_int32(0)
        idx = np.empty(max(V, 1), np.int32)
        r = self._post_call(self._L.sod_postprocess, C.byref(nb), ptr(idx, C.c_int32), n=V, a=a)
        n = nb.value
        r["bin_index"] = idx[:n].copy()
        r["pos_members"] = r["pos_members"][:n]
        r["ori_members"] = r["ori_members"][:n]
        return r

    def query_window(self, first=0, count=-1):
        """Restrict the Hough-side stages to queries [first, first+count) (one image of a
        batch matched together); count < 0 = all queries."""
        self._chk(self._L.sod_query_window(self._h, int(first), int(count)))

    def share_db(self, src):
        """Use ``src``'s resident database (no copy); ``src`` must outlive this context."""
        self._chk(self._L.sod_db_share(self._h, src._h))
        self.db_gen += 1
        self.n_total = src.n_total
        self._db_src = src

    def query_images(self, offsets, shapes):
        """Declare the uploaded queries as a batch of images (offsets [n+1], shapes [n, 2+]
        = rgb_query.shape) for fused per-image stages; an empty list returns to one image."""
        off = _c(offsets, np.int32)
        n = max(0, len(off) - 1)
        shp = np.ascontiguousarray(np.asarray(shapes, np.int64)[:, :2], np.int32) if n else \
            np.zeros((0, 2), np.int32)
        self._chk(self._L.sod_query_images(self._h, n, ptr(off, C.c_int32), ptr(shp, C.c_int32)))

    def valid_images(self):
        V, _ = self.valid_counts()
        img = np.empty(max(V, 1), np.int32)
        self._chk(self._L.sod_valid_images_get(self._h, ptr(img, C.c_int32)))
        return img[:V]

    def export_packed(self):
        """The DB shard as a packed image (uint8 array): header + fragments + norm words."""
        n = C.c_int64(0)
        self._chk(self._L.sod_db_packed_size(self._h, C.byref(n)))
        out = np.empty(n.value, np.uint8)
        self._chk(self._L.sod_db_export_packed(self._h, out.ctypes.data_as(c_vp), n.value))
        return out

    def import_packed(self, image):
        """Upload a packed DB image (one host->device copy, no packing pass)."""
        a = np.ascontiguousarray(image, np.uint8)
        self._chk(self._L.sod_db_import_packed(self._h, a.ctypes.data_as(c_vp), a.size))

    def comm_init(self, nranks, rank, uid):
        buf = (C.c_uint8 * UNIQUE_ID_BYTES).from_buffer_copy(uid)
        self._chk(self._L.sod_comm_init(self._h, int(nranks), int(rank), C.byref(buf)))

    def comm_info(self):
        """(nranks, rank) of this context's RCCL communicator as RCCL reports them
        (sod_comm_info: ncclCommCount / ncclCommUserRank)."""
        n, r = C.c_int32(), C.c_int32()
        self._chk(self._L.sod_comm_info(self._h, C.byref(n), C.byref(r)))
        return n.value, r.value


def bins4(bins):
    """``bins`` as the live code passes it (one int, main.py:183) or per axis
    (x, y, theta, sigma) following ``HoughTransform.py:8``."""
    if isinstance(bins, (tuple, list, np.ndarray)):
        b = tuple(int(v) for v in bins)
        if len(b) != 4:
            raise ValueError("bins must be an int or a 4-tuple (x, y, theta, sigma)")
        return b
    b = int(bins)
    return (b, b, b, b)


_default = {}


def device_count():
    """HIP devices visible to this process (sod_device_count)."""
    n = C.c_int()
    rc = lib().sod_device_count(C.byref(n))
    if rc != SOD_OK:
        raise SodError(rc, lib().sod_last_error(None).decode())
    return n.value


def default_context(device=0):
    """Process-wide context for the drop-in functions (one per device)."""
    ctx = _default.get(device)
    if ctx is None:
        ctx = Context(device)
        _default[device] = ctx
    return ctx
