"""ctypes mirror of include/tvl1.h (the C-ABI boundary).

This is the binding a Python caller (tests, bench.py) uses; the production
caller is the C++ `optflow` CLI (fibsem-optflow_amd/cli/optflow.cpp), which
links the same library.  Mirrors the reference boundary
/root/reference/src/optflow.cpp:516-520 (TVL1_solve) — see include/tvl1.h.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parent.parent          # fibsem-optflow_amd/
REPO_ROOT = PKG_ROOT.parent
ENGINE_SO = PKG_ROOT / "lib" / "libtvl1_hip.so"

TVL1_MAX_LEVELS = 32
ABI_VERSION = 9          # TVL1_ABI_VERSION of include/tvl1.h
STATUS = {0: "TVL1_OK", 1: "TVL1_EINVAL", 2: "TVL1_ESIZE", 3: "TVL1_EHIP",
          4: "TVL1_ENOMEM", 5: "TVL1_ENODEV"}


class TVL1Params(C.Structure):
    _fields_ = [
        ("tau", C.c_double),
        ("lambda_", C.c_double),
        ("theta", C.c_double),
        ("nscales", C.c_int32),
        ("warps", C.c_int32),
        ("epsilon", C.c_double),
        ("iterations", C.c_int32),
        ("scale_step", C.c_double),
        ("gamma", C.c_double),
        ("use_initial_flow", C.c_int32),
        ("median_filtering", C.c_int32),
        ("fast_math", C.c_int32),
        ("profile", C.c_int32),
        ("inner_iterations", C.c_int32),
        ("outer_iterations", C.c_int32),
    ]


class TVL1Stats(C.Structure):
    _fields_ = [
        ("levels", C.c_int32),
        ("level_width", C.c_int32 * TVL1_MAX_LEVELS),
        ("level_height", C.c_int32 * TVL1_MAX_LEVELS),
        ("level_iterations", C.c_int64 * TVL1_MAX_LEVELS),
        ("iterations_total", C.c_int64),
        ("checks_total", C.c_int64),
        ("algorithmic_bytes", C.c_double),
        ("warp_iterations", C.POINTER(C.c_int32)),
        ("warp_iterations_capacity", C.c_int32),
        ("speculation_misses", C.c_int32),
        ("kernel_ms", C.c_double * 4),
        ("kernel_launches", C.c_int64 * 4),
        ("kernel_bytes", C.c_double * 4),
        ("kernel_hbm_bytes", C.c_double * 4),
    ]


class TVL1AlignParams(C.Structure):
    """tvl1_align_params (include/tvl1.h): orb_defaults (features.cpp:19-31) + ratio / homo /
    ransac (:109, :133)."""
    _fields_ = [
        ("nfeatures", C.c_int32),
        ("scale_factor", C.c_float),
        ("nlevels", C.c_int32),
        ("edge_threshold", C.c_int32),
        ("first_level", C.c_int32),
        ("wta_k", C.c_int32),
        ("patch_size", C.c_int32),
        ("fast_threshold", C.c_int32),
        ("blur_for_descriptor", C.c_int32),
        ("ratio", C.c_float),
        ("method", C.c_int32),
        ("ransac_threshold", C.c_double),
    ]


# generate_TV_args defaults, /root/reference/src/optflow.cpp:503-512
DEFAULTS = dict(tau=0.25, lambda_=0.05, theta=0.3, nscales=10, warps=5, epsilon=0.01,
                iterations=300, scale_step=0.8, gamma=0.0, use_initial_flow=0,
                median_filtering=1, fast_math=0, profile=0, inner_iterations=30,
                outer_iterations=10)

# JSON key -> struct field (JSON keys are the reference's, optflow.cpp:503-512)
JSON_KEYS = {"tau": "tau", "lambda": "lambda_", "theta": "theta", "nscales": "nscales",
             "warps": "warps", "epsilon": "epsilon", "iterations": "iterations",
             "scaleStep": "scale_step", "gamma": "gamma", "useInitialFlow": "use_initial_flow",
             "medianFiltering": "median_filtering", "fastMath": "fast_math",
             "profile": "profile", "innerIterations": "inner_iterations",
             "outerIterations": "outer_iterations"}


def make_params(**kw) -> TVL1Params:
    d = dict(DEFAULTS)
    for k, v in kw.items():
        k = JSON_KEYS.get(k, k)
        if k == "lambda":
            k = "lambda_"
        if k not in d:
            raise KeyError(f"unknown TV-L1 parameter {k!r}")
        d[k] = v
    p = TVL1Params()
    for k, v in d.items():
        setattr(p, k, v)
    return p


def stats_dict(st: TVL1Stats, warps: int | None = None) -> dict:
    L = st.levels
    out = {
        "levels": L,
        "sizes": [(st.level_width[i], st.level_height[i]) for i in range(L)],
        "level_iterations": [int(st.level_iterations[i]) for i in range(L)],
        "iterations_total": int(st.iterations_total),
        "checks_total": int(st.checks_total),
        "speculation_misses": int(st.speculation_misses),
        "algorithmic_bytes": float(st.algorithmic_bytes),
        "kernel_ms": [float(st.kernel_ms[i]) for i in range(4)],
        "kernel_launches": [int(st.kernel_launches[i]) for i in range(4)],
        "kernel_bytes": [float(st.kernel_bytes[i]) for i in range(4)],
        "kernel_hbm_bytes": [float(st.kernel_hbm_bytes[i]) for i in range(4)],
    }
    return out


def _u8_ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def _f32_ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class Library:
    """Loads the HIP engine library."""

    def __init__(self, path: Path):
        if not Path(path).exists():
            raise FileNotFoundError(f"{path} not built (run __graft_entry__.build())")
        self.path = Path(path)
        self.lib = C.CDLL(str(path))


def load_engine() -> C.CDLL:
    """The product: libtvl1_hip.so (HIP kernels for gfx950 + C-ABI).  Raises
    if it was not built — there is no CPU fallback."""
    # TVL1_ENGINE_SO: another build of the same engine (A/B runs of tools/ab_lib.sh)
    path = Path(os.environ.get("TVL1_ENGINE_SO", ENGINE_SO))
    lib = Library(path).lib
    lib.tvl1_params_default.argtypes = [C.POINTER(TVL1Params)]
    lib.tvl1_params_default.restype = None
    lib.tvl1_create.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.POINTER(TVL1Params)]
    lib.tvl1_create.restype = C.c_int
    lib.tvl1_set_params.argtypes = [C.c_void_p, C.POINTER(TVL1Params)]
    lib.tvl1_set_params.restype = C.c_int
    lib.tvl1_calc.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                              C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_size_t,
                              C.POINTER(TVL1Stats), C.c_void_p]
    lib.tvl1_calc.restype = C.c_int
    lib.tvl1_calc_f32.argtypes = lib.tvl1_calc.argtypes
    lib.tvl1_calc_f32.restype = C.c_int
    lib.tvl1_calc_batch.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_size_t, C.c_size_t,
                                    C.c_void_p, C.c_size_t, C.c_size_t, C.c_int32, C.c_int32,
                                    C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                    C.POINTER(TVL1Stats), C.c_void_p]
    lib.tvl1_calc_batch.restype = C.c_int
    lib.tvl1_align_params_default.argtypes = [C.POINTER(TVL1AlignParams)]
    lib.tvl1_align_params_default.restype = None
    lib.tvl1_find_alignment.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int32, C.c_int32,
                                        C.c_void_p, C.c_size_t, C.c_int32, C.c_int32,
                                        C.POINTER(TVL1AlignParams), C.POINTER(C.c_float),
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_void_p]
    lib.tvl1_find_alignment.restype = C.c_int
    lib.tvl1_orb_detect.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int32, C.c_int32,
                                    C.POINTER(TVL1AlignParams), C.c_void_p, C.c_void_p, C.c_int32,
                                    C.POINTER(C.c_int32), C.c_void_p]
    lib.tvl1_orb_detect.restype = C.c_int
    lib.tvl1_match_knn2.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32,
                                    C.c_void_p, C.c_void_p, C.c_void_p]
    lib.tvl1_match_knn2.restype = C.c_int
    lib.tvl1_warp_affine_u8.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int32, C.c_int32,
                                        C.c_void_p, C.c_size_t, C.c_int32, C.c_int32,
                                        C.POINTER(C.c_float), C.c_void_p]
    lib.tvl1_warp_affine_u8.restype = C.c_int
    lib.tvl1_find_homography.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_double,
                                         C.POINTER(C.c_double), C.c_void_p]
    lib.tvl1_find_homography.restype = C.c_int
    lib.tvl1_postprocess_affine.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                            C.c_void_p, C.c_size_t, C.c_int32, C.c_int32,
                                            C.c_int32, C.POINTER(C.c_float), C.c_void_p]
    lib.tvl1_postprocess_affine.restype = C.c_int
    lib.tvl1_calc_host.argtypes = [C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t,
                                   C.POINTER(C.c_uint8), C.c_size_t, C.c_int32, C.c_int32,
                                   C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_size_t,
                                   C.POINTER(TVL1Stats)]
    lib.tvl1_calc_host.restype = C.c_int
    lib.tvl1_postprocess.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                     C.c_void_p, C.c_size_t, C.c_int32, C.c_int32, C.c_int32,
                                     C.c_void_p]
    lib.tvl1_postprocess.restype = C.c_int
    lib.tvl1_postprocess_batch.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                                           C.c_size_t, C.c_size_t, C.c_void_p, C.c_size_t,
                                           C.c_size_t, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]
    lib.tvl1_postprocess_batch.restype = C.c_int
    lib.tvl1_gather_flow.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p,
                                     C.c_int32,
                                     C.c_void_p, C.c_void_p, C.c_void_p]
    lib.tvl1_gather_flow.restype = C.c_int
    lib.tvl1_stream.argtypes = [C.c_void_p]
    lib.tvl1_stream.restype = C.c_void_p
    lib.tvl1_set_profiling.argtypes = [C.c_void_p, C.c_int32]
    lib.tvl1_set_profiling.restype = C.c_int
    lib.tvl1_destroy.argtypes = [C.c_void_p]
    lib.tvl1_destroy.restype = None
    lib.tvl1_last_error.argtypes = [C.c_void_p]
    lib.tvl1_last_error.restype = C.c_char_p
    lib.tvl1_abi_version.restype = C.c_int32
    lib.tvl1_device_count.restype = C.c_int32
    if lib.tvl1_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{path}: ABI version {lib.tvl1_abi_version()}, binding expects {ABI_VERSION}")
    return lib


class TVL1Error(RuntimeError):
    pass


def align_params(lib, **kw) -> TVL1AlignParams:
    """tvl1_align_params_default (orb_defaults, features.cpp:19-31) with overrides."""
    ap = TVL1AlignParams()
    lib.tvl1_align_params_default(C.byref(ap))
    for k, v in kw.items():
        setattr(ap, k, v)
    return ap


class Engine:
    """Host-side handle on the HIP engine (one ctx per device)."""

    def __init__(self, params: TVL1Params | None = None, device: int = 0):
        self.lib = load_engine()
        self.params = params or make_params()
        self.ctx = C.c_void_p()
        rc = self.lib.tvl1_create(C.byref(self.ctx), int(device), C.byref(self.params))
        if rc != 0:
            raise TVL1Error(f"tvl1_create: {STATUS.get(rc, rc)}: "
                            f"{self.lib.tvl1_last_error(None).decode()}")

    def set_params(self, params: TVL1Params):
        self.params = params
        self._check(self.lib.tvl1_set_params(self.ctx, C.byref(params)), "tvl1_set_params")

    @property
    def stream(self) -> int:
        """The ctx's own non-blocking hipStream_t (as an int handle)."""
        return int(self.lib.tvl1_stream(self.ctx) or 0)

    def set_profiling(self, on: bool):
        self._check(self.lib.tvl1_set_profiling(self.ctx, 1 if on else 0), "tvl1_set_profiling")

    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.tvl1_last_error(self.ctx)
            raise TVL1Error(f"{what}: {STATUS.get(rc, rc)}: {msg.decode() if msg else ''}")

    def calc_host(self, I0: np.ndarray, I1: np.ndarray, warp_iters: bool = True):
        I0 = np.ascontiguousarray(I0, dtype=np.uint8)
        I1 = np.ascontiguousarray(I1, dtype=np.uint8)
        h, w = I0.shape
        if I1.shape != I0.shape:
            raise ValueError("I0 and I1 must have the same size")
        u = np.zeros((h, w), np.float32)
        v = np.zeros((h, w), np.float32)
        st = TVL1Stats()
        wi = None
        if warp_iters:
            cap = TVL1_MAX_LEVELS * max(1, self.params.warps)
            wi = np.full(cap, -1, np.int32)
            st.warp_iterations = wi.ctypes.data_as(C.POINTER(C.c_int32))
            st.warp_iterations_capacity = cap
        rc = self.lib.tvl1_calc_host(self.ctx, _u8_ptr(I0), w, _u8_ptr(I1), w, w, h,
                                     _f32_ptr(u), _f32_ptr(v), 4 * w, C.byref(st))
        self._check(rc, "tvl1_calc_host")
        sd = stats_dict(st)
        if wi is not None:
            wi = wi[: sd["levels"] * self.params.warps].reshape(sd["levels"], self.params.warps)
        return u, v, sd, wi

    def calc_device(self, dI0: int, pitch0: int, dI1: int, pitch1: int, w: int, h: int,
                    du: int, dv: int, flow_pitch: int, stream: int = 0, stats: bool = True,
                    warp_iters: bool = False, f32: bool = False):
        """tvl1_calc on device buffers (u8 frames, pitches in bytes), or tvl1_calc_f32 with
        f32=True (float frames in [0, 1], pitches in bytes)."""
        st = TVL1Stats() if stats or warp_iters else None
        wi = None
        if warp_iters:
            cap = TVL1_MAX_LEVELS * max(1, self.params.warps)
            wi = np.full(cap, -1, np.int32)
            st.warp_iterations = wi.ctypes.data_as(C.POINTER(C.c_int32))
            st.warp_iterations_capacity = cap
        fn = self.lib.tvl1_calc_f32 if f32 else self.lib.tvl1_calc
        rc = fn(self.ctx, C.c_void_p(dI0), pitch0, C.c_void_p(dI1), pitch1,
                w, h, C.c_void_p(du), C.c_void_p(dv), flow_pitch,
                C.byref(st) if st is not None else None,
                C.c_void_p(stream) if stream else None)
        self._check(rc, "tvl1_calc_f32" if f32 else "tvl1_calc")
        if st is None:
            return None
        sd = stats_dict(st)
        if wi is not None:
            sd["warp_iters"] = wi[: sd["levels"] * self.params.warps].reshape(sd["levels"],
                                                                              self.params.warps)
        return sd

    def calc_batch_device(self, n: int, dI0: int, pitch0: int, stride0: int, dI1: int,
                          pitch1: int, stride1: int, w: int, h: int, du: int, dv: int,
                          flow_pitch: int, flow_stride: int, stream: int = 0,
                          warp_iters: bool = False):
        """tvl1_calc_batch on device buffers: n pairs of one size, pair b at base + b*stride
        (bytes).  Returns one stats dict per pair (+ per-warp iterations if asked)."""
        sts = (TVL1Stats * n)()
        wis = []
        if warp_iters:
            cap = TVL1_MAX_LEVELS * max(1, self.params.warps)
            for b in range(n):
                wi = np.full(cap, -1, np.int32)
                sts[b].warp_iterations = wi.ctypes.data_as(C.POINTER(C.c_int32))
                sts[b].warp_iterations_capacity = cap
                wis.append(wi)
        rc = self.lib.tvl1_calc_batch(self.ctx, n, C.c_void_p(dI0), pitch0, stride0,
                                      C.c_void_p(dI1), pitch1, stride1, w, h, C.c_void_p(du),
                                      C.c_void_p(dv), flow_pitch, flow_stride, sts,
                                      C.c_void_p(stream) if stream else None)
        self._check(rc, "tvl1_calc_batch")
        out = [stats_dict(sts[b]) for b in range(n)]
        if warp_iters:
            for b in range(n):
                L = out[b]["levels"]
                out[b]["warp_iters"] = wis[b][: L * self.params.warps].reshape(L, self.params.warps)
        return out

    def find_alignment(self, d1: int, pitch1: int, w1: int, h1: int, d0: int, pitch0: int,
                       w0: int, h0: int, **kw):
        """tvl1_find_alignment(frame1, frame0) on device frames -> (affine (2, 3), n_good,
        outcome)."""
        ap = align_params(self.lib, **kw)
        aff = (C.c_float * 6)()
        ng, oc = C.c_int32(0), C.c_int32(0)
        rc = self.lib.tvl1_find_alignment(self.ctx, C.c_void_p(d1), pitch1, w1, h1, C.c_void_p(d0),
                                          pitch0, w0, h0, C.byref(ap), aff, C.byref(ng),
                                          C.byref(oc), None)
        self._check(rc, "tvl1_find_alignment")
        return np.array(list(aff), np.float32).reshape(2, 3), int(ng.value), int(oc.value)

    def orb_detect(self, d: int, pitch: int, w: int, h: int, cap: int = 10000, **kw):
        """tvl1_orb_detect on a device frame -> (kp (n, 5): x, y, octave, angle, response;
        desc (n, 32) u8)."""
        ap = align_params(self.lib, **kw)
        kp = np.zeros((cap, 5), np.float32)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int32(0)
        self._check(self.lib.tvl1_orb_detect(self.ctx, C.c_void_p(d), pitch, w, h, C.byref(ap),
                                             kp.ctypes.data, desc.ctypes.data, cap, C.byref(n),
                                             None), "tvl1_orb_detect")
        m = min(n.value, cap)
        return kp[:m], desc[:m]

    def match_knn2(self, query: np.ndarray, train: np.ndarray):
        """tvl1_match_knn2 on host descriptor arrays (n, 32) u8 -> (idx (nq, 2), dist (nq, 2))."""
        q = np.ascontiguousarray(query, np.uint8)
        t = np.ascontiguousarray(train, np.uint8)
        idx = np.zeros((len(q), 2), np.int32)
        dist = np.zeros((len(q), 2), np.int32)
        self._check(self.lib.tvl1_match_knn2(self.ctx, q.ctypes.data, len(q), t.ctypes.data,
                                             len(t), idx.ctypes.data, dist.ctypes.data, None),
                    "tvl1_match_knn2")
        return idx, dist

    def warp_affine_u8(self, src: int, sp: int, sw: int, sh: int, dst: int, dp: int, dw: int,
                       dh: int, affine) -> None:
        a = (C.c_float * 6)(*[float(x) for x in np.asarray(affine, np.float32).ravel()])
        self._check(self.lib.tvl1_warp_affine_u8(self.ctx, C.c_void_p(src), sp, sw, sh,
                                                 C.c_void_p(dst), dp, dw, dh, a, None),
                    "tvl1_warp_affine_u8")

    def postprocess_batch(self, n: int, du: int, dv: int, fpitch: int, fstride: int, dI1: int,
                          pitch1: int, stride1: int, w: int, h: int, mode: int, stream: int = 0):
        """tvl1_postprocess_batch: solve_wrapper's map grid + I1 <= 1 mask on n pairs."""
        self._check(self.lib.tvl1_postprocess_batch(self.ctx, n, du, dv, fpitch, fstride, dI1,
                                                    pitch1, stride1, w, h, mode, stream),
                    "tvl1_postprocess_batch")

    def gather_flow(self, du: int, dv: int, plane_elems: int, offsets, stream: int = 0):
        """tvl1_gather_flow: (u[off], v[off]) for element offsets in [0, plane_elems) into
        device planes (any other offset raises, TVL1_EINVAL)."""
        off = np.ascontiguousarray(offsets, np.int64)
        ou = np.zeros(len(off), np.float32)
        ov = np.zeros(len(off), np.float32)
        self._check(self.lib.tvl1_gather_flow(self.ctx, du, dv, plane_elems, off.ctypes.data,
                                              len(off),
                                              ou.ctypes.data, ov.ctypes.data, stream),
                    "tvl1_gather_flow")
        return ou, ov

    def close(self):
        if self.ctx:
            self.lib.tvl1_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def epe(u, v, u_ref, v_ref) -> np.ndarray:
    """Per-pixel end-point error."""
    return np.sqrt((u.astype(np.float64) - u_ref) ** 2 + (v.astype(np.float64) - v_ref) ** 2)


def find_homography(src: np.ndarray, dst: np.ndarray, method: int = 8, thresh: float = 5.0):
    """tvl1_find_homography (cv::findHomography restated, host only): src, dst (n, 2) point
    arrays; returns (H 3x3, inlier mask) or raises TVL1Error."""
    lib = load_engine()
    a = np.ascontiguousarray(src, dtype=np.float32)
    b = np.ascontiguousarray(dst, dtype=np.float32)
    n = a.shape[0]
    H = (C.c_double * 9)()
    mask = np.zeros(n, np.uint8)
    rc = lib.tvl1_find_homography(a.ctypes.data, b.ctypes.data, n, method, thresh, H,
                                  mask.ctypes.data)
    if rc != 0:
        raise TVL1Error(f"tvl1_find_homography: {STATUS.get(rc, rc)}: "
                        f"{lib.tvl1_last_error(None).decode()}")
    return np.array(H[:], dtype=np.float64).reshape(3, 3), mask.astype(bool)
