"""TEST INFRASTRUCTURE: ctypes access to the oracle (liboracle_tvl1.so, built by
oracle/Makefile).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg call
this; it lives here, outside the product package, so a Python caller of optflow_amd cannot
reach the oracle (VERDICT r1 "test infrastructure lives in the product module")."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from optflow_amd.capi import (STATUS, TVL1_MAX_LEVELS, TVL1Error, TVL1Params, TVL1Stats,
                              _f32_ptr, _u8_ptr, make_params, stats_dict)

ORACLE_SO = Path(__file__).resolve().parent / "liboracle_tvl1.so"


def load_oracle(so: str | Path | None = None) -> C.CDLL:
    """The CPU restatement (oracle/tvl1_oracle.c) behind the engine's host-call shape;
    `so`: another build of the same sources (bench.py's host-tuned cpu_baseline build)."""
    path = Path(so) if so else ORACLE_SO
    if not path.exists():
        raise FileNotFoundError(f"{path} not built (run __graft_entry__.build())")
    lib = C.CDLL(str(path))
    lib.orc_tvl1_calc.restype = C.c_int
    lib.orc_tvl1_calc.argtypes = [C.POINTER(TVL1Params), C.POINTER(C.c_uint8), C.c_size_t,
                                  C.POINTER(C.c_uint8), C.c_size_t, C.c_int, C.c_int,
                                  C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_size_t,
                                  C.POINTER(TVL1Stats)]
    lib.orc_tvl1_calc_f32.restype = C.c_int
    lib.orc_tvl1_calc_f32.argtypes = [C.POINTER(TVL1Params), C.POINTER(C.c_float), C.c_size_t,
                                      C.POINTER(C.c_float), C.c_size_t, C.c_int, C.c_int,
                                      C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_size_t,
                                      C.POINTER(TVL1Stats)]
    lib.orc_num_threads.restype = C.c_int
    lib.orc_set_num_threads.argtypes = [C.c_int]
    return lib


def oracle_calc(I0: np.ndarray, I1: np.ndarray, params: TVL1Params | None = None,
                warp_iters: bool = True, threads: int | None = None,
                so: str | Path | None = None):
    """Run the CPU restatement on host u8 images (or float32 images: tvl1_calc_f32's
    contract, values scaled by 255); returns (u, v, stats, warp_iters)."""
    lib = load_oracle(so)
    if threads:
        lib.orc_set_num_threads(int(threads))
    params = params or make_params()
    f32 = np.asarray(I0).dtype == np.float32
    dt = np.float32 if f32 else np.uint8
    I0 = np.ascontiguousarray(I0, dtype=dt)
    I1 = np.ascontiguousarray(I1, dtype=dt)
    h, w = I0.shape
    u = np.zeros((h, w), np.float32)
    v = np.zeros((h, w), np.float32)
    st = TVL1Stats()
    wi = None
    if warp_iters:
        cap = TVL1_MAX_LEVELS * max(1, params.warps)
        wi = np.full(cap, -1, np.int32)
        st.warp_iterations = wi.ctypes.data_as(C.POINTER(C.c_int32))
        st.warp_iterations_capacity = cap
    if f32:
        rc = lib.orc_tvl1_calc_f32(C.byref(params), _f32_ptr(I0), 4 * w, _f32_ptr(I1), 4 * w, w,
                                   h, _f32_ptr(u), _f32_ptr(v), 4 * w, C.byref(st))
    else:
        rc = lib.orc_tvl1_calc(C.byref(params), _u8_ptr(I0), w, _u8_ptr(I1), w, w, h,
                               _f32_ptr(u), _f32_ptr(v), 4 * w, C.byref(st))
    if rc != 0:
        raise TVL1Error(f"oracle: {STATUS.get(rc, rc)}")
    sd = stats_dict(st)
    if wi is not None:
        wi = wi[: sd["levels"] * params.warps].reshape(sd["levels"], params.warps)
    return u, v, sd, wi


# ---- feature pre-alignment restatement (oracle/tvl1_oracle_align.c)
def _align_params(**kw):
    from optflow_amd import capi
    return capi.align_params(capi.load_engine(), **kw)   # tvl1_align_params_default + kw


def oracle_orb_detect(img: np.ndarray, cap: int = 10000, **kw):
    """orc_orb_detect on a host u8 frame -> (kp (n, 5), desc (n, 32))."""
    lib = load_oracle()
    a = np.ascontiguousarray(img, np.uint8)
    h, w = a.shape
    kp = np.zeros((cap, 5), np.float32)
    desc = np.zeros((cap, 32), np.uint8)
    ap = _align_params(**kw)
    lib.orc_orb_detect.restype = C.c_int
    n = lib.orc_orb_detect(a.ctypes.data_as(C.c_void_p), C.c_size_t(w), w, h, C.byref(ap),
                           kp.ctypes.data_as(C.c_void_p), desc.ctypes.data_as(C.c_void_p), cap)
    if n < 0:
        raise TVL1Error("oracle: orb_detect out of memory")
    m = min(n, cap)
    return kp[:m], desc[:m]


def oracle_match_knn2(query: np.ndarray, train: np.ndarray):
    lib = load_oracle()
    q = np.ascontiguousarray(query, np.uint8)
    t = np.ascontiguousarray(train, np.uint8)
    idx = np.zeros((len(q), 2), np.int32)
    dist = np.zeros((len(q), 2), np.int32)
    lib.orc_match_knn2(q.ctypes.data_as(C.c_void_p), len(q), t.ctypes.data_as(C.c_void_p), len(t),
                       idx.ctypes.data_as(C.c_void_p), dist.ctypes.data_as(C.c_void_p))
    return idx, dist


def oracle_find_homography(src: np.ndarray, dst: np.ndarray, method: int = 8,
                           thresh: float = 5.0):
    lib = load_oracle()
    a = np.ascontiguousarray(src, np.float64)
    b = np.ascontiguousarray(dst, np.float64)
    H = np.zeros(9, np.float64)
    mask = np.zeros(len(a), np.uint8)
    lib.orc_find_homography.restype = C.c_int
    ok = lib.orc_find_homography(a.ctypes.data_as(C.c_void_p), b.ctypes.data_as(C.c_void_p),
                                 len(a), method, C.c_double(thresh), H.ctypes.data_as(C.c_void_p),
                                 mask.ctypes.data_as(C.c_void_p))
    return bool(ok), H.reshape(3, 3), mask.astype(bool)


def oracle_find_alignment(frame1: np.ndarray, frame0: np.ndarray, **kw):
    """orc_find_alignment(frame1, frame0) -> (affine (2, 3) f32, n_good, outcome)."""
    lib = load_oracle()
    f1 = np.ascontiguousarray(frame1, np.uint8)
    f0 = np.ascontiguousarray(frame0, np.uint8)
    ap = _align_params(**kw)
    aff = np.zeros(6, np.float32)
    ng, oc = C.c_int(0), C.c_int(0)
    rc = lib.orc_find_alignment(f1.ctypes.data_as(C.c_void_p), C.c_size_t(f1.shape[1]),
                                f1.shape[1], f1.shape[0], f0.ctypes.data_as(C.c_void_p),
                                C.c_size_t(f0.shape[1]), f0.shape[1], f0.shape[0], C.byref(ap),
                                aff.ctypes.data_as(C.c_void_p), C.byref(ng), C.byref(oc))
    if rc != 0:
        raise TVL1Error("oracle: find_alignment out of memory")
    return aff.reshape(2, 3), int(ng.value), int(oc.value)


def oracle_warp_affine_u8(src: np.ndarray, dw: int, dh: int, M) -> np.ndarray:
    lib = load_oracle()
    s = np.ascontiguousarray(src, np.uint8)
    d = np.zeros((dh, dw), np.uint8)
    m = np.ascontiguousarray(np.asarray(M, np.float32).ravel())
    lib.orc_warp_affine_u8(s.ctypes.data_as(C.c_void_p), C.c_size_t(s.shape[1]), s.shape[1],
                           s.shape[0], d.ctypes.data_as(C.c_void_p), C.c_size_t(dw), dw, dh,
                           m.ctypes.data_as(C.c_void_p))
    return d


def oracle_postprocess_affine(u: np.ndarray, v: np.ndarray, I1: np.ndarray, flow_output: int, M):
    lib = load_oracle()
    uu = np.array(u, np.float32, copy=True, order="C")
    vv = np.array(v, np.float32, copy=True, order="C")
    i1 = np.ascontiguousarray(I1, np.uint8)
    H, W = uu.shape
    m = np.ascontiguousarray(np.asarray(M, np.float32).ravel())
    lib.orc_postprocess_affine(uu.ctypes.data_as(C.c_void_p), vv.ctypes.data_as(C.c_void_p),
                               C.c_size_t(4 * W), i1.ctypes.data_as(C.c_void_p), C.c_size_t(W), W,
                               H, int(flow_output), m.ctypes.data_as(C.c_void_p))
    return uu, vv


# ---- stopping-rule robustness: the oracle's per-check
# error / scaledEps trace and an alternative residual accumulation order
def oracle_check_trace(I0: np.ndarray, I1: np.ndarray, params: TVL1Params | None = None,
                       residual_mode: int = 0, cap: int = 1 << 16):
    """oracle_calc with every check recorded: returns (u, v, stats, warp_iters, trace) where
    trace is an (n, 4) array of (level, warp, n, error / scaledEps).  residual_mode 1 sums the
    residual in float, rows reversed (orc_set_residual_mode)."""
    lib = load_oracle()
    buf = np.zeros((cap, 4), np.float64)
    lib.orc_set_residual_mode(int(residual_mode))
    lib.orc_set_check_trace(buf.ctypes.data_as(C.c_void_p), cap)
    try:
        u, v, st, wi = oracle_calc(I0, I1, params)
        n = int(lib.orc_check_trace_count())
    finally:
        lib.orc_set_check_trace(None, 0)
        lib.orc_set_residual_mode(0)
    if n > cap:
        raise RuntimeError(f"check trace overflow ({n} > {cap})")
    return u, v, st, wi, buf[:n].copy()


def check_margins(trace: np.ndarray, iterations: int) -> np.ndarray:
    """Relative distance of each check's decision from the nearest threshold that could flip
    the schedule.  After a check at iteration n with r = error / scaledEps the warp stops iff
    r <= 1; otherwise prevError -= scaledEps per unchecked iteration, so the next check comes
    at n + 2 iff r < 2, else at n + 4 iff r < 4, at n + 6 iff r < 6, ... (procOneScale's
    rule).  The thresholds are therefore t in {1, 2, 4, 6, ...} (those reachable
    before `iterations`), and a perturbation of the residual by a relative delta flips a
    decision only if delta >= |r - t| / r for some t.  Returns that relative margin per check."""
    out = np.empty(len(trace))
    for i, (_, _, n, r) in enumerate(trace):
        ts = [1.0] + [float(t) for t in range(2, max(2, iterations - int(n)) + 1, 2)]
        out[i] = min(abs(r - t) for t in ts) / r
    return out
