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
