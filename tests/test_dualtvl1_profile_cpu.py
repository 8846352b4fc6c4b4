"""Profile 1: OpenCV's CPU cv::DualTVL1OpticalFlow schedule,
restated in oracle/tvl1_oracle_dualtvl1.c.  PARITY UNPINNED (OpenCV absent; the recalled
details are listed in that file's header): these known-answer tests pin the restatement.
"""
import ctypes as C

import numpy as np
import pytest

from optflow_amd import capi, synth
from oracle import checker

F32P = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")


@pytest.fixture(scope="module")
def oracle(built):
    lib = checker.load_oracle()
    lib.orc_resize_hp.restype = None
    lib.orc_resize_hp.argtypes = [F32P, C.c_int, C.c_int, F32P, C.c_int, C.c_int, C.c_double,
                                  C.c_double, C.c_int]
    lib.orc_remap_cubic.restype = None
    lib.orc_remap_cubic.argtypes = [F32P] * 6 + [C.c_int, C.c_int] + [F32P] * 4
    return lib


def resize(lib, src, dw, dh, area_fast=0):
    sh, sw = src.shape
    dst = np.zeros((dh, dw), np.float32)
    lib.orc_resize_hp(np.ascontiguousarray(src, np.float32), sw, sh, dst, dw, dh,
                      1.0 / (dw / sw), 1.0 / (dh / sh), area_fast)
    return dst


def test_resize_hp_constant_and_identity(oracle):
    c = np.full((40, 50), 7.25, np.float32)
    assert np.all(resize(oracle, c, 40, 32) == 7.25)     # downscale keeps a constant
    assert np.all(resize(oracle, c, 62, 50) == 7.25)     # upscale too
    r = np.random.default_rng(1).random((13, 17)).astype(np.float32)
    assert np.array_equal(resize(oracle, r, 17, 13), r)  # same size -> copy


def test_resize_hp_half_pixel_centres(oracle):
    # a horizontal ramp x: half-pixel sampling maps dst column d to (d + .5) * s - .5
    sw, dw = 50, 40
    ramp = np.tile(np.arange(sw, dtype=np.float32), (8, 1))
    out = resize(oracle, ramp, dw, 8)
    s = sw / dw
    want = np.clip((np.arange(dw) + 0.5) * s - 0.5, 0, sw - 1)
    np.testing.assert_allclose(out[3], want, atol=1e-5)


def test_resize_hp_area_fast(oracle):
    r = np.random.default_rng(2).random((16, 20)).astype(np.float32)
    out = resize(oracle, r, 10, 8, area_fast=1)
    want = (r[0::2, 0::2] + r[0::2, 1::2] + r[1::2, 0::2] + r[1::2, 1::2]) * np.float32(0.25)
    np.testing.assert_allclose(out, want, rtol=1e-6)


def test_remap_zero_flow_is_identity(oracle):
    """interpolateCubic(0) = (0, 1, 0, 0): a zero map samples I1 and its gradients exactly."""
    h, w = 24, 31
    rng = np.random.default_rng(3)
    I0 = rng.random((h, w)).astype(np.float32) * 200
    I1 = rng.random((h, w)).astype(np.float32) * 200
    I1x, I1y = np.gradient(I1, axis=1).astype(np.float32), np.gradient(I1, axis=0).astype(np.float32)
    z = np.zeros((h, w), np.float32)
    outs = [np.zeros((h, w), np.float32) for _ in range(4)]
    oracle.orc_remap_cubic(I0, I1, I1x, I1y, z, z, w, h, *outs)
    wx, wy, grad, rho = outs
    assert np.array_equal(wx, I1x) and np.array_equal(wy, I1y)
    assert np.array_equal(rho, I1 - I0)


def test_remap_outside_is_zero(oracle):
    """BORDER_CONSTANT 0: a map far outside the image samples nothing."""
    h, w = 20, 20
    I = np.full((h, w), 50, np.float32)
    u1 = np.full((h, w), 100, np.float32)
    outs = [np.zeros((h, w), np.float32) for _ in range(4)]
    oracle.orc_remap_cubic(I, I, I, I, u1, u1, w, h, *outs)
    assert np.all(outs[0] == 0) and np.all(outs[1] == 0)
    assert np.all(outs[3] == -50)    # rho_c = 0 - 0 - 0 - I0


def test_identity_pair_one_iteration_per_warp(built):
    I0, _ = synth.gen_pair(96, 80, seed=5)
    p = capi.make_params(profile=1, nscales=4, warps=3)
    u, v, st, wi = checker.oracle_calc(I0, I0, p)
    assert np.all(u == 0) and np.all(v == 0)
    assert np.all(wi == 1)          # the residual is checked at every inner iteration
    assert st["iterations_total"] == st["checks_total"]


def test_translation_recovered(built):
    from scipy import ndimage
    base = synth.base_texture(192, 160, seed=31)
    ys, xs = np.mgrid[0:160, 0:192].astype(np.float32)
    A = np.clip(np.rint(base), 0, 255).astype(np.uint8)
    B = np.clip(np.rint(ndimage.map_coordinates(base, [ys + 0.4, xs - 0.7], order=3,
                                                mode="nearest")), 0, 255).astype(np.uint8)
    # cv::DualTVL1OpticalFlow defaults: lambda 0.15, nscales 5, warps 5, median 5
    p = capi.make_params(profile=1, nscales=5, warps=5, lambda_=0.15, median_filtering=5)
    u, v, st, wi = checker.oracle_calc(A, B, p)
    c = (slice(20, -20), slice(20, -20))
    assert abs(float(np.median(u[c])) - 0.7) < 0.05
    assert abs(float(np.median(v[c])) + 0.4) < 0.05


def test_schedule_bounds(built):
    """epsilon 0: every warp runs exactly outer x inner iterations."""
    I0, I1 = synth.gen_pair(64, 48, seed=7)
    p = capi.make_params(profile=1, nscales=2, warps=2, epsilon=0.0, inner_iterations=3,
                         outer_iterations=2)
    _, _, st, wi = checker.oracle_calc(I0, I1, p)
    assert np.all(wi == 6)


def test_bad_profile_rejected(built):
    I0, I1 = synth.gen_pair(32, 32, seed=1)
    with pytest.raises(Exception):
        checker.oracle_calc(I0, I1, capi.make_params(profile=3))
