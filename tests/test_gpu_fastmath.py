"""Arithmetic modes vs the IEEE oracle: the per-pixel tolerance parity is held to.

The reference's OpenCV was built by nvcc with CUDA_FAST_MATH (singularity/optflow.def:33-34;
SURVEY A.7): a*b + c contracted to fma (nvcc's default -fmad=true) and approximate division
and sqrt.  No OpenCV exists here to compare against (parity unpinned), so the
distance between the candidate arithmetics is measured instead and bounded:

  IEEE  fast_math = 0  the oracle / engine default (bit-identical to each other)
  fma   fast_math = 2  contraction only (bit-identical to oracle/'s fma mode,
                       tests/test_gpu_parity.py::test_fma_mode_bit_identical)
  fast  fast_math = 1  contraction + v_rcp_f32 / v_sqrt_f32 (CUDA_FAST_MATH restated)

Every mode must keep the oracle's per-warp iteration schedule (a changed iteration would
move u by ~epsilon = 0.01 px RMS), and the per-pixel end-point error against the IEEE result
must stay within TOL: mean, 99.9th percentile and maximum.  The maximum is a handful of px
where the TH operator's branch (rho against +-lambda*theta*|grad I|) flips under 1-ulp
differences; DESIGN.md 2 tabulates the same figures for the C2 pair (bench.py "math_modes").
"""
import numpy as np
import pytest

from optflow_amd import capi, synth
from oracle import checker

pytestmark = pytest.mark.gpu

# per-pixel EPE budget against the IEEE result (px): mean (BASELINE.json north_star), 99.9th
# percentile, max
TOL = {1: (1e-3, 2e-2, 0.5), 2: (1e-3, 2e-2, 0.5)}
NAME = {1: "fast", 2: "fma"}

KNOBS = ("TVL1_ROLL_SEG", "TVL1_ROLL_PX4_MIN", "TVL1_ROLL_LONG_MIN", "TVL1_FUSE", "TVL1_FUSE_MIN",
         "TVL1_BUF_LIMIT")


def _solve(monkeypatch, env, W, H, seed, kw, math):
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for kv in filter(None, env.split(",")):
        monkeypatch.setenv(*kv.split("="))
    I0, I1 = synth.gen_pair(W, H, seed=seed)
    eng = capi.Engine(capi.make_params(fast_math=math, **kw))
    u, v, st, wi = eng.calc_host(I0, I1)
    eng.close()
    ur, vr, sr, wr = checker.oracle_calc(I0, I1, capi.make_params(**kw))
    return u, v, st, wi, ur, vr, sr, wr


def check_budget(e, math, what):
    mean, p999, mx = float(e.mean()), float(np.quantile(e, 0.999)), float(e.max())
    print(f"{NAME[math]} vs IEEE {what}: mean {mean:.3g} p99.9 {p999:.3g} max {mx:.3g} px")
    tm, tq, tx = TOL[math]
    assert np.isfinite(e).all()
    assert mean <= tm, f"mean EPE {mean}"
    assert p999 <= tq, f"p99.9 EPE {p999}"
    assert mx <= tx, f"max EPE {mx}"


CASES = [
    (64, 48, 1, dict(nscales=5, warps=3)),
    (17, 16, 2, dict(nscales=3, warps=2)),
    (250, 131, 5, dict(nscales=5, warps=5)),
    (512, 512, 6, dict(nscales=5, warps=30)),
    (300, 77, 7, dict(epsilon=0.0, iterations=7, nscales=3, warps=2)),
    (96, 64, 9, dict(median_filtering=5, nscales=4, warps=3)),
]
# every kernel of the contracting modes: the default dispatch, the fused warp + first pass,
# 4 px / lane 2-iteration passes, streaming long passes, the 64-bit-addressed fallbacks
ENVS = ["", "TVL1_FUSE_MIN=0,TVL1_ROLL_PX4_MIN=0", "TVL1_ROLL_LONG_MIN=0", "TVL1_BUF_LIMIT=0"]


@pytest.mark.parametrize("math", [1, 2])
@pytest.mark.parametrize("env", ENVS)
@pytest.mark.parametrize("W,H,seed,kw", CASES)
def test_mode_within_tolerance(built, monkeypatch, env, W, H, seed, kw, math):
    u, v, st, wi, ur, vr, sr, wr = _solve(monkeypatch, env, W, H, seed, kw, math)
    assert st["levels"] == sr["levels"]
    np.testing.assert_array_equal(wi, wr)
    check_budget(capi.epe(u, v, ur, vr), math, f"{W}x{H}")


@pytest.mark.parametrize("math", [1, 2])
def test_mode_benchmark_shape(built, monkeypatch, math):
    """A 1536x1024 pair at the benchmark parameters (5 scales, 30 warps)."""
    u, v, st, wi, ur, vr, sr, wr = _solve(monkeypatch, "", 1536, 1024, 0x5EED,
                                          dict(nscales=5, warps=30), math)
    np.testing.assert_array_equal(wi, wr)
    check_budget(capi.epe(u, v, ur, vr), math, "1536x1024")


def test_fast_vs_fma_distance(built):
    """fast (approximate division / sqrt) against fma (the same contraction, IEEE division):
    the share of the distance the approximations alone add."""
    I0, I1 = synth.gen_pair(512, 384, seed=17)
    kw = dict(nscales=5, warps=10)
    out = {}
    for m in (1, 2):
        eng = capi.Engine(capi.make_params(fast_math=m, **kw))
        out[m] = eng.calc_host(I0, I1)
        eng.close()
    np.testing.assert_array_equal(out[1][3], out[2][3])
    check_budget(capi.epe(out[1][0], out[1][1], out[2][0], out[2][1]), 1, "(against fma)")


@pytest.mark.parametrize("math", [1, 2])
def test_mode_gamma_stays_ieee(built, math):
    """gamma != 0 solves run the IEEE kernels: bit-identical to the IEEE oracle."""
    I0, I1 = synth.gen_pair(97, 80, seed=12)
    kw = dict(nscales=4, warps=3, gamma=0.2)
    eng = capi.Engine(capi.make_params(fast_math=math, **kw))
    u, v, _, wi = eng.calc_host(I0, I1)
    eng.close()
    ur, vr, _, wr = checker.oracle_calc(I0, I1, capi.make_params(**kw))
    np.testing.assert_array_equal(wi, wr)
    assert np.array_equal(u.view(np.uint32), ur.view(np.uint32))
    assert np.array_equal(v.view(np.uint32), vr.view(np.uint32))
