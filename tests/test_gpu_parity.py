"""HIP engine vs the oracle (CPU restatement of OpenCV 3.4.1 CUDA TV-L1).

Bar: identical per-warp iteration counts (the data-dependent stopping rule of
procOneScale) and EPE <= 1e-3 px (north_star tolerance); in practice the two
evaluate the same IEEE float32 operations and agree bit for bit.
"""
import numpy as np
import pytest

from optflow_amd import capi, synth
from oracle import checker

torch = pytest.importorskip("torch")   # device buffers of the f32 test; imported before HIP init

pytestmark = pytest.mark.gpu

EPE_TOL = 1e-3  # px, BASELINE.json north_star


def bits_equal(a, b):
    """Bitwise equality of float arrays (distinguishes -0.0 from +0.0, NaN payloads)."""
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.fixture(scope="module")
def engine(built):
    return capi.Engine(capi.make_params())


CASES = [
    # (W, H, seed, params)
    (64, 48, 1, dict(nscales=5, warps=3)),
    (17, 16, 2, dict(nscales=3, warps=2)),
    (33, 19, 3, dict(nscales=4, warps=3)),
    (128, 96, 4, dict()),                        # reference defaults (nscales 10, warps 5)
    (250, 131, 5, dict(nscales=5, warps=5)),     # odd width, > one wave segment
    (512, 512, 6, dict(nscales=5, warps=30)),    # benchmark parameters, small frame
    (300, 77, 7, dict(epsilon=0.0, iterations=7, nscales=3, warps=2)),  # fixed-work mode
    (96, 64, 8, dict(gamma=0.2, nscales=4, warps=3)),                  # gamma != 0 (A.5)
    (96, 64, 9, dict(median_filtering=5, nscales=4, warps=3)),         # build-only median
    (96, 64, 10, dict(median_filtering=3, nscales=4, warps=3)),
]


@pytest.mark.parametrize("W,H,seed,kw", CASES)
def test_engine_matches_oracle(engine, W, H, seed, kw):
    I0, I1 = synth.gen_pair(W, H, seed=seed)
    p = capi.make_params(**kw)
    engine.set_params(p)
    u, v, st, wi = engine.calc_host(I0, I1)
    ur, vr, sr, wr = checker.oracle_calc(I0, I1, p)
    assert st["levels"] == sr["levels"]
    assert st["sizes"] == sr["sizes"]
    np.testing.assert_array_equal(wi, wr)
    e = capi.epe(u, v, ur, vr)
    assert float(e.max()) <= EPE_TOL, f"max EPE {e.max()}"
    # bit-exactness is expected (same IEEE ops, no FMA); report if it ever drifts
    assert bits_equal(u, ur) and bits_equal(v, vr), \
        f"not bit-exact: max|du|={np.abs(u-ur).max()} max|dv|={np.abs(v-vr).max()}"


@pytest.mark.parametrize("tau,theta", [(-0.05, 0.3), (0.25, -0.3)])
def test_negative_taut_takes_exact_division_path(engine, tau, theta):
    """tau/theta < 0 breaks ng >= 1, which the projection's shared-reciprocal division
    relies on: the engine must route such parameters to plain IEEE divisions."""
    I0, I1 = synth.gen_pair(70, 50, seed=11)
    p = capi.make_params(nscales=3, warps=2, iterations=12, tau=tau, theta=theta)
    engine.set_params(p)
    u, v, _, wi = engine.calc_host(I0, I1)
    ur, vr, _, wr = checker.oracle_calc(I0, I1, p)
    np.testing.assert_array_equal(wi, wr)
    fin = np.isfinite(ur) & np.isfinite(vr)
    assert np.array_equal(fin, np.isfinite(u) & np.isfinite(v))
    assert bits_equal(u[fin], ur[fin]) and bits_equal(v[fin], vr[fin])


@pytest.mark.parametrize("theta", [2.0 ** -22, 1e-7])
def test_large_taut_bit_exact(engine, theta):
    """tau/theta = 2^20, the largest |taut| for which the host lets the projection's sqrt skip
    its scaled form for x in (0, 2^-96) (IterArgs::taut_small), and 2.5e6, which keeps it:
    bit-exact either way (tools/sqrt_fma_check.hip proves ng unchanged up to 2^20)."""
    I0, I1 = synth.gen_pair(96, 64, seed=12)
    p = capi.make_params(nscales=3, warps=2, iterations=12, tau=0.25, theta=theta)
    engine.set_params(p)
    u, v, _, wi = engine.calc_host(I0, I1)
    ur, vr, _, wr = checker.oracle_calc(I0, I1, p)
    np.testing.assert_array_equal(wi, wr)
    fin = np.isfinite(ur) & np.isfinite(vr)
    assert np.array_equal(fin, np.isfinite(u) & np.isfinite(v))
    assert bits_equal(u[fin], ur[fin]) and bits_equal(v[fin], vr[fin])


def test_identity_pair_gives_zero_flow(engine):
    I0, _ = synth.gen_pair(80, 60, seed=3)
    engine.set_params(capi.make_params(nscales=4, warps=3))
    u, v, st, wi = engine.calc_host(I0, I0)
    assert np.all(u == 0) and np.all(v == 0)
    assert np.all(wi == 2)   # error 0 at the first check (n = 1)


def test_constant_images_give_zero_flow(engine):
    I0 = np.full((40, 70), 100, np.uint8)
    I1 = np.full((40, 70), 140, np.uint8)
    engine.set_params(capi.make_params(nscales=3, warps=2))
    u, v, _, _ = engine.calc_host(I0, I1)
    assert np.all(u == 0) and np.all(v == 0)


# Every shipped kernel instantiation must give the same bits.  The default dispatch
#  on these small levels reaches k_warp_ring<6,2>, k_iterate_roll<G,1|2,2> and
# k_iterate_tb<G,32,1,2>; the knobs (read at tvl1_create) reach the rest:
#   TVL1_ROLL_LONG_MIN=0  >= 3-iteration passes stream too: k_iterate_roll<G,3|4,2>
#   TVL1_ROLL_PX4_MIN=0   2-iteration passes at 4 px per lane: k_iterate_roll<G,1|2,4>
#   TVL1_FUSE_MIN=0       warpBackward fused with each warp's first pass: k_warp_iter<6,-,128,1,2>
#                         (two consumer wavefronts, one per iteration; TVL1_WI_NC=1: <..,1,1>,
#                         both iterations on one wavefront)
#   TVL1_FUSE=0           never fused (k_warp_ring + the pass, on every level)
#   TVL1_ROLL_SEG=8|64    streaming kernels' segment boundaries (8 = many short segments)
#   TVL1_BUF_LIMIT=N      planes >= N bytes take the 64-bit-addressed kernels: k_warp_img and
#                         the blocked passes for every pass (N = 0: every level)
#   TVL1_TB4=0            blocked passes (gamma = 0) in 64 x 32 regions, k_iterate_tb<false,32,1,2>
#                         (the default is k_iterate_tb4<FM>, 64 x 48; gamma != 0 always takes
#                         k_iterate_tb<true,...>)
# k_iterate<G, true> (tau/theta < 0) and the profile-1 kernels have their own tests below.
MID_ALL = "TVL1_ROLL_LONG_MIN=0,TVL1_SPEC=0,TVL1_MID=1,TVL1_MID_MIN=1"
MODES = ["", "TVL1_ROLL_LONG_MIN=0", "TVL1_ROLL_LONG_MIN=0,TVL1_ROLL_SEG=8", "TVL1_ROLL_SEG=8",
         "TVL1_ROLL_SEG=64", "TVL1_ROLL_PX4_MIN=0", "TVL1_ROLL_PX4_MIN=0,TVL1_ROLL_SEG=8",
         "TVL1_FUSE_MIN=0", "TVL1_FUSE_MIN=0,TVL1_ROLL_SEG=8", "TVL1_FUSE_MIN=0,TVL1_ROLL_PX4_MIN=0",
         "TVL1_FUSE=0,TVL1_ROLL_LONG_MIN=0", "TVL1_BUF_LIMIT=100000", "TVL1_BUF_LIMIT=0",
         "TVL1_POLL=0", "TVL1_POLL=0,TVL1_FUSE_MIN=0", "TVL1_SPEC=0", "TVL1_SPEC=0,TVL1_FUSE_MIN=0",
         "TVL1_FUSE_MIN=0,TVL1_WI_NC=1", "TVL1_FUSE_MIN=0,TVL1_WI_NC=1,TVL1_ROLL_SEG=8",
         "TVL1_TB4=0", "TVL1_TB4=0,TVL1_BUF_LIMIT=0",
         MID_ALL, MID_ALL + ",TVL1_ROLL_SEG=8", "TVL1_MID=0,TVL1_SPEC=0,TVL1_ROLL_LONG_MIN=0"]
# (TVL1_POLL=0: residuals read after an event instead of the poll; TVL1_SPEC=0: nothing
# enqueued behind a check before the host reads it; MID_ALL: every 2-iteration
# continuation after a warp's first check as a mid-check pass, k_iterate_roll_mid, whatever
# the error -- so some end on the mid state, DESIGN.md §4.1 of r6)
KNOBS = ("TVL1_ROLL_SEG", "TVL1_ROLL_PX4_MIN", "TVL1_ROLL_LONG_MIN", "TVL1_FUSE", "TVL1_FUSE_MIN",
         "TVL1_BUF_LIMIT", "TVL1_BATCH_FUSE", "TVL1_POLL", "TVL1_SPEC", "TVL1_WI_NC", "TVL1_TB4",
         "TVL1_MID", "TVL1_MID_MIN", "TVL1_SPEC_TRACE")
CONFIG_CASES = [
    (250, 131, 21, dict(nscales=5, warps=5)),
    (97, 201, 22, dict(nscales=4, warps=3, gamma=0.1)),
    (400, 300, 23, dict(nscales=3, warps=4, epsilon=0.0, iterations=9)),
    (300, 200, 24, dict(nscales=1, warps=2)),
]


def set_knobs(monkeypatch, env):
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for kv in filter(None, env.split(",")):
        monkeypatch.setenv(*kv.split("="))


@pytest.mark.parametrize("env", MODES)
@pytest.mark.parametrize("W,H,seed,kw", CONFIG_CASES)
def test_kernel_configs_bit_identical(built, monkeypatch, env, W, H, seed, kw):
    set_knobs(monkeypatch, env)
    p = capi.make_params(**kw)
    eng = capi.Engine(p)
    I0, I1 = synth.gen_pair(W, H, seed=seed)
    u, v, st, wi = eng.calc_host(I0, I1)
    eng.close()
    ur, vr, sr, wr = checker.oracle_calc(I0, I1, p)
    np.testing.assert_array_equal(wi, wr)
    assert bits_equal(u, ur) and bits_equal(v, vr)


# fma mode (tvl1_params.fast_math = 2): nvcc's -fmad=true contraction restated in both the
# engine and the oracle -- bit-identical too, on every shipped kernel instantiation
@pytest.mark.parametrize("env", MODES)
@pytest.mark.parametrize("W,H,seed,kw", [CONFIG_CASES[0], CONFIG_CASES[2],
                                         (128, 96, 25, dict(median_filtering=5, nscales=4))])
def test_fma_mode_bit_identical(built, monkeypatch, env, W, H, seed, kw):
    set_knobs(monkeypatch, env)
    p = capi.make_params(fast_math=2, **kw)
    eng = capi.Engine(p)
    I0, I1 = synth.gen_pair(W, H, seed=seed)
    u, v, st, wi = eng.calc_host(I0, I1)
    eng.close()
    ur, vr, sr, wr = checker.oracle_calc(I0, I1, p)
    np.testing.assert_array_equal(wi, wr)
    assert bits_equal(u, ur) and bits_equal(v, vr)
    ui, vi, _, _ = checker.oracle_calc(I0, I1, capi.make_params(**kw))
    assert not (bits_equal(u, ui) and bits_equal(v, vi)), "fma mode computed the IEEE result"


# Speculation: launches enqueued behind a residual check, gated on the device by
# that check's own evaluation of the stopping rule.  Same bits, iterations and checks as with
# nothing enqueued ahead; the guesses are mostly right.
@pytest.mark.parametrize("env", ["", "TVL1_FUSE_MIN=0", "TVL1_POLL=0,TVL1_FUSE_MIN=0",
                                 "TVL1_FUSE_MIN=0,TVL1_ROLL_LONG_MIN=0"])
@pytest.mark.parametrize("W,H,seed,kw", [(320, 240, 31, dict(nscales=4, warps=10)),
                                         (256, 200, 32, dict(nscales=3, warps=6, epsilon=0.002)),
                                         (200, 150, 33, dict(nscales=3, warps=4, gamma=0.2))])
def test_speculation_same_schedule(built, monkeypatch, env, W, H, seed, kw):
    p = capi.make_params(**kw)
    I0, I1 = synth.gen_pair(W, H, seed=seed)
    res = {}
    for spec in ("1", "0"):
        set_knobs(monkeypatch, env + ",TVL1_SPEC=" + spec)
        eng = capi.Engine(p)
        res[spec] = eng.calc_host(I0, I1)
        eng.close()
    (u, v, st, wi), (u0, v0, st0, wi0) = res["1"], res["0"]
    np.testing.assert_array_equal(wi, wi0)
    assert bits_equal(u, u0) and bits_equal(v, v0)
    assert st["checks_total"] == st0["checks_total"]
    assert st0["speculation_misses"] == 0
    print(f"checks {st['checks_total']} misses {st['speculation_misses']}")
    assert st["speculation_misses"] < st["checks_total"]
    ur, vr, _, wr = checker.oracle_calc(I0, I1, p)
    np.testing.assert_array_equal(wi, wr)
    assert bits_equal(u, ur) and bits_equal(v, vr)


GOLDEN = __import__("pathlib").Path(__file__).resolve().parent / "golden"


@pytest.mark.parametrize("path", sorted(GOLDEN.glob("*.npz")), ids=lambda p: p.stem)
def test_engine_reproduces_golden(engine, path):
    import json
    g = np.load(path, allow_pickle=False)
    p = capi.make_params(**json.loads(str(g["params"])))
    engine.set_params(p)
    u, v, st, wi = engine.calc_host(g["I0"], g["I1"])
    assert st["levels"] == int(g["levels"])
    np.testing.assert_array_equal(wi, g["warp_iters"])
    assert bits_equal(u, g["u"]) and bits_equal(v, g["v"])


@pytest.mark.parametrize("env", ["", "TVL1_FUSE_MIN=0", "TVL1_FUSE_MIN=0,TVL1_ROLL_SEG=8",
                                 "TVL1_BUF_LIMIT=0"])
@pytest.mark.parametrize("math", [0, 2])
def test_large_flow_uses_global_gather_fallback(built, monkeypatch, env, math):
    """A ~7 px shift puts taps outside the warp kernels' LDS windows (margin 6 px): the
    global-memory fallback must give the same bits (IEEE and fma mode)."""
    set_knobs(monkeypatch, env)
    engine = capi.Engine(capi.make_params())
    from scipy import ndimage
    base = synth.base_texture(192, 160, seed=31)
    ys, xs = np.mgrid[0:160, 0:192].astype(np.float32)
    I0 = np.clip(np.rint(base), 0, 255).astype(np.uint8)
    I1 = np.clip(np.rint(ndimage.map_coordinates(base, [ys + 6.75, xs - 7.5], order=3,
                                                 mode="nearest")), 0, 255).astype(np.uint8)
    p = capi.make_params(nscales=4, warps=6, fast_math=math)
    engine.set_params(p)
    u, v, st, wi = engine.calc_host(I0, I1)
    engine.close()
    ur, vr, sr, wr = checker.oracle_calc(I0, I1, p)
    assert float(np.abs(ur).max()) > 5.0   # the case really leaves the window
    np.testing.assert_array_equal(wi, wr)
    assert bits_equal(u, ur) and bits_equal(v, vr)


MID_RE = __import__("re").compile(r"mid-check passes (\d+), ended on the mid state (\d+)")


# The mid-check pass (k_iterate_roll_mid): two 2-iteration passes of a converging warp as one
# 4-iteration launch that keeps the state and residual after its first 2 iterations.  Cases
# whose schedules hold such runs (checks every second iteration at 1 < error / eps^2 W H < 2),
# with every continuation taken as a mid-check pass (MID_MIN=1: some end on the mid state)
# and at the default threshold: the same bits, per-warp counts and number of checks as without.
@pytest.mark.parametrize("mid_min", ["1", "1.1"])
@pytest.mark.parametrize("W,H,seed,kw", [(250, 131, 21, dict(nscales=5, warps=5)),
                                         (320, 240, 31, dict(nscales=4, warps=10)),
                                         (256, 200, 32, dict(nscales=3, warps=6, epsilon=0.002)),
                                         (640, 480, 42, dict(nscales=4, warps=10, epsilon=0.003))])
def test_mid_check_passes(built, monkeypatch, capfd, mid_min, W, H, seed, kw):
    p = capi.make_params(**kw)
    I0, I1 = synth.gen_pair(W, H, seed=seed)
    res = {}
    for mid in ("1", "0"):
        set_knobs(monkeypatch, f"TVL1_ROLL_LONG_MIN=0,TVL1_SPEC=0,TVL1_SPEC_TRACE=1,TVL1_MID={mid},"
                               f"TVL1_MID_MIN={mid_min}")
        capfd.readouterr()
        eng = capi.Engine(p)
        res[mid] = eng.calc_host(I0, I1)
        eng.close()
        res[mid + "err"] = capfd.readouterr().err
    m = MID_RE.search(res["1err"])
    assert m and int(m.group(1)) > 0, "no mid-check pass ran"
    assert not MID_RE.search(res["0err"])
    (u, v, st, wi), (u0, v0, st0, wi0) = res["1"], res["0"]
    np.testing.assert_array_equal(wi, wi0)
    assert bits_equal(u, u0) and bits_equal(v, v0)
    assert st["checks_total"] == st0["checks_total"]
    ur, vr, _, wr = checker.oracle_calc(I0, I1, p)
    np.testing.assert_array_equal(wi, wr)
    assert bits_equal(u, ur) and bits_equal(v, vr)
    print(f"mid-check passes {m.group(1)}, ended on the mid state {m.group(2)}")
    if mid_min == "1" and (W, H) == (250, 131):
        assert int(m.group(2)) > 0, "no mid-check pass ended on its first check"


@pytest.fixture(scope="module")
def c2_oracle():
    I0, I1 = synth.gen_pair(6144, 4096, seed=0x5EED, z=1)
    p = capi.make_params(nscales=5, warps=30)
    return I0, I1, p, checker.oracle_calc(I0, I1, p)


def test_benchmark_pair_bit_exact(engine, c2_oracle):
    """The bench workload itself (BASELINE configs[1], C2): one 6144x4096 synthetic pair,
    5 scales, 30 warps -- the same bits and the same 880-odd iterations as the oracle."""
    I0, I1, p, (ur, vr, sr, wr) = c2_oracle
    engine.set_params(p)
    u, v, st, wi = engine.calc_host(I0, I1)
    assert st["levels"] == sr["levels"] == 5
    np.testing.assert_array_equal(wi, wr)
    assert bits_equal(u, ur) and bits_equal(v, vr)
    print(f"C2 pair: {int(wi.sum())} iterations, bit-exact vs oracle")


def test_benchmark_pair_bit_exact_mid_checks(built, monkeypatch, capfd, c2_oracle):
    """The C2 pair as the bench's in-flight solves run it (nothing enqueued behind a check, so
    its converging warps' 2-iteration passes run as mid-check passes): the same bits."""
    I0, I1, p, (ur, vr, sr, wr) = c2_oracle
    set_knobs(monkeypatch, "TVL1_SPEC=0,TVL1_SPEC_TRACE=1,TVL1_MID=1")
    capfd.readouterr()
    eng = capi.Engine(p)
    u, v, st, wi = eng.calc_host(I0, I1)
    eng.close()
    m = MID_RE.search(capfd.readouterr().err)
    assert m and int(m.group(1)) >= 4, "the C2 pair's level-0 run took no mid-check passes"
    np.testing.assert_array_equal(wi, wr)
    assert bits_equal(u, ur) and bits_equal(v, vr)
    print(f"C2 pair: mid-check passes {m.group(1)}, ended on the mid state {m.group(2)}")


def test_benchmark_pair_bit_exact_fma_mode(engine):
    """The same C2 pair in fma mode (fast_math = 2, nvcc's -fmad=true contraction restated):
    bit-identical to the oracle's fma mode at full size, with its own iteration schedule (the
    bench's `math_modes.fma` leg runs this arithmetic)."""
    I0, I1 = synth.gen_pair(6144, 4096, seed=0x5EED, z=1)
    p = capi.make_params(nscales=5, warps=30, fast_math=2)
    engine.set_params(p)
    u, v, st, wi = engine.calc_host(I0, I1)
    ur, vr, sr, wr = checker.oracle_calc(I0, I1, p)
    assert st["levels"] == sr["levels"] == 5
    np.testing.assert_array_equal(wi, wr)
    assert bits_equal(u, ur) and bits_equal(v, vr)
    print(f"C2 pair, fma mode: {int(wi.sum())} iterations, bit-exact vs the oracle's fma mode")


# Profile 1: OpenCV's CPU DualTVL1OpticalFlow schedule, bit-identical to
# its restatement (oracle/tvl1_oracle_dualtvl1.c; parity with OpenCV itself unpinned).
P1_CASES = [
    (64, 48, 41, dict(nscales=4, warps=3)),
    (17, 16, 42, dict(nscales=3, warps=2)),
    (250, 131, 43, dict(nscales=5, warps=5, lambda_=0.15, median_filtering=5)),  # CPU defaults
    (96, 64, 44, dict(nscales=4, warps=3, gamma=0.2, median_filtering=5)),
    (96, 64, 45, dict(nscales=4, warps=3, median_filtering=3)),
    (120, 90, 46, dict(nscales=3, warps=2, epsilon=0.0, inner_iterations=3, outer_iterations=2)),
    (128, 96, 47, dict(nscales=4, warps=2, scale_step=0.5)),                     # 2x area path
    (70, 50, 48, dict(nscales=3, warps=2, tau=-0.05, inner_iterations=4, outer_iterations=2)),
]


@pytest.mark.parametrize("W,H,seed,kw", P1_CASES)
def test_dualtvl1_profile_matches_oracle(engine, W, H, seed, kw):
    I0, I1 = synth.gen_pair(W, H, seed=seed)
    p = capi.make_params(profile=1, **kw)
    engine.set_params(p)
    u, v, st, wi = engine.calc_host(I0, I1)
    ur, vr, sr, wr = checker.oracle_calc(I0, I1, p)
    assert st["levels"] == sr["levels"]
    np.testing.assert_array_equal(wi, wr)
    fin = np.isfinite(ur) & np.isfinite(vr)
    assert np.array_equal(fin, np.isfinite(u) & np.isfinite(v))
    assert bits_equal(u[fin], ur[fin]) and bits_equal(v[fin], vr[fin]), \
        f"max|du|={np.abs(u - ur)[fin].max()} max|dv|={np.abs(v - vr)[fin].max()}"


def test_dualtvl1_profile_identity(engine):
    I0, _ = synth.gen_pair(80, 60, seed=3)
    engine.set_params(capi.make_params(profile=1, nscales=4, warps=3))
    u, v, st, wi = engine.calc_host(I0, I0)
    assert np.all(u == 0) and np.all(v == 0)
    assert np.all(wi == 1)


@pytest.mark.parametrize("profile", [0, 1])
def test_f32_inputs_match_oracle(built, profile):
    """tvl1_calc_f32 (CV_32FC1 frames, scaled by 255 on entry) vs the oracle's f32 path,
    bitwise, on off-grid float frames; and u8 frames given as k / 255 reproduce tvl1_calc."""
    I0, I1 = synth.gen_pair(203, 131, seed=77)
    kw = dict(nscales=4, warps=5) if profile == 0 else dict(profile=1, nscales=3, warps=2,
                                                               inner_iterations=4,
                                                               outer_iterations=2)
    p = capi.make_params(**kw)
    eng = capi.Engine(p)
    rng = np.random.default_rng(5)
    J0 = (I0 / 255.0 + rng.normal(0, 2e-3, I0.shape)).astype(np.float32)
    J1 = (I1 / 255.0 + rng.normal(0, 2e-3, I1.shape)).astype(np.float32)
    H, W = I0.shape
    dev = torch.device("cuda", 0)
    for F0, F1 in ((J0, J1), (I0.astype(np.float32) / np.float32(255),
                               I1.astype(np.float32) / np.float32(255))):
        d0 = torch.from_numpy(F0).to(dev)
        d1 = torch.from_numpy(F1).to(dev)
        du = torch.zeros((H, W), dtype=torch.float32, device=dev)
        dv = torch.zeros_like(du)
        st = eng.calc_device(d0.data_ptr(), 4 * W, d1.data_ptr(), 4 * W, W, H, du.data_ptr(),
                             dv.data_ptr(), 4 * W, warp_iters=True, f32=True)
        torch.cuda.synchronize()
        u, v = du.cpu().numpy(), dv.cpu().numpy()
        ur, vr, sr, wr = checker.oracle_calc(F0, F1, p)
        assert np.array_equal(u.view(np.uint32), ur.view(np.uint32))
        assert np.array_equal(v.view(np.uint32), vr.view(np.uint32))
        np.testing.assert_array_equal(st["warp_iters"], wr)
    # the k / 255 frames (last loop pass) against the u8 entry point
    uu, vu, _, _ = eng.calc_host(I0, I1)
    assert np.array_equal(u.view(np.uint32), uu.view(np.uint32))
    assert np.array_equal(v.view(np.uint32), vu.view(np.uint32))
    eng.close()
