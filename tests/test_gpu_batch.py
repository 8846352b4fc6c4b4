"""tvl1_calc_batch (the production strip workload): every pair of a batch must
get exactly the single-pair result -- bit-identical flow and the same per-warp iteration
counts as the oracle -- whatever the other pairs of the batch do."""
import numpy as np
import pytest

from optflow_amd import capi, synth
from oracle import checker

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32),
                          np.ascontiguousarray(b).view(np.uint32))


def run_batch(eng, I0s, I1s):
    """Pairs packed contiguously on the device (pair stride = one image)."""
    n, h, w = I0s.shape
    dev = torch.device("cuda", 0)
    d0 = torch.from_numpy(np.ascontiguousarray(I0s)).to(dev)
    d1 = torch.from_numpy(np.ascontiguousarray(I1s)).to(dev)
    du = torch.zeros((n, h, w), dtype=torch.float32, device=dev)
    dv = torch.zeros((n, h, w), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    st = eng.calc_batch_device(n, d0.data_ptr(), w, w * h, d1.data_ptr(), w, w * h, w, h,
                               du.data_ptr(), dv.data_ptr(), 4 * w, 4 * w * h, warp_iters=True)
    torch.cuda.synchronize()
    return du.cpu().numpy(), dv.cpu().numpy(), st


def check_against_oracle(p, I0s, I1s, u, v, st):
    for b in range(I0s.shape[0]):
        ur, vr, sr, wr = checker.oracle_calc(I0s[b], I1s[b], p)
        assert st[b]["levels"] == sr["levels"]
        np.testing.assert_array_equal(st[b]["warp_iters"], wr, err_msg=f"pair {b}")
        assert bits_equal(u[b], ur) and bits_equal(v[b], vr), f"pair {b} not bit-exact"


def pairs(n, w, h, seed):
    I0s, I1s = [], []
    for b in range(n):
        a, c = synth.gen_pair(w, h, seed=seed + b, z=1 + b % 3)
        I0s.append(a)
        I1s.append(c)
    return np.stack(I0s), np.stack(I1s)


@pytest.mark.parametrize("n,w,h,kw", [
    (6, 300, 100, dict(nscales=10, warps=5)),          # production strip shape (scaled down)
    (3, 250, 131, dict(nscales=5, warps=5)),
    (1, 97, 40, dict(nscales=3, warps=3)),
    (5, 200, 60, dict(nscales=4, warps=3, epsilon=0.0, iterations=7)),   # fixed work
])
@pytest.mark.parametrize("env", ["", "TVL1_BATCH_FUSE=0", "TVL1_WI_NC=1", "TVL1_BATCH_STORE=1",
                                 "TVL1_BATCH_GROUP=0", "TVL1_BATCH_PX1_W=0",
                                 "TVL1_BATCH_PX1_W=150", "TVL1_BATCH_SEG_MIN=0",
                                 "TVL1_BATCH_SEG_MIN=16", "TVL1_BATCH_SMALL=0"])
@pytest.mark.parametrize("math", [0, 2])
def test_batch_matches_oracle(built, monkeypatch, env, n, w, h, kw, math):
    """kb_warp_iter (fused warp + first pass; 2 consumer wavefronts, or 1 with
    TVL1_WI_NC=1; constants stored on demand, or always with TVL1_BATCH_STORE=1), passes grouped
    by their length (or r3's lock step with TVL1_BATCH_GROUP=0),
    kb_warp_ring, kb_iterate_roll<K, 1> (every level of these sizes is under the 1700-px
    cut-off; <K, 2> everywhere with TVL1_BATCH_PX1_W=0, above 150 px with =150): IEEE and fma
    mode, each bit-identical to the oracle in that mode."""
    monkeypatch.delenv("TVL1_BATCH_FUSE", raising=False)
    monkeypatch.delenv("TVL1_WI_NC", raising=False)
    monkeypatch.delenv("TVL1_BATCH_STORE", raising=False)
    monkeypatch.delenv("TVL1_BATCH_GROUP", raising=False)
    monkeypatch.delenv("TVL1_BATCH_PX1_W", raising=False)
    monkeypatch.delenv("TVL1_BATCH_SEG_MIN", raising=False)
    monkeypatch.delenv("TVL1_BATCH_SMALL", raising=False)
    for kv in filter(None, env.split(",")):
        monkeypatch.setenv(*kv.split("="))
    p = capi.make_params(fast_math=math, **kw)
    eng = capi.Engine(p)
    I0s, I1s = pairs(n, w, h, seed=100 + n)
    u, v, st = run_batch(eng, I0s, I1s)
    eng.close()
    check_against_oracle(p, I0s, I1s, u, v, st)


def test_batch_of_full_frame_geometry_pairs(built):
    """C2's pyramid and schedule at a quarter of its width and height -- 3
    pairs of 1536x1024, nscales 5, warps 30, iterations 300, epsilon 0.01 -- through one
    tvl1_calc_batch, every pair bit-identical to the oracle with the same per-warp counts
    (the A/B against 3 single-pair solves in flight is profiles/r5/ab/batch_c2/)."""
    p = capi.make_params(nscales=5, warps=30, iterations=300, epsilon=0.01)
    eng = capi.Engine(p)
    I0s, I1s = pairs(3, 1536, 1024, seed=0x5EED)
    u, v, st = run_batch(eng, I0s, I1s)
    eng.close()
    check_against_oracle(p, I0s, I1s, u, v, st)


@pytest.mark.parametrize("w,h", [(576, 15), (529, 17), (65, 17), (64, 3), (130, 1), (1, 17),
                                 (7, 2), (300, 12)])
@pytest.mark.parametrize("kw", [dict(nscales=1, warps=5),
                                dict(nscales=1, warps=3, epsilon=0.0, iterations=9)])
@pytest.mark.parametrize("math", [0, 2])
def test_batch_coarsest_level_on_chip_edges(built, w, h, kw, math):
    """kb_small_level at the edges of what it takes (one level, so the whole solve is the
    coarsest level): 576 px = 9 full wavefronts, 529 x 17 = its row limit, 65 = a one-lane
    last wavefront, one row, one column; stopping rule and fixed work (epsilon 0); IEEE and
    fma mode, each bit-identical to the oracle in that mode."""
    p = capi.make_params(fast_math=math, **kw)
    eng = capi.Engine(p)
    I0s, I1s = pairs(3, w, h, seed=w * 131 + h)
    u, v, st = run_batch(eng, I0s, I1s)
    eng.close()
    check_against_oracle(p, I0s, I1s, u, v, st)


def test_batch_larger_than_one_chunk(built):
    """260 pairs: two chunks (256 + 4), plus an identical pair (stops at n = 2 everywhere)."""
    p = capi.make_params(nscales=3, warps=2)
    eng = capi.Engine(p)
    I0s, I1s = pairs(260, 64, 24, seed=7)
    I1s[5] = I0s[5]
    u, v, st = run_batch(eng, I0s, I1s)
    eng.close()
    assert np.all(u[5] == 0) and np.all(st[5]["warp_iters"] == 2)
    sel = [0, 5, 63, 64, 200, 255, 256, 259]
    check_against_oracle(p, I0s[sel], I1s[sel], u[sel], v[sel], [st[b] for b in sel])


def test_batch_strided_stack(built):
    """Adjacent pairs (z, z+1) of one contiguous device stack: I1 of pair b is I0 of b+1."""
    Z, w, h = 6, 160, 48
    stack = np.stack([synth.gen_pair(w, h, seed=3, z=z)[1] for z in range(Z)])
    p = capi.make_params(nscales=4, warps=4)
    eng = capi.Engine(p)
    dev = torch.device("cuda", 0)
    ds = torch.from_numpy(stack).to(dev)
    n = Z - 1
    du = torch.zeros((n, h, w), dtype=torch.float32, device=dev)
    dv = torch.zeros((n, h, w), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    st = eng.calc_batch_device(n, ds.data_ptr(), w, w * h, ds.data_ptr() + w * h, w, w * h, w,
                               h, du.data_ptr(), dv.data_ptr(), 4 * w, 4 * w * h,
                               warp_iters=True)
    torch.cuda.synchronize()
    eng.close()
    check_against_oracle(p, stack[:-1], stack[1:], du.cpu().numpy(), dv.cpu().numpy(), st)


@pytest.mark.parametrize("kw", [dict(median_filtering=5), dict(median_filtering=3)])
def test_batch_median(built, kw):
    p = capi.make_params(nscales=4, warps=3, **kw)
    eng = capi.Engine(p)
    I0s, I1s = pairs(4, 120, 50, seed=61)
    u, v, st = run_batch(eng, I0s, I1s)
    eng.close()
    check_against_oracle(p, I0s, I1s, u, v, st)


@pytest.mark.parametrize("env", ["", "TVL1_BATCH_FUSE=0", "TVL1_BATCH_PX1_W=0"])
def test_batch_fast_math_within_tolerance(built, monkeypatch, env):
    """fast_math = 1 batches: the oracle's iteration schedule, mean EPE <= 1e-3 px
    (tests/test_gpu_fastmath.py's bar)."""
    monkeypatch.delenv("TVL1_BATCH_FUSE", raising=False)
    monkeypatch.delenv("TVL1_BATCH_PX1_W", raising=False)
    monkeypatch.delenv("TVL1_BATCH_SEG_MIN", raising=False)
    monkeypatch.delenv("TVL1_BATCH_SMALL", raising=False)
    for kv in filter(None, env.split(",")):
        monkeypatch.setenv(*kv.split("="))
    kw = dict(nscales=10, warps=5)
    eng = capi.Engine(capi.make_params(fast_math=1, **kw))
    I0s, I1s = pairs(4, 300, 100, seed=71)
    u, v, st = run_batch(eng, I0s, I1s)
    eng.close()
    p = capi.make_params(**kw)
    for b in range(4):
        ur, vr, sr, wr = checker.oracle_calc(I0s[b], I1s[b], p)
        np.testing.assert_array_equal(st[b]["warp_iters"], wr)
        e = capi.epe(u[b], v[b], ur, vr)
        assert float(e.mean()) <= 1e-3 and float((e > 1e-2).mean()) <= 1e-3


@pytest.mark.parametrize("kw", [dict(gamma=0.2), dict(profile=1)])
def test_batch_falls_back_per_pair(built, kw):
    """Parameter sets outside the batched kernels solve pair by pair: same results."""
    p = capi.make_params(nscales=3, warps=2, **kw)
    eng = capi.Engine(p)
    I0s, I1s = pairs(3, 90, 40, seed=55)
    u, v, st = run_batch(eng, I0s, I1s)
    eng.close()
    check_against_oracle(p, I0s, I1s, u, v, st)


@pytest.mark.parametrize("where", ["top", "bottom"])
def test_batch_roi_strips_of_a_stack(built, where):
    """top / bottom ROI strips (a sub-view of every slice) of adjacent
    pairs of one device stack in one call -- the production layout."""
    Z, w, h, rows = 5, 130, 60, 20
    stack = np.stack([synth.gen_pair(w, h, seed=9, z=z)[1] for z in range(Z)])
    p = capi.make_params(nscales=10, warps=3)
    eng = capi.Engine(p)
    dev = torch.device("cuda", 0)
    ds = torch.from_numpy(stack).to(dev)
    n = Z - 1
    off = 0 if where == "top" else (h - rows) * w
    du = torch.zeros((n, rows, w), dtype=torch.float32, device=dev)
    dv = torch.zeros((n, rows, w), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    st = eng.calc_batch_device(n, ds.data_ptr() + off, w, w * h, ds.data_ptr() + w * h + off, w,
                               w * h, w, rows, du.data_ptr(), dv.data_ptr(), 4 * w, 4 * w * rows,
                               warp_iters=True)
    torch.cuda.synchronize()
    eng.close()
    sl = slice(0, rows) if where == "top" else slice(h - rows, h)
    I0s = np.ascontiguousarray(stack[:-1, sl])
    I1s = np.ascontiguousarray(stack[1:, sl])
    check_against_oracle(p, I0s, I1s, du.cpu().numpy(), dv.cpu().numpy(), st)


def test_batch_of_benchmark_pairs_equals_single_solves(built):
    """Two 6144x4096 pairs (C2) in one batch: the same bits and iteration counts as
    tvl1_calc on each (which matches the oracle at this size, test_benchmark_pair_bit_exact)."""
    p = capi.make_params(nscales=5, warps=30)
    eng = capi.Engine(p)
    I0s, I1s = [], []
    for z in (1, 2):
        a, c = synth.gen_pair(6144, 4096, seed=0x5EED, z=z)
        I0s.append(a)
        I1s.append(c)
    I0s, I1s = np.stack(I0s), np.stack(I1s)
    u, v, st = run_batch(eng, I0s, I1s)
    for b in range(2):
        us, vs, ss, ws = eng.calc_host(I0s[b], I1s[b])
        np.testing.assert_array_equal(st[b]["warp_iters"], ws)
        assert bits_equal(u[b], us) and bits_equal(v[b], vs)
    eng.close()


def test_batch_shared_reference_frame(built):
    """pair_stride0 = 0: every pair registers against the same I0."""
    w, h, n = 140, 50, 4
    I0, _ = synth.gen_pair(w, h, seed=13)
    I1s = np.stack([synth.gen_pair(w, h, seed=13, z=z)[1] for z in range(1, n + 1)])
    p = capi.make_params(nscales=5, warps=3)
    eng = capi.Engine(p)
    dev = torch.device("cuda", 0)
    d0 = torch.from_numpy(I0).to(dev)
    d1 = torch.from_numpy(I1s).to(dev)
    du = torch.zeros((n, h, w), dtype=torch.float32, device=dev)
    dv = torch.zeros((n, h, w), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    st = eng.calc_batch_device(n, d0.data_ptr(), w, 0, d1.data_ptr(), w, w * h, w, h,
                               du.data_ptr(), dv.data_ptr(), 4 * w, 4 * w * h, warp_iters=True)
    torch.cuda.synchronize()
    eng.close()
    check_against_oracle(p, np.stack([I0] * n), I1s, du.cpu().numpy(), dv.cpu().numpy(), st)


def test_batch_arena_relaid_after_scale_step_change(built):
    """set_params with a new scaleStep but the same level count must
    re-lay the batch arena -- the level planes grow (0.5 -> 0.8), and a reused arena would
    let each pair's pyramid spill into its neighbour's planes."""
    w, h, n = 256, 192, 3
    I0s, I1s = pairs(n, w, h, seed=91)
    p05 = capi.make_params(nscales=4, warps=3, scale_step=0.5)
    p08 = capi.make_params(nscales=4, warps=3, scale_step=0.8)
    eng = capi.Engine(p05)
    u, v, st = run_batch(eng, I0s, I1s)
    check_against_oracle(p05, I0s, I1s, u, v, st)
    eng.set_params(p08)
    u, v, st = run_batch(eng, I0s, I1s)
    assert st[0]["levels"] == 4
    check_against_oracle(p08, I0s, I1s, u, v, st)
    for b in range(n):   # and the single-pair path on the same ctx agrees
        us, vs, ss, ws = eng.calc_host(I0s[b], I1s[b])
        np.testing.assert_array_equal(st[b]["warp_iters"], ws)
        assert bits_equal(u[b], us) and bits_equal(v[b], vs)
    eng.close()


def test_arena_growth_keeps_other_contexts_running(built):
    """Arena growth is stream-ordered (no device-wide drain): a ctx whose arena grows while
    another ctx's solve is in flight on its own stream leaves both results exact."""
    pa = capi.make_params(nscales=5, warps=5)
    ea, eb = capi.Engine(pa), capi.Engine(pa)
    dev = torch.device("cuda", 0)
    big0, big1 = synth.gen_pair(1536, 1024, seed=5, z=1)
    sm0, sm1 = synth.gen_pair(200, 120, seed=6, z=2)
    lg0, lg1 = synth.gen_pair(700, 500, seed=7, z=3)
    tb0, tb1 = torch.from_numpy(big0).to(dev), torch.from_numpy(big1).to(dev)
    ub = torch.zeros((1024, 1536), dtype=torch.float32, device=dev)
    vb = torch.zeros_like(ub)
    torch.cuda.synchronize()
    # ctx b: small solve first (small arena), then grow while ctx a runs the big pair
    eb.calc_host(sm0, sm1)
    import threading
    res = {}
    t = threading.Thread(target=lambda: res.setdefault(
        "a", ea.calc_device(tb0.data_ptr(), 1536, tb1.data_ptr(), 1536, 1536, 1024,
                            ub.data_ptr(), vb.data_ptr(), 4 * 1536, stream=ea.stream)))
    t.start()
    ul, vl, sl, wl = eb.calc_host(lg0, lg1)   # grows ctx b's arena
    t.join()
    torch.cuda.synchronize()
    ur, vr, sr, wr = checker.oracle_calc(lg0, lg1, pa)
    assert bits_equal(ul, ur) and bits_equal(vl, vr)
    us, vs, ss, ws = ea.calc_host(big0, big1)
    assert bits_equal(ub.cpu().numpy(), us) and bits_equal(vb.cpu().numpy(), vs)
    ea.close()
    eb.close()


def test_batch_profiling_classes_and_same_bits(built):
    """tvl1_set_profiling on a batch: every pair reports the chunk's per-class launch times,
    launches and accounted bytes (the production_strips roofline of bench.py), and the
    events change no bit."""
    p = capi.make_params(nscales=10, warps=5)
    eng = capi.Engine(p)
    I0s, I1s = pairs(6, 300, 100, seed=121)
    u0, v0, st0 = run_batch(eng, I0s, I1s)
    eng.set_profiling(True)
    u1, v1, st1 = run_batch(eng, I0s, I1s)
    eng.set_profiling(False)
    eng.close()
    assert bits_equal(u0, u1) and bits_equal(v0, v1)
    for b in range(6):
        np.testing.assert_array_equal(st0[b]["warp_iters"], st1[b]["warp_iters"])
        assert st0[b]["kernel_launches"][0] == 0
        assert st1[b]["kernel_launches"][0] > 0 and st1[b]["kernel_ms"][0] > 0
        assert st1[b]["kernel_hbm_bytes"][0] > 0 and st1[b]["kernel_bytes"][0] > 0
        assert st1[b]["kernel_ms"] == st1[0]["kernel_ms"]   # one chunk: shared launches


def test_batch_constants_on_demand_regather(built, monkeypatch):
    """Production strips (3072x100 slices of the host stack recipe, nscales 10, warps 5):
    kb_warp_iter stores the warp constants only for pairs predicted to continue past the first
    check (a level's first warp, or the previous warp ran on); a pair that continues anyway is
    re-gathered (kb_warp_ring) -- counted in speculation_misses.  The prediction is right for
    ~99 % of strip warps; these 12 pairs hold 4 wrong ones (the oracle's per-warp counts: a
    warp of 2 iterations followed by a longer one), so the path must run, and every pair stay
    bit-identical to the oracle."""
    monkeypatch.delenv("TVL1_BATCH_STORE", raising=False)
    n, w, h = 12, 3072, 100
    st_ = synth.gen_stack(w, h, n + 1, seed=0x5EED)
    I0s = np.stack([st_[0]] * n)
    I1s = np.stack([st_[z + 1] for z in range(n)])
    p = capi.make_params(nscales=10, warps=5)
    eng = capi.Engine(p)
    u, v, st = run_batch(eng, I0s, I1s)
    eng.close()
    assert sum(s["speculation_misses"] for s in st) > 0
    check_against_oracle(p, I0s, I1s, u, v, st)


@pytest.mark.parametrize("w,h", [(529, 17), (300, 12)])
def test_batch_small_level_stopping_decisions_across_thresholds(built, monkeypatch, w, h):
    """kb_small_level sums the residual in its own order (column sums, then lanes
    and wavefronts in a fixed order), so its stopping decisions equal the streaming path's only
    while every check sits further from its threshold than the two sums differ.
    Pinned empirically here: one level (the whole solve on chip), 16 epsilons spread over
    0.003 ... 0.06 -- each moves scaledEps, so the checks land at many different distances from
    the thresholds -- times 6 pairs, solved with the on-chip level and with TVL1_BATCH_SMALL=0:
    the per-warp iteration counts, the check counts and the flow bits must be identical, and
    the same as the oracle's for the first and last epsilon."""
    eps = np.geomspace(0.003, 0.06, 16)
    I0s, I1s = pairs(6, w, h, seed=w + 7 * h)
    for k, e in enumerate(eps):
        out = {}
        for small in ("1", "0"):
            monkeypatch.setenv("TVL1_BATCH_SMALL", small)
            p = capi.make_params(nscales=1, warps=5, epsilon=float(e))
            eng = capi.Engine(p)
            out[small] = run_batch(eng, I0s, I1s)
            eng.close()
        (u1, v1, s1), (u0, v0, s0) = out["1"], out["0"]
        for b in range(I0s.shape[0]):
            np.testing.assert_array_equal(s1[b]["warp_iters"], s0[b]["warp_iters"],
                                          err_msg=f"eps {e:.5f} pair {b}")
            assert s1[b]["checks_total"] == s0[b]["checks_total"], (e, b)
        assert bits_equal(u1, u0) and bits_equal(v1, v0), f"eps {e:.5f}"
        if k in (0, len(eps) - 1):
            check_against_oracle(p, I0s, I1s, u1, v1, s1)
    monkeypatch.delenv("TVL1_BATCH_SMALL", raising=False)
