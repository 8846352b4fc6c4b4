"""Context lifecycle and concurrency: re-created contexts, contexts solving at
once with speculation, and batch arenas under alternating geometries.  Every result is held
to the same bar as tests/test_gpu_parity.py: bit-identical to the oracle, same per-warp
iteration counts."""
import threading

import numpy as np
import pytest

from optflow_amd import capi, synth
from oracle import checker

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def bits_equal(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_recreated_ctx_bit_identical(built):
    """tvl1_create after tvl1_destroy in one process: the new ctx's pinned residual slots
    (sequence word included) may come from the freed ctx's block; they must start at zero,
    or the residual poll would read a stale residual and the stopping rule act on it."""
    I0, I1 = synth.gen_pair(320, 240, seed=51)
    p = capi.make_params(nscales=4, warps=8)
    ur, vr, _, wr = checker.oracle_calc(I0, I1, p)
    for rep in range(4):
        eng = capi.Engine(p)
        for _ in range(1 + rep % 2):   # a later ctx inherits a larger sequence number
            u, v, st, wi = eng.calc_host(I0, I1)
            np.testing.assert_array_equal(wi, wr, err_msg=f"ctx {rep}")
            assert bits_equal(u, ur) and bits_equal(v, vr), f"ctx {rep}"
        eng.close()


@pytest.mark.parametrize("spec", ["2", "1"])
def test_concurrent_contexts_with_speculation(built, monkeypatch, spec):
    """3 contexts solving at once on their own streams.  TVL1_SPEC=2: every check enqueues
    its guess even while the other solves share the device, so misses (the rewind path) do
    happen; TVL1_SPEC=1 (default): speculation switches on and off mid-solve as the count of
    solves in progress changes.  Every result equals the oracle's."""
    monkeypatch.setenv("TVL1_SPEC", spec)
    cases = [(256, 200, 61, dict(nscales=3, warps=6, epsilon=0.002)),
             (320, 240, 62, dict(nscales=4, warps=10)),
             (200, 150, 63, dict(nscales=3, warps=4, gamma=0.2))]
    engines = [capi.Engine(capi.make_params(**kw)) for (_, _, _, kw) in cases]
    inputs = [synth.gen_pair(W, H, seed=s) for (W, H, s, _) in cases]
    out = [None] * len(cases)
    errs = []

    def run(i):
        try:
            res = []
            for _ in range(3):
                res.append(engines[i].calc_host(*inputs[i]))
            out[i] = res
        except Exception as e:   # reported below, in the test thread
            errs.append(e)

    ths = [threading.Thread(target=run, args=(i,)) for i in range(len(cases))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for e in engines:
        e.close()
    assert not errs, errs
    misses = 0
    for i, (W, H, s, kw) in enumerate(cases):
        ur, vr, _, wr = checker.oracle_calc(*inputs[i], capi.make_params(**kw))
        for (u, v, st, wi) in out[i]:
            np.testing.assert_array_equal(wi, wr, err_msg=f"case {i}")
            assert bits_equal(u, ur) and bits_equal(v, vr), f"case {i}"
            misses += st["speculation_misses"]
    print(f"TVL1_SPEC={spec}: {misses} speculation misses over 9 solves")
    if spec == "2":
        assert misses > 0, "the miss / rewind path was not reached"


def test_batch_alternating_geometries_hold_one_arena(built):
    """Two strip geometries alternated on one ctx: the batch arena is re-laid, not
    re-allocated, once it is large enough, so device memory stops falling after the first
    round; every batch stays bit-identical to the oracle."""
    p = capi.make_params(nscales=4, warps=3)
    eng = capi.Engine(p)
    dev = torch.device("cuda", 0)
    shapes = [(300, 100, 6), (200, 60, 9)]
    data = {}
    for (w, h, n) in shapes:
        I0s = np.stack([synth.gen_pair(w, h, seed=80 + b)[0] for b in range(n)])
        I1s = np.stack([synth.gen_pair(w, h, seed=80 + b)[1] for b in range(n)])
        data[(w, h, n)] = (I0s, I1s)
    free = []
    for rnd in range(4):
        for (w, h, n) in shapes:
            I0s, I1s = data[(w, h, n)]
            d0 = torch.from_numpy(I0s).to(dev)
            d1 = torch.from_numpy(I1s).to(dev)
            du = torch.zeros((n, h, w), dtype=torch.float32, device=dev)
            dv = torch.zeros_like(du)
            torch.cuda.synchronize()
            st = eng.calc_batch_device(n, d0.data_ptr(), w, w * h, d1.data_ptr(), w, w * h, w, h,
                                       du.data_ptr(), dv.data_ptr(), 4 * w, 4 * w * h,
                                       warp_iters=True)
            torch.cuda.synchronize()
            if rnd in (0, 3):
                u, v = du.cpu().numpy(), dv.cpu().numpy()
                for b in range(n):
                    ur, vr, _, wr = checker.oracle_calc(I0s[b], I1s[b], p)
                    np.testing.assert_array_equal(st[b]["warp_iters"], wr)
                    assert bits_equal(u[b], ur) and bits_equal(v[b], vr), (w, h, b)
            del d0, d1, du, dv
        torch.cuda.empty_cache()
        free.append(torch.cuda.mem_get_info(0)[0])
    eng.close()
    # after round 0 the arena has its final size: no further device memory is taken
    assert min(free[1:]) >= free[0] - (8 << 20), free


def test_concurrent_batches_bit_identical(built):
    """Two tvl1_calc_batch calls at once on their own contexts and streams: each counts as a
    solve in progress on the device (single-pair solves running beside them size their
    streaming launches for the shared share, fill_shared; the batched launches themselves
    keep full-slot sizing, solve_batch_chunk), and every pair still equals the oracle bit for
    bit."""
    p = capi.make_params(nscales=5, warps=4)
    dev = torch.device("cuda", 0)
    jobs = []
    for j in range(2):
        n, w, h = 5, 260, 90
        I0s = np.stack([synth.gen_pair(w, h, seed=140 + 10 * j + b)[0] for b in range(n)])
        I1s = np.stack([synth.gen_pair(w, h, seed=140 + 10 * j + b)[1] for b in range(n)])
        jobs.append(dict(eng=capi.Engine(p), I0s=I0s, I1s=I1s, n=n, w=w, h=h,
                         d0=torch.from_numpy(I0s).to(dev), d1=torch.from_numpy(I1s).to(dev),
                         du=torch.zeros((n, h, w), dtype=torch.float32, device=dev),
                         dv=torch.zeros((n, h, w), dtype=torch.float32, device=dev)))
    torch.cuda.synchronize()
    errs = []

    def run(jb):
        try:
            e, n, w, h = jb["eng"], jb["n"], jb["w"], jb["h"]
            for _ in range(3):
                jb["st"] = e.calc_batch_device(n, jb["d0"].data_ptr(), w, w * h, jb["d1"].data_ptr(),
                                               w, w * h, w, h, jb["du"].data_ptr(), jb["dv"].data_ptr(),
                                               4 * w, 4 * w * h, stream=e.stream, warp_iters=True)
            torch.cuda.ExternalStream(e.stream, device=dev).synchronize()
        except Exception as ex:
            errs.append(ex)

    ths = [threading.Thread(target=run, args=(jb,)) for jb in jobs]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    for jb in jobs:
        u, v = jb["du"].cpu().numpy(), jb["dv"].cpu().numpy()
        for b in range(jb["n"]):
            ur, vr, _, wr = checker.oracle_calc(jb["I0s"][b], jb["I1s"][b], p)
            np.testing.assert_array_equal(jb["st"][b]["warp_iters"], wr)
            assert bits_equal(u[b], ur) and bits_equal(v[b], vr)
        jb["eng"].close()


def test_batch_relaid_across_streams_without_sync(built):
    """one ctx runs tvl1_calc_batch on stream A, then, with no host sync, a smaller
    geometry on stream B -- ensure_batch re-lays the same arena in place.  order_streams makes
    B wait for A's last kernels (kb_output reads the old layout), so both batches equal the
    oracle bit for bit."""
    p = capi.make_params(nscales=4, warps=3)
    dev = torch.device("cuda", 0)
    eng = capi.Engine(p)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    jobs = []
    for (n, w, h, seed) in ((6, 300, 120, 300), (4, 200, 70, 310)):
        I0s = np.stack([synth.gen_pair(w, h, seed=seed + b)[0] for b in range(n)])
        I1s = np.stack([synth.gen_pair(w, h, seed=seed + b)[1] for b in range(n)])
        jobs.append(dict(n=n, w=w, h=h, I0s=I0s, I1s=I1s, d0=torch.from_numpy(I0s).to(dev),
                         d1=torch.from_numpy(I1s).to(dev),
                         du=torch.zeros((n, h, w), dtype=torch.float32, device=dev),
                         dv=torch.zeros((n, h, w), dtype=torch.float32, device=dev)))
    torch.cuda.synchronize()
    for jb, st in zip(jobs, (sa, sb)):
        n, w, h = jb["n"], jb["w"], jb["h"]
        jb["st"] = eng.calc_batch_device(n, jb["d0"].data_ptr(), w, w * h, jb["d1"].data_ptr(), w,
                                         w * h, w, h, jb["du"].data_ptr(), jb["dv"].data_ptr(),
                                         4 * w, 4 * w * h, stream=st.cuda_stream, warp_iters=True)
    sb.synchronize()
    sa.synchronize()
    for jb in jobs:
        u, v = jb["du"].cpu().numpy(), jb["dv"].cpu().numpy()
        for b in range(jb["n"]):
            ur, vr, _, wr = checker.oracle_calc(jb["I0s"][b], jb["I1s"][b], p)
            np.testing.assert_array_equal(jb["st"][b]["warp_iters"], wr)
            assert bits_equal(u[b], ur) and bits_equal(v[b], vr), (jb["w"], b)
    eng.close()


def test_postprocess_batch_and_gather_flow(built):
    """ABI 8: tvl1_postprocess_batch equals tvl1_postprocess per pair (every mode, frame1
    masks with zeros), and tvl1_gather_flow returns exactly the addressed values; ABI 9: an
    offset outside [0, plane_elems) is TVL1_EINVAL, never a device read."""
    dev = torch.device("cuda", 0)
    n, w, h = 5, 70, 33
    rng = np.random.default_rng(9)
    u0 = torch.from_numpy(rng.standard_normal((n, h, w)).astype(np.float32)).to(dev)
    v0 = torch.from_numpy(rng.standard_normal((n, h, w)).astype(np.float32)).to(dev)
    I1 = rng.integers(0, 4, (n, h, w), dtype=np.uint8)
    dI1 = torch.from_numpy(I1).to(dev)
    eng = capi.Engine(capi.make_params())
    for mode in (0, 1, 2):
        ub, vb = u0.clone(), v0.clone()
        eng.postprocess_batch(n, ub.data_ptr(), vb.data_ptr(), 4 * w, 4 * w * h, dI1.data_ptr(),
                              w, w * h, w, h, mode)
        for b in range(n):
            us, vs = u0[b].clone(), v0[b].clone()
            eng.lib.tvl1_postprocess(eng.ctx, us.data_ptr(), vs.data_ptr(), 4 * w,
                                     dI1[b].data_ptr(), w, w, h, mode, None)
            torch.cuda.synchronize()
            assert torch.equal(ub[b].view(torch.int32), us.view(torch.int32)), (mode, b)
            assert torch.equal(vb[b].view(torch.int32), vs.view(torch.int32)), (mode, b)
    off = rng.integers(0, n * w * h, 1000)
    gu, gv = eng.gather_flow(u0.data_ptr(), v0.data_ptr(), n * w * h, off)
    np.testing.assert_array_equal(gu, u0.flatten().cpu().numpy()[off])
    np.testing.assert_array_equal(gv, v0.flatten().cpu().numpy()[off])
    last = np.array([n * w * h - 1])
    gu, gv = eng.gather_flow(u0.data_ptr(), v0.data_ptr(), n * w * h, last)
    assert gu[0] == u0.flatten()[-1].item() and gv[0] == v0.flatten()[-1].item()
    for bad in (n * w * h, -1, 1 << 40):
        with pytest.raises(capi.TVL1Error, match="outside"):
            eng.gather_flow(u0.data_ptr(), v0.data_ptr(), n * w * h, np.array([0, bad]))
    eng.close()


def test_solve_entry_points_reject_bad_arguments(built):
    """The reference's CV_Assert-style checks on the solve boundary (tvl1_calc,
    tvl1_calc_f32, tvl1_calc_batch): null pointers, empty or oversized frames, pitches
    below the width, batch strides that overlap, a non-positive batch size -- each a status
    with a message, before any launch; the ctx then still solves a pair bit-exactly."""
    import ctypes as C
    eng = capi.Engine(capi.make_params(nscales=2, warps=2))
    lib, ctx = eng.lib, eng.ctx
    w, h = 64, 48
    dev = torch.device("cuda", 0)
    d0 = torch.zeros((2, h, w), dtype=torch.uint8, device=dev)
    df = torch.zeros((4, h, w), dtype=torch.float32, device=dev)   # u fields, then v fields
    i0, f0, g0 = d0.data_ptr(), df.data_ptr(), df[2].data_ptr()
    EINVAL, ESIZE = 1, 2

    def calc(I0=i0, p0=w, I1=i0, p1=w, W=w, H=h, u=f0, v=g0, fp=4 * w):
        return lib.tvl1_calc(ctx, C.c_void_p(I0), p0, C.c_void_p(I1), p1, W, H, C.c_void_p(u),
                             C.c_void_p(v), fp, None, None)

    def batch(n=2, p0=w, s0=w * h, s1=w * h, fs=4 * w * h, W=w, H=h):
        return lib.tvl1_calc_batch(ctx, n, C.c_void_p(i0), p0, s0, C.c_void_p(i0), w, s1, W, H,
                                   C.c_void_p(f0), C.c_void_p(g0), 4 * w, fs, None, None)

    cases = [
        (lambda: calc(I0=0), EINVAL, "null"), (lambda: calc(u=0), EINVAL, "null"),
        (lambda: calc(W=0), ESIZE, "bad size"), (lambda: calc(H=-3), ESIZE, "bad size"),
        (lambda: calc(W=1 << 16, H=1 << 16), ESIZE, "too large"),
        (lambda: calc(p0=w - 1), EINVAL, "pitch"), (lambda: calc(fp=4 * w - 4), EINVAL, "pitch"),
        (lambda: calc(fp=4 * w + 2), EINVAL, "pitch"),
        (lambda: lib.tvl1_calc_f32(ctx, C.c_void_p(f0), 4 * w - 4, C.c_void_p(f0), 4 * w, w, h,
                                   C.c_void_p(f0), C.c_void_p(g0), 4 * w, None, None),
         EINVAL, "pitch"),
        (lambda: batch(n=0), EINVAL, "batch size"), (lambda: batch(n=-1), EINVAL, "batch size"),
        (lambda: batch(s0=w * h - 1), EINVAL, "stride"),
        (lambda: batch(fs=4 * w * h - 4), EINVAL, "stride"),
    ]
    for call, want, msg in cases:
        rc = call()   # the message is the ctx's last error, so read it right after the call
        assert rc == want, (rc, want, msg)
        assert msg in lib.tvl1_last_error(ctx).decode(), msg
    assert batch(s0=0, s1=0) == 0   # stride 0: every pair shares one frame
    torch.cuda.synchronize()
    I0, I1 = synth.gen_pair(w, h, seed=5, z=1)
    u, v, st, wi = eng.calc_host(I0, I1)
    eng.close()
    ur, vr, sr, wr = checker.oracle_calc(I0, I1, eng.params)
    assert bits_equal(u, ur) and bits_equal(v, vr)
    np.testing.assert_array_equal(wi, wr)
