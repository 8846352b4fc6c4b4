"""Feature pre-alignment (features.cpp:46-167): tvl1_find_alignment must
recover known affine motions between synthetic slices (property tests), and every stage --
ORB keypoints and descriptors, the 2-NN match list, the fitted affine, and the warps of
frame1 and of the map fields (cv::cuda::warpAffine, optflow.cpp:370, 429-443) -- is
bit-identical to its CPU restatement (oracle/tvl1_oracle_align.c).  PARITY UNPINNED against
OpenCV's ORB / findHomography (absent here; tvl1_align.hpp header)."""
import numpy as np
import pytest

from optflow_amd import capi, synth

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def warped(f0, M):
    """f1 with f1(p) = f0(M p): frame1 coordinates p map onto frame0 by M (2x3)."""
    from scipy import ndimage
    h, w = f0.shape
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float64)
    X = M[0, 0] * xs + M[0, 1] * ys + M[0, 2]
    Y = M[1, 0] * xs + M[1, 1] * ys + M[1, 2]
    return np.clip(np.rint(ndimage.map_coordinates(f0.astype(np.float64), [Y, X], order=1,
                                                   cval=0.0)), 0, 255).astype(np.uint8)


def rot(deg, tx, ty, s=1.0):
    a = np.deg2rad(deg)
    return np.array([[s * np.cos(a), -s * np.sin(a), tx], [s * np.sin(a), s * np.cos(a), ty]])


@pytest.mark.parametrize("M", [rot(0, 12.3, -7.8), rot(1.5, -20.0, 15.0), rot(-3.0, 5.5, 9.0, 1.03)],
                         ids=["shift", "rot1.5", "rot-3_zoom"])
@pytest.mark.parametrize("method", [8, 4])
def test_alignment_recovers_affine(built, M, method):
    h, w = 600, 800
    f0 = np.clip(np.rint(synth.base_texture(w, h, seed=77)), 0, 255).astype(np.uint8)
    f1 = warped(f0, M)
    eng = capi.Engine(capi.make_params())
    dev = torch.device("cuda", 0)
    d0 = torch.from_numpy(f0).to(dev)
    d1 = torch.from_numpy(f1).to(dev)
    torch.cuda.synchronize()
    A, ng, oc = eng.find_alignment(d1.data_ptr(), w, w, h, d0.data_ptr(), w, w, h, method=method)
    eng.close()
    assert oc == 0 and ng > 10, (oc, ng)
    corners = np.array([[50, 50, 1], [w - 50, 50, 1], [50, h - 50, 1], [w - 50, h - 50, 1]], float)
    err = np.abs(corners @ A.T.astype(float) - corners @ M.T).max()
    assert err < 1.5, (A, M, err)   # px at the corners (the homography's top 2x3)


def test_alignment_without_texture_is_identity(built):
    f0 = np.full((300, 300), 120, np.uint8)
    eng = capi.Engine(capi.make_params())
    d0 = torch.from_numpy(f0).to("cuda")
    A, ng, oc = eng.find_alignment(d0.data_ptr(), 300, 300, 300, d0.data_ptr(), 300, 300, 300)
    eng.close()
    assert oc == 1 and ng <= 10
    assert np.array_equal(A, np.array([[1, 0, 0], [0, 1, 0]], np.float32))


def test_alignment_blur_and_small_feature_budget(built):
    """blurForDescriptor (ORB's Gaussian before the descriptors), a single pyramid level and
    a small nfeatures budget still recover a shift."""
    h, w = 480, 640
    f0 = np.clip(np.rint(synth.base_texture(w, h, seed=21)), 0, 255).astype(np.uint8)
    M = rot(0.5, 9.0, -4.0)
    f1 = warped(f0, M)
    eng = capi.Engine(capi.make_params())
    d0 = torch.from_numpy(f0).cuda()
    d1 = torch.from_numpy(f1).cuda()
    torch.cuda.synchronize()
    for kw in ({"blur_for_descriptor": 1}, {"nlevels": 1, "nfeatures": 400}):
        A, ng, oc = eng.find_alignment(d1.data_ptr(), w, w, h, d0.data_ptr(), w, w, h, **kw)
        assert oc == 0 and ng > 10, (kw, oc, ng)
        corners = np.array([[40, 40, 1], [w - 40, 40, 1], [40, h - 40, 1], [w - 40, h - 40, 1]], float)
        assert np.abs(corners @ A.T.astype(float) - corners @ M.T).max() < 1.5, (kw, A)
    eng.close()


def test_alignment_is_deterministic(built):
    h, w = 400, 520
    f0 = np.clip(np.rint(synth.base_texture(w, h, seed=8)), 0, 255).astype(np.uint8)
    f1 = warped(f0, rot(-1.0, 3.0, 6.0))
    eng = capi.Engine(capi.make_params())
    d0 = torch.from_numpy(f0).cuda()
    d1 = torch.from_numpy(f1).cuda()
    torch.cuda.synchronize()
    runs = [eng.find_alignment(d1.data_ptr(), w, w, h, d0.data_ptr(), w, w, h, method=m)
            for m in (8, 8, 4, 4)]
    eng.close()
    assert np.array_equal(runs[0][0], runs[1][0]) and runs[0][1] == runs[1][1]
    assert np.array_equal(runs[2][0], runs[3][0]) and runs[2][1] == runs[3][1]


# ---- bit-for-bit against the restatement of this pipeline (oracle/tvl1_oracle_align.c):
# VERDICT r2 "next" item 4.  Parity with OpenCV's ORB / SURF / findHomography stays unpinned
# (OpenCV is absent; the rBRIEF pattern is a stand-in), so the bar here is the build's own
# stated definition, exactly.
from oracle import checker   # noqa: E402  (the checker only)

ALIGN_CASES = [
    ("shift", rot(0, 12.3, -7.8), dict()),
    ("rot1.5", rot(1.5, -20.0, 15.0), dict(method=4)),
    ("zoom_blur", rot(-3.0, 5.5, 9.0, 1.03), dict(blur_for_descriptor=1)),
    ("small_budget", rot(0.5, 9.0, -4.0), dict(nlevels=3, nfeatures=700, fast_threshold=12)),
]


def frames(M, w=640, h=480, seed=77):
    f0 = np.clip(np.rint(synth.base_texture(w, h, seed=seed)), 0, 255).astype(np.uint8)
    return f0, warped(f0, M)


@pytest.mark.parametrize("name,M,kw", ALIGN_CASES, ids=[c[0] for c in ALIGN_CASES])
def test_orb_detect_bitwise(built, name, M, kw):
    """Keypoints (level-0 x, y, octave, Harris response) and rBRIEF descriptors."""
    f0, f1 = frames(M)
    eng = capi.Engine(capi.make_params())
    for f in (f0, f1):
        d = torch.from_numpy(f).cuda()
        torch.cuda.synchronize()
        kp, desc = eng.orb_detect(d.data_ptr(), f.shape[1], f.shape[1], f.shape[0], **kw)
        kr, dr = checker.oracle_orb_detect(f, **kw)
        assert len(kp) == len(kr) > 100, (len(kp), len(kr))
        cols = [0, 1, 2, 4]
        assert np.array_equal(kp[:, cols].view(np.uint32), kr[:, cols].view(np.uint32))
        assert np.array_equal(desc, dr)
        assert np.all((kp[:, 3] >= 0) & (kp[:, 3] < 360))   # angles (degrees) reported
    eng.close()


@pytest.mark.parametrize("name,M,kw", ALIGN_CASES[:2], ids=[c[0] for c in ALIGN_CASES[:2]])
def test_match_knn2_bitwise(built, name, M, kw):
    """Hamming 2-NN match list (indices and distances, ties to the lower index)."""
    f0, f1 = frames(M)
    _, d1 = checker.oracle_orb_detect(f1, **kw)
    _, d0 = checker.oracle_orb_detect(f0, **kw)
    eng = capi.Engine(capi.make_params())
    idx, dist = eng.match_knn2(d1, d0)
    ir, dr = checker.oracle_match_knn2(d1, d0)
    assert np.array_equal(idx, ir) and np.array_equal(dist, dr)
    # duplicated train descriptors: the tie goes to the lower index
    d0d = np.concatenate([d0[:50], d0[:50]])
    idx, dist = eng.match_knn2(d0[:20], d0d)
    assert np.array_equal(idx[:, 0], np.arange(20)) and np.array_equal(idx[:, 1], np.arange(20) + 50)
    assert np.all(dist == 0)
    idx, dist = eng.match_knn2(d0[:5], d0[:1])   # one train descriptor: no second neighbour
    assert np.all(idx[:, 1] == -1) and np.all(idx[:, 0] == 0)
    eng.close()


@pytest.mark.parametrize("name,M,kw", ALIGN_CASES, ids=[c[0] for c in ALIGN_CASES])
def test_find_alignment_bitwise(built, name, M, kw):
    """The whole find_alignment: ratio test over the reference's loop bound, distance sort,
    RANSAC / LMEDS + LM fit, zoom check -- the same affine bits, good-match count and
    outcome as the restatement."""
    f0, f1 = frames(M)
    eng = capi.Engine(capi.make_params())
    d0 = torch.from_numpy(f0).cuda()
    d1 = torch.from_numpy(f1).cuda()
    torch.cuda.synchronize()
    h, w = f0.shape
    A, ng, oc = eng.find_alignment(d1.data_ptr(), w, w, h, d0.data_ptr(), w, w, h, **kw)
    eng.close()
    Ar, ngr, ocr = checker.oracle_find_alignment(f1, f0, **kw)
    assert (ng, oc) == (ngr, ocr) and oc == 0
    assert np.array_equal(A.view(np.uint32), Ar.view(np.uint32)), (A, Ar)


def test_warp_affine_u8_bitwise(built):
    """cv::cuda::warpAffine(INTER_LINEAR, BORDER_CONSTANT 0) on u8: float inverse map,
    LinearFilter taps, saturate_cast (round half to even) -- bit for bit."""
    rng = np.random.default_rng(5)
    eng = capi.Engine(capi.make_params())
    for (sh, sw, dh, dw, M) in [(40, 50, 45, 55, [[0.98, 0.05, 3.25], [-0.04, 1.01, -2.5]]),
                                (301, 257, 300, 260, [[1.0, 0.0, 0.5], [0.0, 1.0, -0.5]]),
                                (128, 96, 128, 96, rot(2.0, 4.0, -3.0, 0.97))]:
        src = rng.integers(0, 256, (sh, sw), dtype=np.uint8)
        M = np.asarray(M, np.float32)
        ds = torch.from_numpy(src).cuda()
        dd = torch.zeros((dh, dw), dtype=torch.uint8, device="cuda")
        eng.warp_affine_u8(ds.data_ptr(), sw, sw, sh, dd.data_ptr(), dw, dw, dh, M)
        torch.cuda.synchronize()
        assert np.array_equal(dd.cpu().numpy(), checker.oracle_warp_affine_u8(src, dw, dh, M))
    eng.close()


@pytest.mark.parametrize("flow_output", [0, 1])
def test_postprocess_affine_bitwise(built, flow_output):
    import ctypes as C
    H, W = 57, 83
    rng = np.random.default_rng(19)
    u = rng.normal(0, 1.5, (H, W)).astype(np.float32)
    v = rng.normal(0, 1.5, (H, W)).astype(np.float32)
    I1 = rng.integers(0, 256, (H, W), dtype=np.uint8)
    I1[:3, :] = 1
    M = np.array([[1.01, 0.02, 1.75], [-0.015, 0.99, -0.5]], np.float32)
    eng = capi.Engine(capi.make_params())
    du, dv = torch.from_numpy(u).cuda(), torch.from_numpy(v).cuda()
    dI = torch.from_numpy(I1).cuda()
    aff = (C.c_float * 6)(*[float(x) for x in M.ravel()])
    rc = eng.lib.tvl1_postprocess_affine(eng.ctx, C.c_void_p(du.data_ptr()), C.c_void_p(dv.data_ptr()),
                                         4 * W, C.c_void_p(dI.data_ptr()), W, W, H, flow_output,
                                         aff, None)
    assert rc == 0
    torch.cuda.synchronize()
    ur, vr = checker.oracle_postprocess_affine(u, v, I1, flow_output, M)
    assert np.array_equal(du.cpu().numpy().view(np.uint32), ur.view(np.uint32))
    assert np.array_equal(dv.cpu().numpy().view(np.uint32), vr.view(np.uint32))
    eng.close()
