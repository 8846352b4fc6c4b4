"""Feature pre-alignment (features.cpp:46-167): tvl1_find_alignment must
recover known affine motions between synthetic slices, and tvl1_warp_affine_u8 must follow
cv::cuda::warpAffine's definition (dst(x) = src(M^-1 x), bilinear, BORDER_CONSTANT 0).
PARITY UNPINNED against OpenCV's ORB / findHomography (absent here): these are
known-answer tests of the contract (tvl1_align.hpp header)."""
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


def test_warp_affine_u8_definition(built):
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, (40, 50), dtype=np.uint8)
    M = np.array([[0.98, 0.05, 3.25], [-0.04, 1.01, -2.5]], np.float32)
    eng = capi.Engine(capi.make_params())
    ds = torch.from_numpy(src).to("cuda")
    dd = torch.zeros((45, 55), dtype=torch.uint8, device="cuda")
    eng.warp_affine_u8(ds.data_ptr(), 50, 50, 40, dd.data_ptr(), 55, 55, 45, M)
    torch.cuda.synchronize()
    out = dd.cpu().numpy().astype(int)
    eng.close()
    # reference: inverse map in double, bilinear with zero outside
    a, b, c, d, e, f = [float(x) for x in M.ravel()]
    D = 1.0 / (a * e - b * d)
    iM = np.array([[e * D, -b * D, 0], [-d * D, a * D, 0]])
    iM[0, 2] = -iM[0, 0] * c - iM[0, 1] * f
    iM[1, 2] = -iM[1, 0] * c - iM[1, 1] * f
    ys, xs = np.mgrid[0:45, 0:55].astype(np.float64)
    X = iM[0, 0] * xs + iM[0, 1] * ys + iM[0, 2]
    Y = iM[1, 0] * xs + iM[1, 1] * ys + iM[1, 2]
    x1, y1 = np.floor(X).astype(int), np.floor(Y).astype(int)
    def at(yy, xx):
        ok = (xx >= 0) & (yy >= 0) & (xx < 50) & (yy < 40)
        return np.where(ok, src[np.clip(yy, 0, 39), np.clip(xx, 0, 49)], 0).astype(float)
    fx, fy = X - x1, Y - y1
    ref = (at(y1, x1) * (1 - fx) * (1 - fy) + at(y1, x1 + 1) * fx * (1 - fy) +
           at(y1 + 1, x1) * (1 - fx) * fy + at(y1 + 1, x1 + 1) * fx * fy)
    assert np.abs(out - np.clip(np.rint(ref), 0, 255)).max() <= 1


@pytest.mark.parametrize("flow_output", [0, 1])
def test_postprocess_affine_definition(built, flow_output):
    """solve_wrapper's features branch (optflow.cpp:411-443, 468-473): map = flow + grid,
    map' = warpAffine(map, M) (bilinear, BORDER_CONSTANT 0), flow = map' - grid for
    output "flow" (else map'), then 0 wherever I1 <= 1."""
    import ctypes as C
    H, W = 30, 40
    rng = np.random.default_rng(9)
    u = rng.normal(0, 1.5, (H, W)).astype(np.float32)
    v = rng.normal(0, 1.5, (H, W)).astype(np.float32)
    I1 = rng.integers(0, 256, (H, W), dtype=np.uint8)
    I1[:3, :] = 1                      # masked rows
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
    gu, gv = du.cpu().numpy(), dv.cpu().numpy()
    eng.close()
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float64)
    a, b, c, d, e, f = [float(x) for x in M.ravel()]
    D = 1.0 / (a * e - b * d)
    i00, i01, i10, i11 = e * D, -b * D, -d * D, a * D
    X = i00 * xs + i01 * ys + (-i00 * c - i01 * f)
    Y = i10 * xs + i11 * ys + (-i10 * c - i11 * f)
    x1, y1 = np.floor(X).astype(int), np.floor(Y).astype(int)
    fx, fy = X - x1, Y - y1

    def warp(m):
        def at(yy, xx):
            ok = (xx >= 0) & (yy >= 0) & (xx < W) & (yy < H)
            return np.where(ok, m[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)], 0.0)
        return (at(y1, x1) * (1 - fx) * (1 - fy) + at(y1, x1 + 1) * fx * (1 - fy) +
                at(y1 + 1, x1) * (1 - fx) * fy + at(y1 + 1, x1 + 1) * fx * fy)

    ru, rv = warp(u + xs), warp(v + ys)
    if flow_output:
        ru, rv = ru - xs, rv - ys
    ru[I1 <= 1] = 0
    rv[I1 <= 1] = 0
    assert np.abs(gu - ru).max() < 2e-3 and np.abs(gv - rv).max() < 2e-3


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
