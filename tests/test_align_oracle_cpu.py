"""Known-answer tests of the alignment restatement (oracle/tvl1_oracle_align.c) on CPU,
before tests/test_align_gpu.py holds the GPU path to it bit for bit: an exact homography
from exact correspondences, outliers rejected, the identity warp, the 2-NN tie rule, the
keypoint budget, and a known shift recovered end to end (features.cpp:46-167)."""
import numpy as np
import pytest

from optflow_amd import synth
from oracle import checker


def test_find_homography_exact_and_outliers(built):
    rng = np.random.default_rng(1)
    H = np.array([[1.02, 0.03, 5.0], [-0.01, 0.98, -3.0], [1e-5, -2e-5, 1.0]])
    src = rng.uniform(0, 500, (60, 2))
    p = np.c_[src, np.ones(60)] @ H.T
    dst = p[:, :2] / p[:, 2:]
    for method in (8, 4, 0):
        ok, Hr, mask = checker.oracle_find_homography(src, dst, method)
        assert ok and np.allclose(Hr, H, atol=1e-7) and mask.all(), (method, Hr)
    dst2 = dst.copy()
    dst2[:12] += rng.uniform(30, 60, (12, 2))      # 20 % outliers
    for method in (8, 4):
        ok, Hr, mask = checker.oracle_find_homography(src, dst2, method)
        assert ok and np.allclose(Hr, H, atol=1e-6) and not mask[:12].any() and mask[12:].all()


def test_warp_identity_and_shift(built):
    rng = np.random.default_rng(2)
    src = rng.integers(0, 256, (31, 47), dtype=np.uint8)
    assert np.array_equal(checker.oracle_warp_affine_u8(src, 47, 31, [[1, 0, 0], [0, 1, 0]]), src)
    # dst(x) = src(x - 3): integer shift, zeros where the source is outside
    out = checker.oracle_warp_affine_u8(src, 47, 31, [[1, 0, 3], [0, 1, 0]])
    assert np.array_equal(out[:, 3:], src[:, :-3]) and np.all(out[:, :3] == 0)
    # half-pixel shift of a constant: interior constant, border column half weight
    c = np.full((10, 10), 100, np.uint8)
    out = checker.oracle_warp_affine_u8(c, 10, 10, [[1, 0, 0.5], [0, 1, 0]])
    assert np.all(out[:, 1:] == 100) and np.all(out[:, 0] == 50)


def test_postprocess_affine_identity_is_mask_only(built):
    rng = np.random.default_rng(3)
    u = rng.normal(0, 2, (20, 30)).astype(np.float32)
    v = rng.normal(0, 2, (20, 30)).astype(np.float32)
    I1 = rng.integers(0, 256, (20, 30), dtype=np.uint8)
    I1[5] = 0
    uu, vv = checker.oracle_postprocess_affine(u, v, I1, 1, [[1, 0, 0], [0, 1, 0]])
    xs = np.arange(30, dtype=np.float32)
    ys = np.arange(20, dtype=np.float32)[:, None]
    want_u = (u + xs) - xs
    want_v = (v + ys) - ys
    want_u[I1 <= 1] = 0
    want_v[I1 <= 1] = 0
    assert np.array_equal(uu, want_u) and np.array_equal(vv, want_v)


def test_match_ties_and_budget(built):
    f0 = np.clip(np.rint(synth.base_texture(400, 300, seed=4)), 0, 255).astype(np.uint8)
    kp, d = checker.oracle_orb_detect(f0, nfeatures=500)
    assert 100 < len(kp) <= 500
    assert np.all(np.diff(kp[:, 2]) >= 0)                  # levels in order
    for l in np.unique(kp[:, 2]):                           # best response first per level
        r = kp[kp[:, 2] == l, 4]
        assert np.all(np.diff(r) <= 0)
    idx, dist = checker.oracle_match_knn2(d[:10], np.concatenate([d[:10], d[:10]]))
    assert np.array_equal(idx[:, 0], np.arange(10)) and np.array_equal(idx[:, 1], np.arange(10) + 10)


@pytest.mark.parametrize("method", [8, 4])
def test_find_alignment_recovers_shift(built, method):
    from scipy import ndimage
    f0 = np.clip(np.rint(synth.base_texture(640, 480, seed=77)), 0, 255).astype(np.uint8)
    ys, xs = np.mgrid[0:480, 0:640].astype(np.float64)
    f1 = np.clip(np.rint(ndimage.map_coordinates(f0.astype(float), [ys - 6.4, xs + 11.2], order=1,
                                                 cval=0)), 0, 255).astype(np.uint8)
    A, ng, oc = checker.oracle_find_alignment(f1, f0, method=method)
    assert oc == 0 and ng > 10
    assert abs(A[0, 2] - 11.2) < 0.5 and abs(A[1, 2] + 6.4) < 0.5, A
    A2, ng2, oc2 = checker.oracle_find_alignment(f1, f0, method=method)
    assert np.array_equal(A, A2) and ng == ng2   # deterministic
