"""Synthetic FIB-SEM-like slice stacks (SURVEY.md 8(d) "Synthetic inputs").

gen_stack(W, H, Z, seed): a base texture of uniform noise, Gaussian-blurred
(sigma = 2 px) and stretched to u8 [16, 240]; slice z is the base advected by a
smooth known displacement
    d_z(x, y) = (a sin(2 pi y / P) + dx_z,  a cos(2 pi x / P) + dy_z)
with a = 1.5 px, P = 512 px, per-slice drift d ~ U(-0.5, 0.5) px, plus N(0, 2)
grey noise.  Optionally a 32-px zero band exercises the I1 <= 1 output mask
(optflow.cpp:467-473).  Deterministic for a given seed (numpy PCG64).
"""
from __future__ import annotations

import numpy as np
from scipy import ndimage


def base_texture(W: int, H: int, seed: int = 0x5EED) -> np.ndarray:
    rng = np.random.default_rng(seed)
    n = rng.random((H, W), dtype=np.float32)
    b = ndimage.gaussian_filter(n, sigma=2.0, mode="reflect")
    lo, hi = float(b.min()), float(b.max())
    return (16.0 + (b - lo) * (224.0 / max(hi - lo, 1e-12))).astype(np.float32)


def displacement(W: int, H: int, z: int, seed: int = 0x5EED, a: float = 1.5,
                 P: float = 512.0):
    """Known displacement field of slice z (float32 dx, dy)."""
    rng = np.random.default_rng((seed ^ z) + 1)
    ddx, ddy = rng.uniform(-0.5, 0.5, size=2)
    if z == 0:
        ddx = ddy = 0.0
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float32)
    amp = a if z != 0 else 0.0
    dx = amp * np.sin(2 * np.pi * ys / P) + ddx
    dy = amp * np.cos(2 * np.pi * xs / P) + ddy
    return dx.astype(np.float32), dy.astype(np.float32)


def make_slice(base: np.ndarray, z: int, seed: int = 0x5EED, noise: float = 2.0,
               zero_band: bool = False) -> np.ndarray:
    H, W = base.shape
    dx, dy = displacement(W, H, z, seed)
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float32)
    # slice z samples the base at (x - d, y - d): frame z = base advected by d_z
    warped = ndimage.map_coordinates(base, [ys - dy, xs - dx], order=1, mode="nearest")
    rng = np.random.default_rng((seed ^ z) + 7)
    if noise > 0:
        warped = warped + rng.normal(0.0, noise, size=warped.shape).astype(np.float32)
    out = np.clip(np.rint(warped), 0, 255).astype(np.uint8)
    if zero_band:
        out[:, :32] = 0
    return out


def gen_pair(W: int, H: int, seed: int = 0x5EED, z: int = 1, noise: float = 2.0):
    """One slice pair (slice 0 = base + noise, slice z = advected base + noise)."""
    base = base_texture(W, H, seed)
    return make_slice(base, 0, seed, noise), make_slice(base, z, seed, noise)


def gen_stack(W: int, H: int, Z: int, seed: int = 0x5EED, zero_band_every: int = 0):
    base = base_texture(W, H, seed)
    out = np.empty((Z, H, W), np.uint8)
    for z in range(Z):
        zb = bool(zero_band_every) and z % zero_band_every == zero_band_every - 1
        out[z] = make_slice(base, z, seed, zero_band=zb)
    return out
