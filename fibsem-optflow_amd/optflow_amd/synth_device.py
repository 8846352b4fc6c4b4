"""Synthetic FIB-SEM-like slices generated on the GPU ("Inputs are
generated on device so I/O is excluded").

Same recipe as synth.py: a base texture of uniform noise, Gaussian-blurred (sigma = 2
px) and stretched to [16, 240]; slice z is the base advected by the known smooth
displacement d_z(x, y) = (a sin(2 pi y / P) + dx_z, a cos(2 pi x / P) + dy_z) (a = 1.5 px,
P = 512 px, per-slice drift from synth.displacement's generator), plus N(0, 2) grey
noise, rounded to u8.  Built with torch on the device (PyTorch is plumbing here: the
slices are inputs to the HIP engine, not part of the measured path); values are not
bit-identical to synth.py's scipy version, only the same distribution.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as Fn


class DeviceStack:
    def __init__(self, W: int, H: int, device, seed: int = 0x5EED, a: float = 1.5,
                 P: float = 512.0, noise: float = 2.0, zero_band_every: int = 0):
        self.W, self.H, self.dev = W, H, torch.device(device)
        self.seed, self.a, self.P, self.noise = seed, a, P, noise
        self.zero_band_every = zero_band_every
        g = torch.Generator(device=self.dev)
        g.manual_seed(seed)
        n = torch.rand((1, 1, H, W), generator=g, device=self.dev)
        r = 8
        t = torch.arange(-r, r + 1, device=self.dev, dtype=torch.float32)
        k = torch.exp(-0.5 * (t / 2.0) ** 2)
        k = k / k.sum()
        b = Fn.conv2d(Fn.pad(n, (r, r, 0, 0), mode="reflect"), k.view(1, 1, 1, -1))
        b = Fn.conv2d(Fn.pad(b, (0, 0, r, r), mode="reflect"), k.view(1, 1, -1, 1))
        lo, hi = b.min(), b.max()
        self.base = 16.0 + (b - lo) * (224.0 / torch.clamp(hi - lo, min=1e-12))
        ys = torch.arange(H, device=self.dev, dtype=torch.float32)
        xs = torch.arange(W, device=self.dev, dtype=torch.float32)
        self.ys, self.xs = ys.view(H, 1), xs.view(1, W)

    def slice(self, z: int) -> torch.Tensor:
        """Slice z as a (H, W) uint8 device tensor."""
        rng = np.random.default_rng((self.seed ^ z) + 1)
        ddx, ddy = rng.uniform(-0.5, 0.5, size=2)
        amp = self.a if z != 0 else 0.0
        if z == 0:
            ddx = ddy = 0.0
        dx = amp * torch.sin(2 * math.pi * self.ys / self.P) + float(ddx)   # (H, 1)
        dy = amp * torch.cos(2 * math.pi * self.xs / self.P) + float(ddy)   # (1, W)
        sx = (self.xs - dx).expand(self.H, self.W)
        sy = (self.ys - dy).expand(self.H, self.W)
        grid = torch.stack((2.0 * sx / (self.W - 1) - 1.0, 2.0 * sy / (self.H - 1) - 1.0), dim=-1)
        w = Fn.grid_sample(self.base, grid[None], mode="bilinear", padding_mode="border",
                           align_corners=True)[0, 0]
        if self.noise > 0:
            g = torch.Generator(device=self.dev)
            g.manual_seed((self.seed ^ z) + 7)
            w = w + self.noise * torch.randn((self.H, self.W), generator=g, device=self.dev)
        out = torch.clamp(torch.round(w), 0, 255).to(torch.uint8)
        if self.zero_band_every and z % self.zero_band_every == self.zero_band_every - 1:
            out[:, :32] = 0
        return out
