"""Synthetic inputs of the BASELINE.json shapes.

Gaussian mixture: B centres ~ N(0,1)^d, point = centre[uniform label] +
sigma * N(0,1)^d (sigma = 0.35), fp32.  Uniform "random-float" vectors are
valid for throughput and parity; the mixture is what makes the recall@10 >= 0.95
gate meaningful (nearest-centre partitions have structure).  Partition
assignment = nearest centre, as IVF does after k-means (utils.py:325).
"""
from __future__ import annotations

import numpy as np
import torch

CONFIGS = {
    # name: (N, d, B, nprobe, k, metric, nq)
    "sift1m": (1_000_000, 128, 64, 8, 10, "L2", 10_000),
    "gist1m": (1_000_000, 960, 128, 16, 10, "L2", 1_000),
    "deep10m": (10_000_000, 96, 256, 32, 100, "inner_product", 10_000),
    "bigann100m": (100_000_000, 128, 1024, 32, 10, "L2", 10_000),
}


def mixture_np(n, d, n_centres, seed, sigma=0.35, centres=None):
    rng = np.random.default_rng(seed)
    if centres is None:
        centres = rng.standard_normal((n_centres, d), dtype=np.float32)
    lab = rng.integers(0, n_centres, size=n)
    x = centres[lab] + np.float32(sigma) * rng.standard_normal((n, d), dtype=np.float32)
    return x.astype(np.float32), centres.astype(np.float32), lab


def mixture_torch(n, d, n_centres, seed, device, sigma=0.35, centres=None, chunk=1 << 20):
    """Same distribution, generated on the GPU (torch Philox), in chunks."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    if centres is None:
        centres = torch.randn((n_centres, d), generator=g, device=device, dtype=torch.float32)
    x = torch.empty((n, d), device=device, dtype=torch.float32)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        lab = torch.randint(0, n_centres, (e - s,), generator=g, device=device)
        x[s:e] = centres[lab] + sigma * torch.randn((e - s, d), generator=g, device=device)
    return x, centres


def nearest_centre(x: torch.Tensor, centres: torch.Tensor, chunk=1 << 18) -> torch.Tensor:
    """argmin_c ||x - c||^2 per row (offline assignment; int32)."""
    cn = (centres * centres).sum(1)
    out = torch.empty(x.shape[0], dtype=torch.int32, device=x.device)
    for s in range(0, x.shape[0], chunk):
        xs = x[s:s + chunk]
        dd = cn[None, :] - 2.0 * (xs @ centres.T)
        out[s:s + chunk] = dd.argmin(1).to(torch.int32)
    return out
