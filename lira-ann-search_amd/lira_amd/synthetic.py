"""Synthetic inputs of the BASELINE.json shapes.

Two distributions, both fp32:

* ``latent``: x = z A + 0.1 * N(0,1)^d with z ~ N(0,1)^m,
  A a fixed random m x d basis / sqrt(m) -- full-rank vectors of low intrinsic
  dimension m, like real descriptors.  Partitions come from k-means over the
  data (``lira_amd.knn.Kmeans``, as utils.py:321-330 does with faiss), so their
  Voronoi cells cut through a continuum and a query's neighbours often sit in
  the adjacent cells.  m is chosen per config so that recall@k at the config's
  nprobe (nearest centroids) lands near the metric's 0.95 operating point
  (measured: SIFT1M m=12 -> 0.97, GIST1M m=16 -> 0.96, DEEP10M m=20 -> 0.985),
  as it does on the real datasets.  deep10m rows are L2-normalised (DEEP1B is).
* ``uniform``: x ~ U[0, 1)^d i.i.d. (north_star's literal "synthetic random-float
  vectors"), k-means partitions like ``latent``.  No cluster structure: recall@k at
  nprobe << B is low against global ground truth (hard part 7), so
  it is a throughput and parity workload -- both sides scan identical probe lists.
* ``mixture``: B centres ~ N(0,1)^d, point = centre[uniform label] +
  sigma * N(0,1)^d (sigma = 0.35), nearest-centre partitions.  In high d these
  clusters are perfectly separated (recall 1.0 at any nprobe >= 1), so exact
  pruning skips nearly every non-nearest partition: an easy best case.  It is
  SURVEY.md 8(d)'s prescribed distribution, so bench.py's headline uses it
  and reports the ``latent`` run beside it (``contrast_data``).
"""
from __future__ import annotations

import numpy as np
import torch

CONFIGS = {
    # name: (N, d, B, nprobe, k, metric, nq)  (BASELINE.json configs)
    "sift1m": (1_000_000, 128, 64, 8, 10, "L2", 10_000),
    "gist1m": (1_000_000, 960, 128, 16, 10, "L2", 1_000),
    "deep10m": (10_000_000, 96, 256, 32, 100, "inner_product", 10_000),
    "bigann100m": (100_000_000, 128, 1024, 32, 10, "L2", 10_000),
}
# buckets per base row: LIRA_largescale.py's full redundancy (n_mul = 2,
# LIRA_largescale.py:37-39) for the BIGANN-100M path, here each row's n_mul
# nearest centroids; 1 (plain partitions) elsewhere
N_MUL = {"bigann100m": 2}
# intrinsic dimension of the ``latent`` distribution per config (see above)
LATENT_DIM = {"sift1m": 12, "gist1m": 16, "deep10m": 20, "bigann100m": 12}
NORMALISED = {"deep10m"}


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


def uniform_torch(n, d, seed, device, chunk=1 << 20):
    """n rows of U[0, 1)^d (torch Philox on ``device``), in chunks."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.empty((n, d), device=device, dtype=torch.float32)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        x[s:e] = torch.rand((e - s, d), generator=g, device=device)
    return x


def nearest_centre(x: torch.Tensor, centres: torch.Tensor, chunk=1 << 18) -> torch.Tensor:
    """argmin_c ||x - c||^2 per row (offline assignment; int32)."""
    cn = (centres * centres).sum(1)
    out = torch.empty(x.shape[0], dtype=torch.int32, device=x.device)
    for s in range(0, x.shape[0], chunk):
        xs = x[s:s + chunk]
        dd = cn[None, :] - 2.0 * (xs @ centres.T)
        out[s:s + chunk] = dd.argmin(1).to(torch.int32)
    return out


def latent_basis(d: int, m: int, seed: int, device) -> torch.Tensor:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return torch.randn((m, d), generator=g, device=device, dtype=torch.float32) / m ** 0.5


def latent_torch(n, basis, seed, device, noise=0.1, normalise=False, chunk=1 << 20):
    """n rows of z @ basis + noise * N(0,1)^d (torch Philox on ``device``)."""
    m, d = basis.shape
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.empty((n, d), device=device, dtype=torch.float32)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        xs = torch.randn((e - s, m), generator=g, device=device) @ basis
        xs += noise * torch.randn((e - s, d), generator=g, device=device)
        if normalise:
            xs /= xs.norm(dim=1, keepdim=True)
        x[s:e] = xs
    return x


def nearest_m(x: torch.Tensor, centres: torch.Tensor, m: int, chunk=1 << 20) -> torch.Tensor:
    """(N, m) int32: each row's m nearest centres by search.cpp's exact distance
    (lira_rank_nearest; ties -> smaller id) -- the data_2_bkt of n_mul = m."""
    from .index import RankWorkspace, rank_nearest
    out = torch.empty((x.shape[0], m), dtype=torch.int32, device=x.device)
    ws = RankWorkspace(min(chunk, x.shape[0]), centres.shape[0], x.device)
    for s in range(0, x.shape[0], chunk):
        rank_nearest(x[s:s + chunk], centres, m, out=out[s:s + chunk], workspace=ws)
    return out


def workload(config: str, seed: int, device, data: str = "latent", n_override=None, kmeans_iter: int = 10):
    """(x, centroids, assignment, make_queries(nq, seed)) for a config.

    assignment: (N,) int32, or (N, n_mul) for the configs of N_MUL.
    ``latent`` / ``uniform``: k-means centroids (lira_amd.knn.Kmeans, subsample of
    256 points per centroid as faiss) and exact nearest-centroid assignment.
    ``mixture``: generating centres and nearest-centre assignment."""
    N, d, B, _, _, _, _ = CONFIGS[config]
    N = n_override or N
    n_mul = N_MUL.get(config, 1)
    if data == "mixture":
        x, c = mixture_torch(N, d, B, seed, device)
        assign = nearest_centre(x, c) if n_mul == 1 else nearest_m(x, c, n_mul)
        return x, c, assign, lambda nq, s: mixture_torch(nq, d, B, s, device, centres=c)[0]
    if data not in ("latent", "uniform"):
        raise ValueError(f"unknown synthetic distribution {data!r}")
    from .knn import Kmeans
    if data == "uniform":
        x = uniform_torch(N, d, seed + 1, device)
        make_q = lambda nq, s: uniform_torch(nq, d, s, device)  # noqa: E731
    else:
        basis = latent_basis(d, LATENT_DIM[config], seed, device)
        norm = config in NORMALISED
        x = latent_torch(N, basis, seed + 1, device, normalise=norm)
        make_q = lambda nq, s: latent_torch(nq, basis, s, device, normalise=norm)  # noqa: E731
    km = Kmeans(d, B, niter=kmeans_iter, seed=seed, device=device.index)
    km.train(x)
    c = torch.from_numpy(km.centroids).to(device)
    assign = nearest_m(x, c, n_mul)
    if n_mul == 1:
        assign = assign[:, 0]
    return x, c, assign, make_q
