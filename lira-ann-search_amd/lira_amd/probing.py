"""The probing model that sits between partition ranking and the scan.

LIRA scores every partition with a two-tower MLP (model_probing.py:5-39):
sigmoid(fc([dist_tower(standardised centroid distances) || vec_tower(query)])).
It is *called* on the query path (search.cpp:430-445) but it is a handful of
small dense layers, so it runs as a PyTorch-ROCm module (hipBLASLt GEMMs), not
a hand-written kernel.  Parameter names match MLP_2_Input, so a state_dict or a
TorchScript file trained by the reference loads unchanged.
"""
from __future__ import annotations

import torch
from torch import nn


def _tower(n_in: int, hidden: int, n_out: int) -> nn.Sequential:
    return nn.Sequential(nn.Linear(n_in, hidden), nn.ReLU(), nn.Linear(hidden, n_out), nn.ReLU())


class MLP_2_Input(nn.Module):  # noqa: N801 - reference class name, kept for drop-in loading
    """input_dim1 = n_bkt (distance features), input_dim2 = d, output_dim = n_bkt."""

    def __init__(self, input_dim1: int, input_dim2: int, output_dim: int):
        super().__init__()
        self.distance_net = _tower(input_dim1, 128, 64)
        self.vector_net = _tower(input_dim2, 128, 64)
        self.fc = nn.Sequential(nn.Linear(128, 128), nn.ReLU(), nn.Linear(128, output_dim), nn.Sigmoid())

    def forward(self, x_dist: torch.Tensor, x_vec: torch.Tensor) -> torch.Tensor:
        return self.fc(torch.cat((self.distance_net(x_dist), self.vector_net(x_vec)), dim=1))


class NearestCentroidProbe(nn.Module):
    """Scores 1.0 for the nprobe smallest distance features, else 0.0.

    With scaler mean 0 / scale 1 and a threshold in (0, 1], the threshold probe
    of search.cpp:447-466 then selects exactly the IVF nprobe nearest centroids
    (the oracle construction of SURVEY.md 8(c)).  Ties at the boundary score 1.
    """

    def __init__(self, nprobe: int):
        super().__init__()
        self.nprobe = nprobe

    def forward(self, x_dist: torch.Tensor, x_vec: torch.Tensor) -> torch.Tensor:
        kth = torch.topk(x_dist, self.nprobe, dim=1, largest=False).values[:, -1:]
        return (x_dist <= kth).float()


@torch.no_grad()
def probe_scores(model, dist_scaled: torch.Tensor, q: torch.Tensor, batch: int = 65536) -> torch.Tensor:
    """Model scores (n, n_bkt) for a whole query batch (model_infer, model_probing.py:135-156)."""
    outs = [model(dist_scaled[s:s + batch], q[s:s + batch]) for s in range(0, q.shape[0], batch)]
    return torch.cat(outs).float() if outs else torch.zeros((0, dist_scaled.shape[1]), device=q.device)


def standard_scaler(dist: torch.Tensor):
    """sklearn StandardScaler.fit over (n, B) distances, as utils.py:139-142 /
    166-178 save it for search.cpp: per-bucket mean and population std, a zero
    std replaced by 1 (search.cpp:247 does the same at use)."""
    d = dist.double()
    mean = d.mean(0)
    std = d.std(0, unbiased=False)
    std = torch.where(std == 0, torch.ones_like(std), std)
    return mean.float(), std.float()


def fit_probe_to_nearest(model: nn.Module, dist_scaled_fn, nprobe: int, steps: int = 300, batch: int = 4096,
                         lr: float = 2e-3, seed: int = 0) -> nn.Module:
    """Train MLP_2_Input to score each query's nprobe nearest centroids 1 and
    the rest 0 (BCE, Adam), from batches dist_scaled_fn(batch, step) ->
    (standardised distances (n, B), queries (n, d)).

    A synthetic stand-in for LIRA's training on kNN partition labels
    (model_probing.py:41-54, LIRA_smallscale.py:308-329; training is outside
    the query-time hot path), so that the MLP-probed pipeline selects a
    realistic number of partitions at threshold 0.5 instead of a random-init
    model's arbitrary ones.
    """
    torch.manual_seed(seed)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    lossf = nn.BCELoss()
    model.train()
    for it in range(steps):
        xd, xq = dist_scaled_fn(batch, it)
        kth = torch.topk(xd, nprobe, dim=1, largest=False).values[:, -1:]
        target = (xd <= kth).float()
        opt.zero_grad(set_to_none=True)
        loss = lossf(model(xd, xq), target)
        loss.backward()
        opt.step()
    model.eval()
    return model
