"""faiss-shaped flat indexes backed by the HIP scan.

Drop-in for the two faiss classes LIRA's query path uses
(utils.py:415-419 builds them, LIRA_smallscale.py:168-171 searches them):

    index = IndexFlatL2(d)        # or IndexFlatIP(d)
    index.add(xb)                 # (n, d) float32, appends
    D, I = index.search(xq, k)    # numpy (nq, k) float32 / int64
    index.ntotal

Inputs may be numpy arrays (as in the reference) or torch tensors; outputs
follow the input kind (numpy in -> numpy out).  Result convention is faiss':
L2 = ascending squared distance, IP = descending inner product, -1 labels
and +-inf distances when the index holds fewer than k vectors.  Distances are
search.cpp's sequential fp32 sums (faiss's BLAS path rounds differently; they
agree to ~1e-6 relative).  Ties order by smaller label.
"""
from __future__ import annotations

import numpy as np
import torch

from .index import PartitionedIndex, normalize_metric


class IndexFlat:
    def __init__(self, d: int, metric: str = "L2", device=None):
        self.d = int(d)
        self.metric = normalize_metric(metric)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self._chunks: list[torch.Tensor] = []
        self._index: PartitionedIndex | None = None
        self.ntotal = 0
        self.is_trained = True

    @property
    def metric_type(self) -> int:
        return 0 if self.metric == "inner_product" else 1  # faiss METRIC_INNER_PRODUCT / METRIC_L2

    def add(self, x) -> None:
        xt = x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
        if xt.dim() != 2 or xt.shape[1] != self.d:
            raise RuntimeError(f"add: expected (n, {self.d}) vectors, got {tuple(xt.shape)}")
        self._chunks.append(xt.to(device=self.device, dtype=torch.float32).contiguous())
        self.ntotal += xt.shape[0]
        self._index = None

    def reset(self) -> None:
        self._chunks.clear()
        self._index = None
        self.ntotal = 0

    def _built(self) -> PartitionedIndex:
        if self._index is None:
            x = torch.cat(self._chunks) if self._chunks else torch.zeros((0, self.d), device=self.device)
            n = x.shape[0]
            idx = PartitionedIndex(self.d, self.metric, self.device.index)
            idx.add_lists(np.array([0, n], dtype=np.int64),
                          torch.arange(n, dtype=torch.int32, device=self.device), x, 1)
            self._index = idx
        return self._index

    def search(self, x, k: int):
        as_numpy = not isinstance(x, torch.Tensor)
        q = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)) if as_numpy else x
        if q.dim() != 2 or q.shape[1] != self.d:
            raise RuntimeError(f"search: expected (nq, {self.d}) queries")
        q = q.to(device=self.device, dtype=torch.float32).contiguous()
        probe = torch.zeros((q.shape[0], 1), dtype=torch.int32, device=self.device)
        D, I, _ = self._built().search(q, probe, int(k), dedup=False)
        if as_numpy:
            return D.cpu().numpy(), I.cpu().numpy()
        return D, I


class IndexFlatL2(IndexFlat):
    def __init__(self, d: int, device=None):
        super().__init__(d, "L2", device)


class IndexFlatIP(IndexFlat):
    def __init__(self, d: int, device=None):
        super().__init__(d, "inner_product", device)
