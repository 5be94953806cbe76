"""Query-sharded multi-GPU search.

Queries are independent, so a batch is split into contiguous slices, one per
rank (one process per GPU, torch.distributed over RCCL -- backend "nccl" on
ROCm).  Every rank holds a full replica of the partitioned index, runs
ranking + scan + top-k on its slice, and the per-rank (D, I) top-k is
all-gathered so every rank (the caller on rank 0 in particular) sees the whole
batch's results.  That all-gather is the path's only exchange step: 12 bytes x
k per query (1.2 MB for 10k queries at k=10), far below xGMI link rates.

Partition sharding (SURVEY.md 8(e)'s alternative for BIGANN's memory): rank r
holds only the lists of the buckets `partition_owners` gives it (balanced by
list size), every rank ranks and scans the WHOLE query batch against its own
lists (a probe into another rank's bucket finds an empty list), and the ranks'
(nq, k) results are all-gathered and k-way merged on the device
(lira_merge_shards).  The lists of different ranks are disjoint, so the merge
of the per-rank exact top-k is the single-index result bit for bit.

The reference has no distributed code (single GPU chosen by
nvidia-smi, utils.py:90-96); this module is new.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous slice [start, end) of n items for `rank` (sizes differ by <= 1)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("need 0 <= rank < world")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def all_gather_rows(t: torch.Tensor, n_total: int, world: int, group=None) -> torch.Tensor:
    """All-gather row slices laid out by shard_bounds into one (n_total, ...) tensor.

    Slices may differ by one row; they are padded to the largest slice for the
    collective and trimmed afterwards.
    """
    rows = -(-n_total // world)
    pad = torch.zeros((rows,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    out = []
    for r in range(world):
        s, e = shard_bounds(n_total, r, world)
        out.append(parts[r][: e - s])
    return torch.cat(out)


def sharded_search(search_fn, q_all: torch.Tensor, group=None, gather_device=None):
    """Run `search_fn(q_slice, start) -> (D, I)` on this rank's slice of q_all
    (rows start .. start + len) and return the whole batch's (D, I) on every rank.

    The gather runs on the result tensors' device (RCCL for GPU tensors under
    the "nccl" backend) or on ``gather_device`` (e.g. "cpu" under gloo)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    n = q_all.shape[0]
    s, e = shard_bounds(n, rank, world)
    D, I = search_fn(q_all[s:e], s)
    if world == 1:
        return D, I
    if gather_device is not None:
        D, I = D.to(gather_device), I.to(gather_device)
    return all_gather_rows(D, n, world, group), all_gather_rows(I, n, world, group)


# ---- partition sharding ---------------------------------------------------------

def partition_owners(list_sizes, world: int) -> np.ndarray:
    """Owner rank of every bucket: largest lists first, each to the least-loaded
    rank so far (ties -> smaller bucket id, then smaller rank).  Deterministic, so
    every rank computes the same map from the same sizes."""
    if world <= 0:
        raise ValueError("world must be >= 1")
    sizes = np.asarray(list_sizes, dtype=np.int64)
    order = np.lexsort((np.arange(sizes.size), -sizes))
    load = np.zeros(world, dtype=np.int64)
    owner = np.empty(sizes.size, dtype=np.int32)
    for b in order:
        r = int(np.argmin(load))
        owner[b] = r
        load[r] += sizes[b]
    return owner


def bucket_sizes(data_2_bkt: torch.Tensor, n_lists: int) -> np.ndarray:
    """Rows per bucket of an (N,) / (N, n_mul) assignment (-1 = empty slot), on its device."""
    flat = data_2_bkt.reshape(-1)
    flat = flat[flat >= 0].to(torch.int64)
    return torch.bincount(flat, minlength=n_lists).cpu().numpy()


def shard_assignment(data_2_bkt: torch.Tensor, owners, rank: int) -> torch.Tensor:
    """The assignment restricted to this rank's buckets: other buckets' slots -> -1
    (lira_index_build's empty slot), so the rank's index holds only its own lists."""
    own = torch.as_tensor(np.asarray(owners) == rank, device=data_2_bkt.device)
    d2b = data_2_bkt.to(torch.int64)
    keep = (d2b >= 0) & own[d2b.clamp(min=0)]
    return torch.where(keep, data_2_bkt, torch.full_like(data_2_bkt, -1))


def merge_shards(D_parts: torch.Tensor, I_parts: torch.Tensor, metric: str = "L2", dedup: bool = True,
                 out=None, stream=None):
    """k-way merge of (P, nq, k) per-shard top-k results on the device
    (lira_merge_shards): the k smallest keys of the union in the scan's order."""
    from . import _lib
    from .index import METRICS, normalize_metric
    if D_parts.dim() != 3 or I_parts.dim() != 3:
        raise ValueError("D_parts and I_parts must be (P, nq, k)")
    P, nq, k = D_parts.shape
    if I_parts.shape != D_parts.shape:
        raise ValueError("D_parts and I_parts must have the same (P, nq, k) shape")
    if D_parts.dtype != torch.float32 or I_parts.dtype != torch.int64:
        raise ValueError(f"D_parts must be float32 and I_parts int64 (got {D_parts.dtype}, {I_parts.dtype})")
    if D_parts.device != I_parts.device or D_parts.device.type != "cuda":
        raise ValueError("D_parts and I_parts must be on the same GPU")
    D_parts = D_parts.contiguous()
    I_parts = I_parts.contiguous()
    if out is None:
        out = (torch.empty((nq, k), dtype=torch.float32, device=D_parts.device),
               torch.empty((nq, k), dtype=torch.int64, device=D_parts.device))
    else:
        Do, Io = out
        for t, dt, name in ((Do, torch.float32, "out[0]"), (Io, torch.int64, "out[1]")):
            if tuple(t.shape) != (nq, k) or t.dtype != dt or t.device != D_parts.device or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous ({nq}, {k}) {dt} tensor on {D_parts.device}")
    with torch.cuda.device(D_parts.device):
        _lib.call("lira_merge_shards", _lib.ptr(D_parts), _lib.ptr(I_parts), P, nq, k,
                  METRICS[normalize_metric(metric)], int(bool(dedup)), _lib.ptr(out[0]), _lib.ptr(out[1]),
                  _lib.stream_ptr(stream))
    return out


def gather_shards(D: torch.Tensor, I: torch.Tensor, world: int, group=None, gather_device=None):
    """All-gather every rank's (nq, k) result into (world, nq, k) tensors (rank order)."""
    dev = gather_device or D.device
    gd = [torch.empty_like(D, device=dev) for _ in range(world)]
    gi = [torch.empty_like(I, device=dev) for _ in range(world)]
    dist.all_gather(gd, D.to(dev), group=group)
    dist.all_gather(gi, I.to(dev), group=group)
    return torch.stack(gd), torch.stack(gi)


def partition_sharded_search(index, q: torch.Tensor, probe: torch.Tensor, k: int, dedup: bool = True,
                             group=None, gather_device=None):
    """This rank's index holds its buckets' lists only (shard_assignment): scan the
    whole batch against them, all-gather the ranks' top-k and merge on q's device.
    Returns the batch's (D, I) on every rank."""
    D, I, _ = index.search(q, probe, k, dedup=dedup)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return D, I
    Dp, Ip = gather_shards(D, I, world, group, gather_device)
    return merge_shards(Dp.to(q.device), Ip.to(q.device), index.metric, dedup)
