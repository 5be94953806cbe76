"""Readers for the reference's on-disk formats.

* ``.fvecs`` / ``.ivecs`` / ``.bvecs``: per record an int32 dimension followed by
  d values (float32 / int32 / uint8).  utils.py:23-39 (read_xvecs, memmap),
  search.cpp:86-166 (read_fvecs / read_ivecs with dimension checks),
  compute_knn.cpp:14-52 (bvecs, the BIGANN source format).
* index artifacts written by index.py:144-192 and utils.py:170-178, read by
  search.cpp:300-335: ``{prefix}_centroids.npy`` (B,d) f32,
  ``_data_2_bkt.npy`` (N,n_mul) i32, ``_x_d.npy`` (N,d) f32,
  ``_scaler_mean.npy`` / ``_scaler_scale.npy`` (B,) f32, ``_mlp_2_input.pt``.

numpy.load runs with allow_pickle=False: artifacts are plain arrays.
"""
from __future__ import annotations

import os

import numpy as np

_XVEC_DTYPES = {"float32": np.float32, "int32": np.int32, "uint8": np.uint8}


def read_xvecs(file_path: str, dtype: str = "float32") -> np.ndarray:
    """(n, d) view of an xvecs file (utils.py:23-39 semantics, memory-mapped).

    The dimension is checked on every record (search.cpp:108-122 rejects a file
    whose records disagree); the result is read-only.
    """
    if not os.path.exists(file_path):
        raise FileNotFoundError(f"File not found: {file_path}")
    dt = np.dtype(_XVEC_DTYPES[dtype])
    raw = np.memmap(file_path, dtype=np.uint8, mode="r")
    if raw.size < 4:
        raise ValueError(f"Invalid xvecs file size: {file_path}")
    d = int(raw[:4].view(np.int32)[0])
    rec = 4 + d * dt.itemsize
    if d <= 0 or raw.size % rec:
        raise ValueError(f"Invalid xvecs file size: {file_path}")
    n = raw.size // rec
    recs = raw.reshape(n, rec)
    dims = recs[:, :4].copy().view(np.int32)[:, 0]
    if (dims != d).any():
        raise ValueError(f"Inconsistent dim in xvecs: {file_path}")
    if dt.itemsize == 4:  # aligned records: zero-copy strided view like utils.py
        return np.memmap(file_path, dtype=dt, mode="r").reshape(n, d + 1)[:, 1:]
    return recs[:, 4:].view(dt)


def read_fvecs(path: str) -> np.ndarray:
    return read_xvecs(path, "float32")


def read_ivecs(path: str) -> np.ndarray:
    return read_xvecs(path, "int32")


def read_bvecs(path: str) -> np.ndarray:
    return read_xvecs(path, "uint8")


def write_xvecs(path: str, a: np.ndarray) -> None:
    """Inverse of read_xvecs (for fixtures and tools)."""
    a = np.ascontiguousarray(a)
    n, d = a.shape
    with open(path, "wb") as f:
        hdr = np.array([d], dtype=np.int32).tobytes()
        for i in range(n):
            f.write(hdr)
            f.write(a[i].tobytes())


def load_dataset(dataset_name: str, data_path: str = "/data/vector_datasets"):
    """utils.py:41-88: {name}_base.fvecs (or _learn), _query.fvecs, _groundtruth.ivecs."""
    ddir = os.path.join(data_path, dataset_name)
    base = os.path.join(ddir, f"{dataset_name}_base.fvecs")
    if not os.path.exists(base):
        base = os.path.join(ddir, f"{dataset_name}_learn.fvecs")
    x_d = np.ascontiguousarray(read_fvecs(base))
    x_q = np.ascontiguousarray(read_fvecs(os.path.join(ddir, f"{dataset_name}_query.fvecs")))
    gt = os.path.join(ddir, f"{dataset_name}_groundtruth.ivecs")
    gt_ids = np.ascontiguousarray(read_ivecs(gt)) if os.path.exists(gt) else None
    return x_d, x_q, gt_ids


def _load2d(path, dtype):
    a = np.load(path, allow_pickle=False)
    if a.dtype != dtype:
        raise ValueError(f"Expected {np.dtype(dtype).name} npy: {path}")
    if a.ndim != 2:
        raise ValueError(f"Expected 2D npy: {path}")
    return a


def load_artifacts(prefix: str, load_model: bool = True, device="cpu") -> dict:
    """search.cpp:300-335: the index contract written by index.py."""
    out = {
        "centroids": _load2d(prefix + "_centroids.npy", np.float32),
        "data_2_bkt": _load2d(prefix + "_data_2_bkt.npy", np.int32),
        "x_d": _load2d(prefix + "_x_d.npy", np.float32),
    }
    n_bkt, dc = out["centroids"].shape
    if out["x_d"].shape[0] != out["data_2_bkt"].shape[0]:
        raise ValueError("x_d.npy and data_2_bkt.npy mismatch in N.")
    if out["x_d"].shape[1] != dc:
        raise ValueError("centroids dim and x_d dim mismatch.")
    for key in ("scaler_mean", "scaler_scale"):
        a = np.load(prefix + f"_{key}.npy", allow_pickle=False)
        if a.dtype != np.float32 or a.ndim != 1:
            raise ValueError(f"Expected 1D float32 npy: {prefix}_{key}.npy")
        if a.shape[0] != n_bkt:
            raise ValueError("Scaler length must equal n_bkt.")
        out[key] = a
    if load_model:
        import torch
        out["model"] = torch.jit.load(prefix + "_mlp_2_input.pt", map_location=device).eval()
    return out


def save_artifacts(prefix: str, centroids, data_2_bkt, x_d, scaler_mean, scaler_scale,
                   model=None) -> None:
    """Write the same contract (index.py:161-184, utils.py:172-175)."""
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    np.save(prefix + "_centroids.npy", np.asarray(centroids, np.float32))
    np.save(prefix + "_data_2_bkt.npy", np.asarray(data_2_bkt, np.int32))
    np.save(prefix + "_x_d.npy", np.asarray(x_d, np.float32))
    np.save(prefix + "_scaler_mean.npy", np.asarray(scaler_mean, np.float32))
    np.save(prefix + "_scaler_scale.npy", np.asarray(scaler_scale, np.float32))
    if model is not None:
        import torch
        torch.jit.save(model if isinstance(model, torch.jit.ScriptModule) else torch.jit.script(model),
                       prefix + "_mlp_2_input.pt")
