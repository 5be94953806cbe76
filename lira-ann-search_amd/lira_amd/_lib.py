"""ctypes binding of liblira_hip.so (include/lira_hip.h).

This is the binding the reference's Python side would add to reach the HIP
module.  There is no fallback: if the shared library is
missing or cannot be loaded, every entry point raises ``LiraError`` -- the hot
path never silently runs on the CPU or in plain PyTorch.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LIRA_HIP_LIB", os.path.join(_HERE, "liblira_hip.so"))

LIRA_OK = 0
LIRA_METRIC_L2 = 0
LIRA_METRIC_IP = 1
LIRA_SCAN_DEDUP = 1
LIRA_SCAN_PER_PARTITION = 2
LIRA_SCAN_FMA = 4
LIRA_SCAN_NO_PRUNE = 8
LIRA_SCAN_EXACT = 16
LIRA_SCAN_NO_SPLIT = 32
# lira_index_set_option keys (include/lira_hip.h LIRA_OPT_*)
OPTIONS = {"keep_tiles": 1, "screen": 2, "split": 3, "qr": 4, "two_phase": 5, "prune": 6, "seed": 7,
           "share": 8, "rounds": 9, "near_rounds": 10, "mfma": 11, "debug": 12, "pipeline": 13, "ring": 14, "probes_hint": 15, "xhi": 16,
           "order": 17, "wide": 18, "rscreen": 19, "near_first": 20,
           "rescan": 21, "spill": 22,
           "seed_tiles": 23, "ip_centre": 24, "chunk": 25}
LIRA_PROBE_NEAREST = 0
LIRA_PROBE_THRESHOLD_GE = 1
LIRA_PROBE_THRESHOLD_GT = 2
LIRA_PROBE_BY_SCORE = 16

_STATUS = {
    -1: "EINVAL",
    -2: "ERANGE",
    -3: "ENOMEM",
    -4: "EHIP",
    -5: "ESTATE",
    -6: "EUNSUPPORTED",
}

# (name, restype, argtypes) for every symbol include/lira_hip.h declares
_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_INT = ctypes.c_int
_F = ctypes.c_float
_SZ = ctypes.c_size_t
SIGNATURES = {
    "lira_abi_version": (_INT, []),
    "lira_last_error": (ctypes.c_char_p, []),
    "lira_device_cu_count": (_INT, [_INT, ctypes.POINTER(_INT)]),
    "lira_index_create": (_INT, [_INT, _I64, _INT, ctypes.POINTER(_P)]),
    "lira_index_destroy": (_INT, [_P]),
    "lira_index_add_partitions": (_INT, [_P, _I64, _P, _P, _P, _I64, _I32, _P]),
    "lira_index_build": (_INT, [_P, _I64, _P, _I64, _I32, _P, _P]),
    "lira_index_list_ids": (_INT, [_P, _I64, _P, _P]),
    "lira_index_info": (_INT, [_P, ctypes.POINTER(_I64), ctypes.POINTER(_INT),
                               ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "lira_index_list_size": (_INT, [_P, _I64, ctypes.POINTER(_I64)]),
    "lira_index_memory": (_INT, [_P, ctypes.POINTER(_I64)]),
    "lira_index_set_option": (_INT, [_P, _INT, _I64]),
    "lira_index_get_option": (_INT, [_P, _INT, ctypes.POINTER(_I64)]),
    "lira_index_has_tiles": (_INT, [_P, ctypes.POINTER(_INT)]),
    "lira_centroid_dist": (_INT, [_P, _I64, _P, _I64, _I64, _P, _P, _P, _P]),
    "lira_centroid_gemm": (_INT, [_P, _I64, _P, _I64, _I64, _P, _P, _P]),
    "lira_rank_workspace_size": (_INT, [_I64, _I64, ctypes.POINTER(_SZ)]),
    "lira_rank_nearest": (_INT, [_P, _I64, _P, _I64, _I64, _I64, _P, _P, _SZ, _P]),
    "lira_select_probes": (_INT, [_P, _I64, _I64, _INT, _F, _I64, _P, _P, _P]),
    "lira_order_probes": (_INT, [_P, _I64, _I64, _P, _I64, _P]),
    "lira_merge_shards": (_INT, [_P, _P, _I64, _I64, _I64, _INT, _INT, _P, _P, _P]),
    "lira_scan_workspace_size": (_INT, [_P, _I64, _I64, _I64, ctypes.c_uint, ctypes.POINTER(_SZ)]),
    "lira_scan_topk": (_INT, [_P, _P, _I64, _P, _I64, _I64, ctypes.c_uint, _P, _P, _P, _P, _SZ, _P]),
    "lira_scan_describe": (_INT, [_P, _I64, _I64, _I64, ctypes.c_uint, ctypes.c_char_p, _SZ]),
    "lira_index_check": (_INT, [_P, _P]),
    "lira_index_set_profiling": (_INT, [_P, _INT]),
    "lira_index_set_stats": (_INT, [_P, _INT]),
    "lira_index_stats_read": (_INT, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    "lira_index_stats_paths": (_INT, [_P, ctypes.POINTER(_INT)]),
    "lira_index_profile_read": (_INT, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I64)]),
}


class LiraError(RuntimeError):
    """A liblira_hip.so call failed (mirrors faiss's FaissException -> RuntimeError)."""


_lock = threading.Lock()
_lib = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Load (once) and type liblira_hip.so.  Raises LiraError if absent."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise LiraError(
                f"liblira_hip.so not found at {p}: build it with `make -C lira-ann-search_amd` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        try:
            # torch first: it owns the process's HIP runtime (same SONAME), so the
            # module shares its device pointers and streams
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is part of the image
            pass
        try:
            lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise LiraError(f"cannot load {p}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str = "") -> None:
    if rc != LIRA_OK:
        msg = load().lira_last_error()
        msg = msg.decode() if msg else ""
        raise LiraError(f"{what or 'lira call'} failed [{_STATUS.get(rc, rc)}]: {msg}")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def ptr(t) -> int:
    """Device/host pointer of a torch tensor (or None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
