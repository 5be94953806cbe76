"""lira_amd -- MI355X (gfx950) implementation of LIRA's query-time hot path.

The hot path of qfshen23/LIRA-ANN-search (partition ranking, candidate scan,
exact top-k) as hand-written HIP kernels behind a C-ABI (include/lira_hip.h,
liblira_hip.so), with the reference's Python-side interfaces on top:

* ``PartitionedIndex``       -- search.cpp's inverted lists + scan (search.cpp:366-514)
* ``IndexFlatL2/IndexFlatIP`` -- the faiss flat indexes LIRA builds per bucket
* ``utils``                  -- get_dist_cid / create_flat_indexes / get_cmp_recall /
                                query_tuning (utils.py, LIRA_smallscale.py)
* ``search``                 -- search.cpp's end-to-end artifact search
* ``knn``                    -- compute_knn.cpp self-kNN, k-means (utils.py:222-330)
"""
from ._lib import LiraError, load as load_library  # noqa: F401
from .index import (PartitionedIndex, build_csr, centroid_dist, centroid_gemm,  # noqa: F401
                    normalize_metric, order_probes, rank_nearest, select_probes, RankWorkspace)
from .faiss_compat import IndexFlatIP, IndexFlatL2  # noqa: F401

__all__ = [
    "LiraError", "PartitionedIndex", "build_csr", "centroid_dist", "centroid_gemm",
    "rank_nearest", "select_probes", "order_probes", "normalize_metric", "IndexFlatL2", "IndexFlatIP",
    "RankWorkspace", "load_library",
]
