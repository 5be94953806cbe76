"""GPU: faiss-shaped IndexFlatL2/IndexFlatIP (utils.py:415-419 usage) against the
oracle's exhaustive scan."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cls,metric", [("IndexFlatL2", oracle.L2), ("IndexFlatIP", oracle.IP)])
def test_flat_index(cls, metric):
    import lira_amd
    rng = np.random.default_rng(1)
    xb = rng.standard_normal((3000, 40), dtype=np.float32)
    xq = rng.standard_normal((25, 40), dtype=np.float32)
    index = getattr(lira_amd, cls)(40)
    index.add(xb[:1000])
    index.add(xb[1000:])  # faiss add appends
    assert index.ntotal == 3000
    D, I = index.search(xq, 10)
    assert isinstance(D, np.ndarray) and D.dtype == np.float32 and I.dtype == np.int64
    off = np.array([0, 3000], np.int64)
    ids = np.arange(3000, dtype=np.int32)
    Do, Io, _ = oracle.scan_topk(xq, off, ids, xb, np.zeros((25, 1), np.int32), 10, metric, 0)
    assert np.array_equal(I, Io) and np.array_equal(D.view(np.uint32), Do.view(np.uint32))
    if metric == oracle.L2:
        assert (np.diff(D, axis=1) >= 0).all()
    else:
        assert (np.diff(D, axis=1) <= 0).all()


def test_fewer_than_k_vectors_pads():
    import lira_amd
    index = lira_amd.IndexFlatL2(8)
    index.add(np.eye(8, dtype=np.float32)[:3])
    D, I = index.search(np.zeros((2, 8), np.float32), 5)
    assert I[:, 3:].tolist() == [[-1, -1], [-1, -1]] and np.isinf(D[:, 3:]).all()
    empty = lira_amd.IndexFlatIP(8)
    D, I = empty.search(np.zeros((1, 8), np.float32), 2)
    assert (I == -1).all() and (D == -np.inf).all()
