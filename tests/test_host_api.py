"""CPU: host-side mirrors of the reference interfaces (readers, threshold
sweep, metric names, device-independent helpers)."""
import numpy as np
import pytest
import torch


def test_xvecs_roundtrip(tmp_path):
    from lira_amd.io import read_bvecs, read_fvecs, read_ivecs, write_xvecs
    rng = np.random.default_rng(0)
    f = rng.standard_normal((7, 5)).astype(np.float32)
    i = rng.integers(-5, 100, (4, 3)).astype(np.int32)
    b = rng.integers(0, 255, (6, 9)).astype(np.uint8)
    write_xvecs(tmp_path / "a.fvecs", f)
    write_xvecs(tmp_path / "a.ivecs", i)
    write_xvecs(tmp_path / "a.bvecs", b)
    assert np.array_equal(read_fvecs(str(tmp_path / "a.fvecs")), f)
    assert np.array_equal(read_ivecs(str(tmp_path / "a.ivecs")), i)
    assert np.array_equal(read_bvecs(str(tmp_path / "a.bvecs")), b)
    # a record with a different dimension is rejected (search.cpp:114-117)
    raw = bytearray(open(tmp_path / "a.fvecs", "rb").read())
    raw[24:28] = np.array([4], np.int32).tobytes()  # record 1's dim field
    open(tmp_path / "bad.fvecs", "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        read_fvecs(str(tmp_path / "bad.fvecs"))


def test_artifacts_roundtrip(tmp_path):
    from lira_amd.io import load_artifacts, save_artifacts
    from lira_amd.probing import MLP_2_Input
    rng = np.random.default_rng(1)
    prefix = str(tmp_path / "art" / "sift-k=10")
    m = MLP_2_Input(8, 16, 8)
    save_artifacts(prefix, rng.random((8, 16)), rng.integers(-1, 8, (50, 2)), rng.random((50, 16)),
                   rng.random(8), rng.random(8), m)
    a = load_artifacts(prefix)
    assert a["centroids"].dtype == np.float32 and a["data_2_bkt"].dtype == np.int32
    x = torch.randn(3, 8), torch.randn(3, 16)
    assert torch.allclose(a["model"](*x), m(*x))
    np.save(prefix + "_scaler_mean.npy", np.zeros(7, np.float32))
    with pytest.raises(ValueError, match="Scaler length"):
        load_artifacts(prefix, load_model=False)


def test_mlp_state_dict_layout():
    # the reference's parameter names (model_probing.py:12-31) load unchanged
    from lira_amd.probing import MLP_2_Input
    keys = set(MLP_2_Input(64, 128, 64).state_dict())
    want = {f"{t}.{i}.{p}" for t in ("distance_net", "vector_net", "fc") for i in (0, 2)
            for p in ("weight", "bias")}
    assert keys == want


def test_threshold_sweep_matches_float_accumulation():
    from lira_amd.search import thresholds
    t = thresholds(0.02, 0.80, 0.02)
    ref, thr = [], np.float32(0.02)
    while thr <= np.float32(np.float32(0.80) + np.float32(1e-6)):
        ref.append(thr)
        thr = np.float32(thr + np.float32(0.02))
    assert t.tolist() == ref and len(t) == len(ref)
    assert len(thresholds(0.5, 0.5, 0.02)) == 1


def test_metric_names():
    from lira_amd.index import normalize_metric
    assert normalize_metric("euclidean") == "L2" and normalize_metric("IP") == "inner_product"
    with pytest.raises(ValueError):
        normalize_metric("cosine")


def test_build_csr_torch_matches_oracle():
    import oracle
    from lira_amd.index import build_csr
    rng = np.random.default_rng(3)
    d2b = rng.integers(-1, 9, (500, 3)).astype(np.int32)
    d2b[5] = [4, 4, -1]
    off, ids, rep = build_csr(torch.from_numpy(d2b), 9)
    o_off, o_ids = oracle.build_csr(d2b, 9)
    assert np.array_equal(off, o_off) and np.array_equal(ids.numpy(), o_ids)
    assert rep == max(np.bincount(o_ids))


@pytest.mark.parametrize("paths", [0, 1, 2, 3])
def test_parse_stats_every_path(paths):
    """lira_index_stats_read's slots [1] / [3] change meaning with the path that
    ran; the path-specific keys exist only for that path (callers use .get)."""
    from lira_amd.index import parse_stats
    v = [10, 11, 12, 13, 14, 15, 16, 17]
    st = parse_stats(v, paths)
    assert (st["chunks_computed"], st["blocks"], st["blocks_skipped"]) == (10, 12, 14)
    assert (st["rechecked"], st["rescans"], st["survivors"]) == (15, 16, 17)
    assert st["paths"] == {0: "none", 1: "exact", 2: "screen", 3: "exact+screen"}[paths]
    if paths == 1:
        assert (st["chunks_nominal"], st["blocks_dropped"]) == (11, 13)
    elif paths == 2:
        assert (st["pairs_pruned_plan"], st["candidates_pruned_plan"]) == (11, 13)
    else:
        assert (st["slot1"], st["slot3"]) == (11, 13)
        assert st.get("pairs_pruned_plan") is None  # what bench.py's work block reads
