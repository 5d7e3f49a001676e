"""Device snapshot construction (csrc/graphbuild.hip) vs the host build
and the reference's golden indexing (rgcn/utils.py:78-134), -m gpu.

Bar: bit-exact.  Every kernel work list, the CSR, the r2e lists and the DGL-visible
tensors must equal the numpy build's element for element (r_to_e spans: the same entity
sets as the reference, whose order is Python set order)."""
import numpy as np
import pytest
import torch

from regcn_amd import graph as G
from regcn_amd.synthetic import CONFIGS, snapshot_series, zipf_triples

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)

SCALARS = ("n_pos", "n_pos_tiles", "n_heavy", "heavy_slots", "n_slots", "rel_slots", "rel_max_span", "budget",
           "pack_items", "chunk_edges")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def assert_same_graph(V, R, tr, **kw):
    host = G.build_sub_graph(V, R, tr, True, DEV, device_build=False, **kw)
    dev = G.build_sub_graph(V, R, tr, True, DEV, **kw)
    assert isinstance(dev, G.DeviceSnapshotGraph)
    for k in SCALARS:
        assert getattr(dev, k) == getattr(host, k), k
    assert set(dev.dev) == set(host.dev)
    for k, v in host.dev.items():
        w = dev.dev[k]
        assert w.dtype == v.dtype and tuple(w.shape) == tuple(v.shape), (k, w.shape, v.shape)
        assert torch.equal(w, v), k
    for frame in ("ndata", "edata"):
        for k, v in getattr(host, frame).items():
            w = getattr(dev, frame)[k]
            assert w.dtype == v.dtype and torch.equal(w.cpu(), v.cpu()), (frame, k)
    np.testing.assert_array_equal(np.asarray(dev.uniq_r), np.asarray(host.uniq_r))
    assert list(dev.r_len) == [tuple(x) for x in host.r_len]
    np.testing.assert_array_equal(dev.in_degrees().cpu().numpy(), host.in_deg_np)
    np.testing.assert_array_equal(dev.r_to_e.numpy(), host.r_to_e.numpy())
    s0, d0 = host.edges()
    s1, d1 = dev.edges()
    assert torch.equal(s0, s1) and torch.equal(d0, d1)
    return dev


@pytest.mark.parametrize("tag", ["small", "mid", "empty_rel"])
def test_device_build_matches_reference_goldens(golden, tag):
    z = golden("graph_indexing.npz")
    V, R = (int(v) for v in z[tag + "_meta"])
    g = G.build_sub_graph(V, R, z[tag + "_triples"], True, DEV)
    assert isinstance(g, G.DeviceSnapshotGraph)
    src, dst = g.edges()
    np.testing.assert_array_equal(src.numpy(), z[tag + "_src"])
    np.testing.assert_array_equal(dst.numpy(), z[tag + "_dst"])
    np.testing.assert_array_equal(g.edata["type"].cpu().numpy(), z[tag + "_type"])
    np.testing.assert_array_equal(g.in_degrees(range(V)).cpu().numpy(), z[tag + "_in_deg"])
    np.testing.assert_array_equal(g.ndata["norm"].cpu().numpy().reshape(-1), z[tag + "_norm"])
    np.testing.assert_array_equal(g.edata["norm"].cpu().numpy().reshape(-1), z[tag + "_enorm"])
    np.testing.assert_array_equal(np.asarray(g.uniq_r), z[tag + "_uniq_r"])
    np.testing.assert_array_equal(np.asarray(g.r_len).reshape(-1, 2), z[tag + "_r_len"])
    r2e = g.r_to_e.numpy()
    for a, b in z[tag + "_r_len"]:
        assert set(r2e[a:b].tolist()) == set(z[tag + "_r_to_e"][a:b].tolist())
    # the destination-sorted CSR keeps the reference's edge order within a row (stable)
    order = np.argsort(z[tag + "_dst"], kind="stable")
    np.testing.assert_array_equal(g.dev["col_src"].cpu().numpy(), z[tag + "_src"][order])
    np.testing.assert_array_equal(g.dev["col_type"].cpu().numpy(), z[tag + "_type"][order])


@pytest.mark.parametrize("chunk", [1, 3, 64, 512, None])
def test_device_build_matches_host_uniform(chunk):
    rng = np.random.default_rng(0)
    V, R, T = 200, 7, 1500
    tr = np.stack([rng.integers(0, V, T), rng.integers(0, R, T), rng.integers(0, V, T)], 1)
    assert_same_graph(V, R, tr, chunk_edges=chunk)


@pytest.mark.parametrize("case", ["empty", "one", "single_node", "self_loops_dups", "sparse_rel"])
def test_device_build_edge_cases(case):
    if case == "empty":
        V, R, tr = 10, 3, np.zeros((0, 3), np.int64)
    elif case == "one":
        V, R, tr = 10, 3, np.array([[0, 1, 2]])
    elif case == "single_node":
        V, R, tr = 1, 2, np.array([[0, 1, 0], [0, 0, 0], [0, 1, 0]])
    elif case == "self_loops_dups":
        V, R = 30, 4
        tr = np.array([[1, 0, 1], [1, 0, 1], [2, 3, 5], [2, 3, 5], [5, 3, 2], [7, 2, 7], [0, 0, 29]] * 3)
    else:  # most relations absent, ids at the top of their ranges
        V, R = 1000, 500
        tr = np.array([[999, 499, 0], [0, 0, 999], [500, 250, 500], [999, 499, 998]])
    g = assert_same_graph(V, R, tr)
    assert g.number_of_edges() == 2 * len(tr)


def test_device_build_rejects_bad_ids():
    with pytest.raises(ValueError):
        G.build_sub_graph(10, 3, np.array([[0, 3, 1]]), True, DEV)
    with pytest.raises(ValueError):
        G.build_sub_graph(10, 3, np.array([[0, 1, 10]]), True, DEV)


@pytest.mark.parametrize("chunk,budget", [(None, None), (16, 64), (2, 64)])
def test_device_build_matches_host_zipf_hubs(chunk, budget):
    """Zipf in-degrees: heavy rows over the tile budget, hubs with > 64 chunk slots (first-level
    fix-up groups), the sequential greedy tile prefix followed by regular 16-row tiles."""
    rng = np.random.default_rng(3)
    V, R, T = 5000, 64, 60000
    tr = zipf_triples(rng, V, R, T)
    g = assert_same_graph(V, R, tr, chunk_edges=chunk, tile_budget=budget)
    assert g.n_heavy > 0
    if chunk == 2:
        assert (g.dev["fixups"][:, 3] > 0).any()  # first-level groups exist


@pytest.mark.parametrize("name", ["icews14s_lgcn_roth", "icews18_roth", "gdelt"])
def test_device_build_matches_host_dataset_shapes(name):
    cfg = CONFIGS[name]
    for tr in snapshot_series(1, cfg["V"], cfg["R"], 3, cfg["per_snap"]):
        assert_same_graph(cfg["V"], cfg["R"], tr)


def test_device_build_matches_host_large():
    """|V| = 200k, |E| = 2M (multi-block radix passes, 4 sort passes for the r2e pairs, large
    chunk sizes and tile budget)."""
    rng = np.random.default_rng(7)
    V, R, T = 200_000, 256, 1_000_000
    assert_same_graph(V, R, zipf_triples(rng, V, R, T))


def test_device_build_deterministic():
    rng = np.random.default_rng(5)
    V, R, T = 3000, 40, 20000
    tr = zipf_triples(rng, V, R, T)
    a = G.build_sub_graph(V, R, tr, True, DEV)
    b = G.build_sub_graph(V, R, torch.from_numpy(tr).to(DEV), True, DEV)  # triples already in HBM
    for k in a.dev:
        assert torch.equal(a.dev[k], b.dev[k]), k
