"""Config 5 (|V| = 1M, |E| = 50M per snapshot, R = 256, d = 200, the bench's
own synthetic snapshot) pinned against the oracle row by row.

The whole-graph oracle does not fit this size in a test, so ~4.1k rows are pinned: the largest
hubs (4.5M, 2.5M in-edges: the hub pass of k_union_runs / the heavy-row reduction), hubs of
rank 10 / 100 / 1000, 4,000 random rows with in-edges (the inline tiles), the rows of 24 random
crel tiles (>= 2,048 inline items each: the rowtail gather's k_gather_crel, asserted to run) and
64 rows without (W_evolve).  Their oracle outputs come from oracle.graph.row_subgraph (the rows' in-edges with
the full graph's in-degrees) through oracle.layers.union_layer / lorentz_layer in float64, the
messages materialised 2^18 edges at a time.  Both device paths are checked: the 64-row tail
(regcn_layer_rowtail_f32, the default at this size) and the fused 16-row kernel
(regcn_layer_f32), each within 1e-4 * max(1, |ref|)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from gpu_helpers import assert_close

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
C = 0.01
V, R, D, PER_SNAP = 1_000_000, 256, 200, 25_000_000


@pytest.fixture(scope="module")
def case():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from regcn_amd import graph as G
    from regcn_amd.synthetic import snapshot_series
    snap = snapshot_series(100, V, R, 1, PER_SNAP)[0]  # bench.py's config-5 snapshot
    g = G.build_sub_graph(V, R, snap, True, DEV)
    deg = np.bincount(snap[:, 2], minlength=V) + np.bincount(snap[:, 0], minlength=V)
    order = np.argsort(-deg, kind="stable")
    rng = np.random.default_rng(5)
    # rows of the crel gather's tiles (>= CREL_MIN_ITEMS inline items per tile, k_gather_crel:
    # the relation half as one MFMA product per tile), which the rowtail path takes by default
    from regcn_amd import hyperbolic_layers as HL
    wk = g.work()
    tiles = wk["tiles"][:g.n_pos_tiles].cpu().numpy()
    big = np.flatnonzero(np.diff(wk["item_ptr"][:g.n_pos_tiles + 1].cpu().numpy()) >= HL.CREL_MIN_ITEMS)
    assert len(big) >= HL.CREL_MIN_TILES
    prow = wk["rows"].cpu().numpy()
    crel_rows = np.concatenate([prow[tiles[t, 0]:tiles[t, 0] + tiles[t, 1]]
                                for t in rng.choice(big, 24, replace=False)])
    rows = np.unique(np.concatenate([order[[0, 1, 10, 100, 1000]],
                                     rng.choice(np.flatnonzero(deg > 0), 4000, replace=False),
                                     rng.choice(np.flatnonzero(deg == 0), 64, replace=False), crel_rows]))
    assert len(np.intersect1d(rows, crel_rows)) >= 64
    gen = torch.Generator().manual_seed(6)
    # points at hyperbolic radii spread over [0.2, 3] (|x| < 1/sqrt(c) = 10)
    u = torch.randn(V, D, generator=gen)
    rad = 0.2 + 2.8 * torch.rand(V, 1, generator=gen)
    h = (u / u.norm(dim=1, keepdim=True) * rad).to(DEV)
    rel = (0.1 * torch.randn(2 * R, D, generator=gen)).to(DEV)
    return dict(snap=snap, g=g, rows=rows, h=h, rel=rel, deg=deg)


def _oracle(case, kind, layer):
    from oracle import graph as OG
    from oracle import layers as OL
    gs, nodes = OG.row_subgraph(V, R, case["snap"], case["rows"])
    hs = case["h"][torch.from_numpy(nodes).to(DEV)].double().cpu()
    rel = case["rel"].double().cpu()
    dd = lambda p: p.detach().double().cpu()  # noqa: E731
    if kind == "union":
        out = OL.union_layer(gs, hs, rel, dd(layer.weight_neighbor), dd(layer.loop_weight),
                             dd(layer.evolve_loop_weight), C, 0.15, edge_chunk=1 << 18)
    else:
        out = OL.lorentz_layer(gs, hs, rel, dd(layer.weight), dd(layer.loop_weight), dd(layer.evolve_loop_weight),
                               C, layer.num_bases, edge_chunk=1 << 18)
    return out[:len(case["rows"])]


@pytest.mark.parametrize("kind", ["union", "lorentz"])
def test_config5_rows_vs_oracle(case, kind, monkeypatch):
    from regcn_amd import _lib
    from regcn_amd import hyperbolic_layers as HL
    torch.manual_seed(8)
    if kind == "union":
        layer = HL.HyperbolicUnionRGCNLayer(D, D, 2 * R, c=C, activation=F.rrelu, self_loop=True,
                                            radius_msg_gamma=0.15)
    else:
        layer = HL.LorentzRGCNLayer(D, D, 2 * R, num_bases=D // 2, c=C, activation=F.rrelu, self_loop=True)
    layer = layer.to(DEV).eval()
    ref = _oracle(case, kind, layer)
    rows = torch.from_numpy(case["rows"]).to(DEV)
    g = case["g"]
    assert g.n_heavy > 0 and case["deg"].max() > 4_000_000
    for path, threshold, entry in (("rowtail", 1, "regcn_layer_rowtail_f32"), ("fused", 1 << 30, "regcn_layer_f32")):
        monkeypatch.setattr(HL, "ROWTAIL_MIN_ROWS", threshold)
        calls = []
        _lib.EVENT_TRACE = calls
        try:
            with torch.no_grad():
                out = layer(g, case["h"], case["rel"])
            torch.cuda.synchronize()
        finally:
            _lib.EVENT_TRACE = None
        assert entry in {n for n, _ in calls}, (path, calls)
        if path == "rowtail" and kind == "union":  # the crel gather ran over the big tiles
            hit = g.__dict__.get("_crel_tiles")
            assert hit is not None and hit[1] - hit[2] >= HL.CREL_MIN_TILES, hit
            assert HL._crel(g, _lib.AGG_UNION, case["rel"]) is not None
        assert_close(out[rows], ref, what="config-5 %s rows (%s)" % (kind, path))
