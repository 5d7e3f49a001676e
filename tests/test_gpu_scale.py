"""Config-5 scale parity (-m gpu): BASELINE.json configs[4] snapshot shape, |V| = 1M,
|E| = 50M directed edges, R2 = 512, d = 200 (Zipf(1.1) subjects and objects).

At this size the oracle's per-edge message tensor alone is 40 GB, so the check is a
size-independent property of the layer (linearity of W_n): the fused layer
launch (inline gathers of the in-budget rows in per-tile item order + the hub rows'
pre-aggregation in row/type order + MFMA tail) equals the chunked aggregation of every row
in CSR edge order (regcn_union_aggregate_f32 / regcn_lorentz_aggregate_f32) followed by the
reference tail in plain torch fp32 on the device (hyperbolic_layers.py:242-323, :627-694,
the oracle's op sequence): |delta| <= 1e-4 * max(1, |ref|) over all 1M rows."""
import numpy as np
import pytest
import torch

from gpu_helpers import assert_close

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
C = 0.01


@pytest.fixture(scope="module")
def snapshot():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from regcn_amd import graph as G
    from regcn_amd.synthetic import snapshot_series
    V, R, d = 1_000_000, 256, 200
    snap = snapshot_series(3, V, R, 1, 25_000_000)[0]
    g = G.build_sub_graph(V, R, snap, True, DEV)
    del snap
    assert g.n_heavy > 0 and g.number_of_edges() == 50_000_000
    gen = torch.Generator(device=DEV).manual_seed(5)
    from oracle import ops
    v = torch.randn(V, d, device=DEV, generator=gen)
    h = ops.apply_radius(ops.exp0(v, C), torch.rand(V, device=DEV, generator=gen) * 2.5 + 0.5, C).contiguous()
    rel = (torch.randn(2 * R, d, device=DEV, generator=gen) * 0.3).contiguous()
    yield g, h, rel
    torch.cuda.empty_cache()


def _tail(agg, x, g, w_loop, w_evolve):
    """clamp(agg) + self loop (W_loop rows with in-edges, W_evolve the others) -> clamp ->
    rrelu(11/48) -> exp0 (hyperbolic_layers.py:273-321)."""
    from oracle import ops
    deg = g.in_degrees()
    loop = torch.where((deg > 0).unsqueeze(1), x @ w_loop, x @ w_evolve)
    hn = torch.clamp(torch.clamp(agg, -10.0, 10.0) + loop, -10.0, 10.0)
    return ops.exp0(ops.leaky(hn), C)


def test_union_layer_config5(snapshot):
    import torch.nn.functional as F
    from oracle import ops
    from regcn_amd import _lib
    from regcn_amd.hyperbolic_layers import HyperbolicUnionRGCNLayer
    g, h, rel = snapshot
    V, d = h.shape
    torch.manual_seed(0)
    lay = HyperbolicUnionRGCNLayer(d, d, rel.shape[0], c=C, activation=F.rrelu, self_loop=True,
                                   radius_msg_gamma=0.15).to(DEV).eval()
    with torch.no_grad():
        got = lay(g, h, rel)
        x = ops.log0(h, C).contiguous()
        r = h.norm(dim=1).contiguous()
        wk = g.work()
        ch, fx = wk["chunks"], wk["fixups"]
        part = torch.empty(max(g.n_slots, 1), d, device=DEV)
        s = torch.zeros(V, d, device=DEV)  # norm * sum_e w_e (x_src + rel_type), CSR edge order; 0 without in-edges
        f, i = _lib.fptr, _lib.iptr
        _lib.call("regcn_union_aggregate_f32", f(x), f(r), f(rel), i(wk["col_src"]), i(wk["col_type"]),
                  f(wk["norm"]), i(ch), ch.shape[0], i(fx), fx.shape[0], 0.15, d, f(part), d, f(s), _lib.stream())
        ref = _tail(s @ lay.weight_neighbor, x, g, lay.loop_weight, lay.evolve_loop_weight)
    assert torch.isfinite(got).all()
    assert_close(got, ref, what="config-5 union layer")


def test_lorentz_layer_config5(snapshot):
    import torch.nn.functional as F
    from oracle import ops
    from regcn_amd import _lib
    from regcn_amd.hyperbolic_layers import LorentzRGCNLayer
    g, h, rel = snapshot
    V, d = h.shape
    torch.manual_seed(1)
    lay = LorentzRGCNLayer(d, d, rel.shape[0], 100, c=C, activation=F.rrelu, self_loop=True).to(DEV).eval()
    with torch.no_grad():
        got = lay(g, h, rel)
        x = ops.log0(h, C).contiguous()
        wk = g.work()
        ch, fx = wk["chunks"], wk["fixups"]
        part = torch.empty(max(g.n_slots, 1), d + 4, device=DEV)
        s = torch.zeros(V, d, device=DEV)  # log0(to_poincare(centroid)), CSR edge order; 0 without in-edges
        f, i = _lib.fptr, _lib.iptr
        _lib.call("regcn_lorentz_aggregate_f32", f(x), f(rel), f(lay.weight.detach().contiguous()),
                  i(wk["col_src"]), i(wk["col_type"]), i(ch), ch.shape[0], i(fx), fx.shape[0], 100, C, d, f(part),
                  d + 4, f(s), _lib.stream())
        ref = _tail(s, x, g, lay.loop_weight, lay.evolve_loop_weight)
    assert torch.isfinite(got).all()
    assert_close(got, ref, what="config-5 lorentz layer")
    # rows without in-edges: zero aggregate, W_evolve loop only
    zero = (g.in_degrees() == 0)
    if bool(zero.any()):
        assert_close(got[zero], ref[zero], what="rows without in-edges")
    np.testing.assert_array_equal(int(zero.sum()), V - g.n_pos)


def test_relation_means_entity_blocks(snapshot):
    """Relation means at config 5 over the entity-block chunks (graph.rel_block_lists: spans cut
    at entity-block boundaries, a block's chunks dealt to one XCD) against a float64 segment
    mean of the same r_to_e spans (hyperbolic_model.py:802-812) and against the plain relation
    chunks: |delta| <= 1e-5 * max(1, |ref|); the inverse rows copy the forward ones."""
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_model import relation_context
    g, h, rel = snapshot
    R2, d = rel.shape[0], h.shape[1]
    R = R2 // 2
    g.__dict__.pop("_rel_block", None)
    assert G.rel_block_work(g, R) is not None, "config 5 must take the entity-block lists"
    with torch.no_grad():
        got = relation_context(h, g, R2)
        wk = g.work()
        lens = wk["rel_count"][:R].long()
        first = torch.cumsum(lens, 0) - lens
        pos = torch.arange(int(lens.sum()), device=DEV) + torch.repeat_interleave(wk["rel_start"][:R].long() - first, lens)
        ent = wk["rel_idx"].long()[pos]
        rel_of = torch.repeat_interleave(torch.arange(R, device=DEV), lens)
        ref = torch.zeros(R, d, device=DEV, dtype=torch.float64)
        for c in range(0, ent.numel(), 1 << 20):
            ref.index_add_(0, rel_of[c:c + (1 << 20)], h[ent[c:c + (1 << 20)]].double())
        ref = ref / lens.clamp(min=1).double().unsqueeze(1)
        saved = G.REL_BLOCK
        try:
            G.REL_BLOCK = 0
            g.__dict__.pop("_rel_block", None)
            plain = relation_context(h, g, R2)
        finally:
            G.REL_BLOCK = saved
            g.__dict__.pop("_rel_block", None)
    tol = 1e-5 * max(1.0, float(ref.abs().max()))
    assert float((got[:R].double() - ref).abs().max()) <= tol
    assert float((got[:R] - plain[:R]).abs().max()) <= tol
    assert torch.equal(got[R:], got[:R])


@pytest.mark.parametrize("euclid", [False, True])
def test_hub_pass_source_blocks(snapshot, euclid):
    """The hub rows' pre-aggregation over source-block chunks (graph.hub_block_work: each hub
    row's source-ordered span cut at source-id blocks, XCD-dealt) equals the plain heavy chunks'
    within 1e-5 * max(1, |ref|) on every hub row (same sums, another fp32 association)."""
    from oracle import ops
    from regcn_amd import _lib
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_layers import _heavy_aggregate
    g, h, rel = snapshot
    mode = _lib.AGG_EUCLID if euclid else _lib.AGG_UNION
    with torch.no_grad():
        x = ops.log0(h, C).contiguous()
        r = h.norm(dim=1).contiguous()
        g.__dict__.pop("_hub_block", None)
        assert G.hub_block_work(g) is not None, "config 5 must take the source-block hub lists"
        got = _heavy_aggregate(mode, g, x, r, rel, None, 1, 0.15, C)
        saved = G.HUB_BLOCK
        try:
            G.HUB_BLOCK = 0
            g.__dict__.pop("_hub_block", None)
            ref = _heavy_aggregate(mode, g, x, r, rel, None, 1, 0.15, C)
        finally:
            G.HUB_BLOCK = saved
            g.__dict__.pop("_hub_block", None)
    hubs = g.work()["rows"][:g.n_heavy].long()
    a, b = got[hubs], ref[hubs]
    assert torch.isfinite(a).all()
    assert float((a - b).abs().max()) <= 1e-5 * max(1.0, float(b.abs().max()))


def test_config5_predict_entity_blocks_vs_plain():
    """The headline workload end to end (BASELINE.json configs[4]: 3 snapshots of |E| = 50M,
    2 uvrgcn layers, RotH + RotHRel on 256 queries; bench.build_model) with the entity-block
    relation and hub lists against the plain chunk lists: the same sums in another fp32
    association, so the scores agree to 1e-4 * max(1, |ref|) and each target's raw rank moves
    by at most its near-ties (candidates within twice the largest score change of it)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bench
    from regcn_amd import graph as G
    from regcn_amd.synthetic import CONFIGS, snapshot_series
    cfg = CONFIGS["synthetic_1m"]
    snaps = snapshot_series(11, cfg["V"], cfg["R"], cfg["T"] + 1, cfg["per_snap"])
    glist = [G.build_sub_graph(cfg["V"], cfg["R"], s, True, DEV) for s in snaps[:cfg["T"]]]
    test = torch.from_numpy(snaps[cfg["T"]][:256]).to(DEV)
    del snaps
    model = bench.build_model(cfg, 200, DEV, seed=7)
    model.param_caches = False
    saved = (G.REL_BLOCK, G.HUB_BLOCK)
    outs = []
    try:
        for rb, hb in (saved, (0, 0)):
            G.REL_BLOCK, G.HUB_BLOCK = rb, hb
            for g in glist:
                g.__dict__.pop("_rel_block", None)
                g.__dict__.pop("_hub_block", None)
            with torch.no_grad():
                r = model.predict(glist, cfg["R"], None, test, True)
            outs.append([t.clone() for t in r[1:3]])
            if rb:
                assert all(G.rel_block_work(g, cfg["R"]) is not None and G.hub_block_work(g) is not None for g in glist)
    finally:
        G.REL_BLOCK, G.HUB_BLOCK = saved
        for g in glist:
            g.__dict__.pop("_rel_block", None)
            g.__dict__.pop("_hub_block", None)
    (s_b, sr_b), (s_p, sr_p) = outs
    for a, b in ((s_b, s_p), (sr_b, sr_p)):
        assert torch.isfinite(a).all()
        assert float((a - b).abs().max()) <= 1e-4 * max(1.0, float(b.abs().max()))
    tgt = torch.cat([test[:, 2], test[:, 0]]).long()  # queries and their inverses (predict)
    assert s_b.shape[0] == tgt.numel()
    # a candidate can swap order with the target only if their plain scores lie within twice
    # the largest score change: the raw ranks differ by at most that many near-ties
    rank = lambda s: (s > s.gather(1, tgt[:, None])).sum(1)
    band = 2.0 * float((s_b - s_p).abs().max())
    ties = ((s_p - s_p.gather(1, tgt[:, None])).abs() <= band).sum(1)
    assert bool(((rank(s_b) - rank(s_p)).abs() <= ties).all())
