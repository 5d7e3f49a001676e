"""CPU-side checks: host graph construction (bit-exact vs the reference's golden
indexing), work-list invariants, and that the C-ABI library loads and exports every
symbol include/regcn_hip.h declares (no compute call: there is no GPU here)."""
import ctypes
import math
import os
import re

import numpy as np
import pytest

from conftest import REPO
from regcn_amd import graph as G

HEADER = os.path.join(REPO, "include", "regcn_hip.h")
LIB = os.path.join(REPO, "re-gcn_amd", "regcn_amd", "libregcn_hip.so")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*|size_t)\s+(regcn_\w+)\s*\(", txt, re.M)))


@pytest.mark.skipif(not os.path.exists(LIB), reason="libregcn_hip.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    import torch  # noqa: F401  (binds the HIP runtime first, as the package does)
    lib = ctypes.CDLL(LIB)
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    from regcn_amd import _lib
    assert sorted(_lib.exported_symbols()) == syms
    assert _lib.lib().regcn_version() == _lib.ABI_VERSION
    assert _lib.lib().regcn_hyp_ce_workspace_bytes(3, 130) == (3 * 256 * 2 + 3) * 4  # >= 256 partial slots


@pytest.mark.parametrize("tag", ["small", "mid", "empty_rel"])
def test_graph_matches_reference_indexing(golden, tag):
    z = golden("graph_indexing.npz")
    V, R = (int(v) for v in z[tag + "_meta"])
    g = G.build_sub_graph(V, R, z[tag + "_triples"], False, 0)
    src, dst = g.edges()
    np.testing.assert_array_equal(src.numpy(), z[tag + "_src"])
    np.testing.assert_array_equal(dst.numpy(), z[tag + "_dst"])
    np.testing.assert_array_equal(g.edata["type"].numpy(), z[tag + "_type"])
    np.testing.assert_array_equal(g.in_degrees(range(V)).numpy(), z[tag + "_in_deg"])
    np.testing.assert_array_equal(g.ndata["norm"].numpy().reshape(-1), z[tag + "_norm"])
    np.testing.assert_array_equal(g.edata["norm"].numpy().reshape(-1), z[tag + "_enorm"])
    np.testing.assert_array_equal(np.asarray(g.uniq_r), z[tag + "_uniq_r"])
    np.testing.assert_array_equal(np.asarray(g.r_len).reshape(-1, 2), z[tag + "_r_len"])
    r2e = np.asarray(g.r_to_e)
    for a, b in z[tag + "_r_len"]:
        assert set(r2e[a:b].tolist()) == set(z[tag + "_r_to_e"][a:b].tolist())
    np.testing.assert_array_equal(g.ndata["id"].numpy().reshape(-1), np.arange(V))


@pytest.mark.parametrize("chunk", [1, 3, 64, 512])
def test_work_lists_cover_every_edge_once(chunk):
    rng = np.random.default_rng(0)
    V, R, T = 200, 7, 1500
    p = 1.0 / np.arange(1, V + 1) ** 1.2
    p /= p.sum()
    tr = np.stack([rng.choice(V, T, p=p), rng.integers(0, R, T), rng.choice(V, T, p=p)], 1)
    g = G.build_sub_graph(V, R, tr, False, 0, chunk_edges=chunk)
    h = g._host
    ch, fx = h["chunks"], h["fixups"]
    # chunks tile each row's CSR range exactly, in order
    deg = g.in_deg_np
    ptr = np.concatenate([[0], np.cumsum(deg)])
    seen = np.zeros(ptr[-1], dtype=np.int64)
    for row, b, e, s in ch:
        assert ptr[row] <= b < e <= ptr[row + 1]
        assert e - b <= chunk
        seen[b:e] += 1
        if s < 0:
            assert (b, e) == (ptr[row], ptr[row + 1])
    assert (seen == 1).all()
    slots = sorted(int(s) for s in ch[:, 3] if s >= 0)
    assert slots == list(range(len(slots)))
    # fix-ups: first-level groups (out > 0) cover <= 64 consecutive chunk slots each and
    # write new slots; every row's final fix-up covers its chunk slots, directly or
    # through its groups, in chunk order
    group_of = {int(o) - 1: (int(b), int(e)) for _, b, e, o in fx if o > 0}
    assert all(e - b <= 64 for b, e in group_of.values())
    assert sorted(group_of) == list(range(len(slots), g.n_slots))
    finals = [f for f in fx if f[3] == 0]
    assert len(finals) == len({int(f[0]) for f in finals})
    for row, sb, se, _ in finals:
        covered = []
        for s_ in range(sb, se):
            b, e = group_of.get(s_, (s_, s_ + 1))
            covered.extend(range(b, e))
        assert covered == list(ch[ch[:, 0] == row][:, 3])
        assert all(e - b <= 64 for b, e in [(sb, se)])
    # CSR columns: stable dst sort of the reference edge order
    order = np.argsort(g.dst_np, kind="stable")
    np.testing.assert_array_equal(h["col_src"], g.src_np[order])
    np.testing.assert_array_equal(h["col_type"], g.type_np[order])
    # rows: deg>0 first
    assert (deg[h["rows"][:g.n_pos]] > 0).all() and (deg[h["rows"][g.n_pos:]] == 0).all()
    assert sorted(h["rows"].tolist()) == list(range(V))
    # relation spans
    # relation spans: the forward relations' spans are chunked exactly once; the inverse
    # spans (second half of rel_idx) repeat them and are not chunked
    rc = h["rel_chunks"]
    cov = np.zeros(len(h["rel_idx"]), dtype=np.int64)
    for r, b, e, s in rc:
        cov[b:e] += 1
        assert h["rel_count"][r] > 0 and r < g.num_rels
    half = len(h["rel_idx"]) // 2
    assert (cov[:half] == 1).all() and (cov[half:] == 0).all()
    np.testing.assert_array_equal(h["rel_idx"][:half], h["rel_idx"][half:])


@pytest.mark.parametrize("V,T", [(200, 1500), (50, 40), (3000, 70000)])
def test_fused_layer_tiles(V, T):
    """Tiles of the fused layer kernel (csrc/layer.hip): each positive row in exactly one
    tile, <= 16 rows, inline edges within budget (a lone row may exceed only if heavy),
    heavy rows pre-aggregated by chunks covering exactly their CSR spans."""
    rng = np.random.default_rng(V)
    p = 1.0 / np.arange(1, V + 1) ** 1.3
    p /= p.sum()
    tr = np.stack([rng.choice(V, T, p=p), rng.integers(0, 9, T), rng.choice(V, T, p=p)], 1)
    g = G.build_sub_graph(V, 9, tr, False, 0)
    h = g._host
    deg = g.in_deg_np
    rows = h["rows"]
    np.testing.assert_array_equal(h["rowptr"], np.concatenate([[0], np.cumsum(deg)]))
    assert (np.diff(deg[rows[:g.n_pos]]) <= 0).all()  # in-degree descending
    tiles = h["tiles"]
    assert len(tiles) == g.n_pos_tiles
    assert tiles[0, 0] == 0 and (tiles[1:, 0] == tiles[:-1, 0] + tiles[:-1, 1]).all()
    assert tiles[-1, 0] + tiles[-1, 1] == g.n_pos
    assert ((tiles[:, 1] >= 1) & (tiles[:, 1] <= 16)).all()
    heavy = set()
    for s, c in tiles:
        d = deg[rows[s:s + c]]
        inl = np.where(d > g.budget, 0, d)
        assert inl.sum() <= g.budget
        heavy.update(rows[s:s + c][d > g.budget].tolist())
    assert len(heavy) == g.n_heavy
    cov = np.zeros(len(h["col_src"]), dtype=np.int64)
    for row, b, e, s in h["heavy_chunks"]:
        assert row in heavy and h["rowptr"][row] <= b < e <= h["rowptr"][row + 1]
        cov[b:e] += 1
    for row in heavy:
        assert (cov[h["rowptr"][row]:h["rowptr"][row + 1]] == 1).all()
    assert cov.sum() == sum(deg[r] for r in heavy)


def test_empty_snapshot():
    g = G.build_sub_graph(10, 3, np.zeros((0, 3), dtype=np.int64), False, 0)
    assert g.number_of_edges() == 0 and g.n_pos == 0
    assert g._host["chunks"].shape == (0, 4) and g._host["rel_chunks"].shape == (0, 4)


def test_cpu_graph_has_no_kernel_path():
    g = G.build_sub_graph(10, 3, np.array([[0, 1, 2]]), False, 0)
    with pytest.raises(ValueError):
        g.work()


def test_split_by_time_and_filter_answers():
    """rgcn/utils.py:264-339 host helpers (no GPU)."""
    from regcn_amd.ranking import load_all_answers_for_filter, split_by_time
    data = np.array([[0, 1, 2, 5], [3, 1, 4, 5], [0, 2, 4, 7], [1, 0, 2, 9], [2, 0, 1, 9]])
    snaps = split_by_time(data)
    assert [s.tolist() for s in snaps] == [[[0, 1, 2], [3, 1, 4]], [[0, 2, 4]], [[1, 0, 2], [2, 0, 1]]]
    ans = load_all_answers_for_filter(snaps[0], 10)
    assert ans == {0: {1: {2}}, 2: {11: {0}}, 3: {1: {4}}, 4: {11: {3}}}
    ans_r = load_all_answers_for_filter(snaps[0], 10, rel_p=True)
    assert ans_r == {0: {2: {1}}, 2: {0: {11}}, 3: {4: {1}}, 4: {3: {11}}}


def test_multistep_filter_and_snap_vs_reference(golden):
    """--multi-step host logic (no GPU): the reference's in-place -1e7 filter of the score
    (rgcn/utils.py:51-75) via the filter CSR, then construct_snap(_r)'s top-k triples
    (rgcn/utils.py:367-405), against the reference's outputs on the same scores."""
    import torch
    from regcn_amd.ranking import _filter_csr, apply_filter_, construct_snap, construct_snap_r, \
        load_all_answers_for_filter
    z, zm = golden("rank.npz"), golden("multistep.npz")
    V, R = (int(v) for v in z["meta"])
    k = int(zm["topk"][0])
    tr = torch.from_numpy(z["all_triples"])
    for rel, key, ref_score, make in ((False, "score", "filtered_score", construct_snap),
                                      (True, "score_rel", "filtered_score_rel", construct_snap_r)):
        score = torch.from_numpy(z[key]).clone()
        fp, fi = _filter_csr(tr, load_all_answers_for_filter(z["snap"], R, rel), rel)
        apply_filter_(score, fp, fi)
        np.testing.assert_array_equal(score.numpy(), zm[ref_score])
        np.testing.assert_array_equal(make(tr, V, R, score, k), zm["snap_r" if rel else "snap_e"])


def test_dataset_directory_vs_reference(golden):
    """The reference's on-disk format read by the CLI loader (knowledge_graph.py:189-206,
    :526-555: num_nodes = len of the id-keyed dict, rows s r o t) and split into snapshots
    (rgcn/utils.py:306-339) as the reference's own load_from_local + split_by_time did on the
    same directory (tests/golden/tkg_tiny, tools/goldens/make_golden.py gen_dataset)."""
    import os
    from regcn_amd import cli, ranking
    z = golden("dataset_tiny.npz")
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    args = cli.build_parser().parse_args(["-d", "tkg_tiny", "--data-dir", root, "--test"])
    V, R, train, valid, test = cli.load_dataset(args)
    assert (V, R) == (int(z["num_nodes"]), int(z["num_rels"]))
    for name, arr in (("train", train), ("valid", valid), ("test", test)):
        np.testing.assert_array_equal(arr, z[name])
        snaps = ranking.split_by_time(arr)
        np.testing.assert_array_equal([len(s) for s in snaps], z[name + "_snap_len"])
        np.testing.assert_array_equal(np.concatenate(snaps), z[name + "_snaps"])


def test_bump_versions_restores_the_cache_key_after_a_fused_step():
    """Fused Adam updates parameters without bumping their version counters, which the packed
    weight and parameter-state caches key on; the CLI bumps them after each step
    (weights.bump_versions: x *= 1, a bitwise identity)."""
    import torch
    from regcn_amd.weights import bump_versions
    p = torch.nn.Parameter(torch.tensor([1.5, -0.0, 2.0, -3.0]))
    opt = torch.optim.Adam([p], lr=0.1, fused=True)
    p.grad = torch.ones(4)
    v0 = p._version
    opt.step()
    stepped = p.detach().clone()
    assert p._version == v0  # the contract fused optimizers break
    bump_versions([p, None])
    assert p._version > v0
    assert torch.equal(p.detach(), stepped) and torch.equal(torch.signbit(p.detach()), torch.signbit(stepped))


@pytest.mark.parametrize("block,chunk", [(512, 100), (64, 7), (100000, 256)])
def test_relation_entity_block_lists(block, chunk):
    """graph.rel_block_lists: every forward pair in exactly one chunk, a chunk inside one entity
    block, block k's chunks at dispatch positions p with (p // 4) % 8 == k % 8, and the
    chunk -> partial -> group -> fix-up walk (aggregate.hip k_gather_sum / k_fixup_groups /
    k_gather_fixup) giving each relation's mean."""
    rng = np.random.default_rng(block + chunk)
    R, V = 9, 6000
    lists = [np.unique(rng.integers(0, V, size=int(rng.integers(0, 4000)))) for _ in range(R)]
    lists[3] = np.zeros(0, np.int64)  # a relation absent from the snapshot
    lens = np.array([len(x) for x in lists])
    idx = np.concatenate(lists + lists)  # forward spans, then the inverse copies
    start = np.cumsum(lens) - lens
    ch, fx, ns = G.rel_block_lists(idx, start, lens, block, chunk=chunk)
    assert ch.dtype == np.int32 and fx.dtype == np.int32 and ch.shape[1] == 4
    covered = np.zeros(int(lens.sum()), np.int64)
    for r, b, e, s in ch:
        if e == b:
            assert s == ns - 1  # padding: the spare slot, read by no fix-up
            continue
        assert start[r] <= b < e <= start[r] + lens[r] and e - b <= chunk
        assert idx[b] // block == idx[e - 1] // block
        covered[b:e] += 1
    assert (covered == 1).all()
    p = np.arange(len(ch))
    real = ch[:, 2] > ch[:, 1]
    xcd, q = (p // 4) % 8, (p // 32) * 4 + p % 4  # the XCD a position's workgroup lands on, queue index
    blk = idx[ch[:, 1]] // block
    # the default deal (graph.XCD_DEAL = "cost"): each XCD's queue is a contiguous run of the
    # block-ordered chunks, the runs in XCD order
    last = -1
    for x in range(8):
        sel = real & (xcd == x)
        b = blk[sel][np.argsort(q[sel], kind="stable")]
        assert (np.diff(b) >= 0).all() and (len(b) == 0 or b[0] >= last)
        last = b[-1] if len(b) else last
    assert not ((fx[:, 1] <= ns - 1) & (fx[:, 2] > ns - 1)).any()
    x = rng.standard_normal((V, 5))
    part, out = np.zeros((ns, 5)), np.zeros((R, 5))
    for r, b, e, s in ch:
        acc = x[idx[b:e]].sum(0)
        if s < 0:
            out[r] = acc / lens[r]
        else:
            part[s] = acc
    for r, b, e, pad in fx:
        if pad > 0:
            part[pad - 1] = part[b:e].sum(0)
    for r, b, e, pad in fx:
        if pad == 0:
            out[r] = part[b:e].sum(0) / lens[r]
    ref = np.stack([x[l].mean(0) if len(l) else np.zeros(5) for l in lists])
    np.testing.assert_allclose(out, ref, rtol=1e-12, atol=1e-12)


def test_analysis_containers_on_host():
    """--run-analysis bookkeeping (regcn_amd/analysis.py) without a GPU: training_stats keeps the
    reference's keys and reads device-kept values as python numbers; the radius evolution's
    stats and the embedding stats are computed from per-row vectors like the reference's."""
    import torch
    from regcn_amd import analysis as A
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    m = HyperbolicRecurrentRGCN("roth", "hyperbolic_uvrgcn", 16, 4, 0, 0, 8, "sub", 3, num_bases=4,
                                num_hidden_layers=2, analysis=True)
    assert set(m.training_stats) == {"embedding_norms", "gradient_norms", "loss_components", "time_gate_values"}
    A.record_losses(m, torch.tensor([1.5]), torch.tensor([0.25]), torch.zeros(1), torch.tensor(0.125))
    assert m.training_stats["loss_components"] == [{"loss_ent": 1.5, "loss_rel": 0.25, "loss_static": 0.0,
                                                    "loss_radius": 0.125}]
    dict.__setitem__(m.training_stats, "time_gate_values", torch.tensor([0.25, 0.75]))
    assert m.training_stats["time_gate_values"] == [0.25, 0.75]
    delta, dyn, st = torch.tensor([0.1, -0.1, 0.05]), torch.tensor([1.0, 2.0, 3.0]), torch.tensor([2.0, 2.0, 2.0])
    base = 0.5 * st + 0.5 * dyn
    m.temporal_radius_evolution.last_evolution_stats = A.evolution_terms(delta, dyn, base, st, 0.5, 0.1)
    ev = m.temporal_radius_evolution.get_evolution_stats()
    assert abs(ev["delta_std"] - float(delta.std())) < 1e-7 and ev["base_radius_mean"] == 2.0
    s = m.get_training_summary()
    assert list(s) == ["curvature", "radius_delta_mean", "radius_delta_std", "dynamic_radius_mean",
                       "static_radius_mean", "base_radius_mean", "anchor_beta", "avg_time_gate"]
    assert abs(s["avg_time_gate"] - 0.5) < 1e-12 and abs(s["curvature"] - 0.01) < 1e-9
    r = torch.tensor([1.0, 9.5, 3.0])
    e = A.embedding_dict(A.embedding_stats(r, 0.01), "x", 0.01)
    assert abs(e["pct_near_boundary"] - 100.0 / 3) < 1e-4 and e["max_norm"] == 9.5
    for p in m.parameters():
        p.grad = torch.ones_like(p)
    gn = m.log_gradient_stats()
    assert abs(float(gn) - math.sqrt(sum(p.numel() for p in m.parameters()))) < 1e-3
    assert len(m.training_stats["gradient_norms"]) == 1


def test_loss_group_size_dense_fp64():
    """the dense fp64 decoder paths group DENSE_FP64_WORDS x fewer mini-batches than the fused CE."""
    import types
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN as M
    ns = types.SimpleNamespace(num_ents=23033, num_rels=256, use_relation_specific_curvature=False,
                               DENSE_FP64_WORDS=M.DENSE_FP64_WORDS)
    assert M._loss_group_size(ns, 1024, 1 << 28, False) == 5
    assert M._loss_group_size(ns, 1024, 1 << 28, True) == 1
    ns.use_relation_specific_curvature = True
    assert M._loss_group_size(ns, 1024, 1 << 28, False) == 1
    ns.num_ents = 500
    assert M._loss_group_size(ns, 64, 1 << 28, False) == (1 << 28) // (2 * 64 * 512 * M.DENSE_FP64_WORDS)


def test_spread_block_fills_every_xcd_queue():
    """a small key range (V < 8 blocks) with many pairs spreads its chunks over all 8
    XCD queues once the block is shrunk by graph.spread_block (the default block put them all in
    one queue and padded the other seven)."""
    rng = np.random.default_rng(1)
    V, R = 20000, 4
    lists = [np.unique(rng.integers(0, V, size=15000)) for _ in range(R)]
    lens = np.array([len(x) for x in lists])
    idx = np.concatenate(lists + lists)
    start = np.cumsum(lens) - lens
    fill = []
    for block in (G.REL_BLOCK * 8, G.spread_block(V, G.REL_BLOCK * 8)):
        ch, _, _ = G.rel_block_lists(idx, start, lens, block, chunk=256)
        p = np.arange(len(ch))
        real = ch[:, 2] > ch[:, 1]
        fill.append((np.bincount(((p // 4) % 8)[real], minlength=8) > 0).sum())
    assert fill[1] == 8, fill
    assert G.spread_block(V, 64) == 64 and G.spread_block(10 ** 6, 4096) == 4096


@pytest.mark.parametrize("deal", ["mod", "cost"])
def test_xcd_deal_balances_work(deal, monkeypatch):
    """graph.blocked_span_chunks' XCD queues over Zipf-skewed spans (one hot key block): "mod"
    puts block k on XCD k % 8 (every chunk of a block on one XCD); "cost" cuts the block-ordered
    chunks into 8 runs of equal positions + XCD_RUN_COST x key runs (config 5's hub pass:
    804 -> 750 us per launch), each XCD within one chunk's cost of the mean."""
    import torch
    monkeypatch.setattr(G, "XCD_DEAL", deal)
    rng = np.random.default_rng(7)
    V, n_spans = 50_000, 40
    p = 1.0 / np.arange(1, V + 1) ** 1.1
    p /= p.sum()
    spans = [np.sort(rng.choice(V, size=int(rng.integers(2000, 9000)), p=p)) for _ in range(n_spans)]
    lens = np.array([len(x) for x in spans])
    keys = torch.from_numpy(np.concatenate(spans))
    beg = torch.from_numpy(np.cumsum(lens) - lens)
    ch, _, _ = G.blocked_span_chunks(torch.arange(n_spans), beg, torch.from_numpy(lens), keys, 4096, 256)
    ch = ch.numpy().astype(np.int64)
    k = keys.numpy()
    pos = np.arange(len(ch))
    real = ch[:, 2] > ch[:, 1]
    xcd = (pos // 4) % 8
    if deal == "mod":
        assert (xcd[real] == (k[ch[real, 1]] // 4096) % 8).all()
        return
    runs = np.array([len(np.unique(k[b:e])) if e > b else 0 for _, b, e, _ in ch])
    cost = (ch[:, 2] - ch[:, 1]) + G.XCD_RUN_COST * runs
    per = np.bincount(xcd, weights=cost, minlength=8)
    assert per.max() - per.mean() <= cost.max(), (per, cost.max())


def test_rowtail_chunks_partition_tiles_and_rows():
    """hyperbolic_layers._rowtail_chunks (the two-stream rowtail pipeline): k chunks whose tile
    ranges partition the in-edge tiles and whose row ranges partition the row list, each row
    boundary at a tile start (a chunk's tail reads only rows its own gather finished)."""
    from regcn_amd import graph as G
    import torch
    from regcn_amd.hyperbolic_layers import _rowtail_chunks
    from regcn_amd.synthetic import zipf_triples
    rng = np.random.default_rng(2)
    V, R = 5000, 8
    host = G.build_sub_graph(V, R, zipf_triples(rng, V, R, 20000), False, "cpu")
    wk = {k: torch.from_numpy(np.asarray(host._host[k])) for k in ("tiles", "rows")}

    class Lists:  # the host lists behind the work() a device snapshot would give
        n_pos_tiles = host.n_pos_tiles

        def work(self):
            return wk

    g = Lists()
    n_t, n_rows = int(g.n_pos_tiles), int(wk["rows"].shape[0])
    starts = wk["tiles"][:n_t, 0].tolist()
    for k in (1, 3, 6):
        ch = _rowtail_chunks(g, k)
        assert len(ch) == min(k, n_t)
        assert ch[0][0] == 0 and ch[-1][1] == n_t and ch[0][2] == 0 and ch[-1][3] == n_rows
        for (t0, t1, r0, r1), nxt in zip(ch, ch[1:] + [None]):
            assert t0 < t1 and r0 <= r1
            if nxt is not None:
                assert nxt[0] == t1 and nxt[2] == r1 and r1 == starts[t1]


def test_hub_chunk_size():
    """graph.hub_chunk: the snapshot's chunk size for a whole config-5 snapshot's hubs (32.7M
    edges), shrunk towards 256 for an owner rank's eighth so the pass keeps >= 16k chunks."""
    assert G.hub_chunk(32_700_000, 1024) == 1024
    assert G.hub_chunk(4_100_000, 1024) == 256
    assert G.hub_chunk(8_000_000, 1024) == 489
    assert G.hub_chunk(1 << 20, None) == 256
