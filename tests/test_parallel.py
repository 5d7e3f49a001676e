"""Multi-GPU partitions (regcn_amd/parallel.py) on CPU: the plans, and the collectives of
both partitions in a world-size-2 gloo job.  The per-rank compute between
the collectives is the HIP library (covered on the GPU by test_gpu_parity.py, ranks
simulated on one device); here a test-local segment sum stands in for it so that the
partition + all-reduce / all-gather algebra is checked against the unpartitioned sum."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from regcn_amd import graph as G
from regcn_amd import parallel as P


def _snapshot(V=300, R=7, T=2500, seed=0):
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, V + 1) ** 1.2
    p /= p.sum()
    tr = np.stack([rng.choice(V, T, p=p), rng.integers(0, R, T), rng.choice(V, T, p=p)], 1)
    return G.build_sub_graph(V, R, tr, False, 0, chunk_edges=16)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_edge_plan_covers_every_edge_once(world):
    g = _snapshot()
    E = g.number_of_edges()
    rowptr = g._host["rowptr"].astype(np.int64)
    cov = np.zeros(E, dtype=np.int64)
    for rank in range(world):
        pl = P.EdgePlan(g, rank, world)
        assert pl.e0 <= pl.e1 and pl.e1 - pl.e0 <= E // world + 1  # balanced by edges
        slots = []
        for row, b, e, s in pl.chunks:
            assert rowptr[row] <= b < e <= rowptr[row + 1] and pl.e0 <= b and e <= pl.e1
            assert e - b <= g.chunk_edges
            cov[b:e] += 1
            slots.append(s)
        assert sorted(slots) == list(range(len(slots)))
        group_of = {int(o) - 1: (int(b), int(e)) for _, b, e, o in pl.fixups if o > 0}
        assert sorted(group_of) == list(range(len(slots), pl.n_slots))
        for row, sb, se, o in pl.fixups:  # each touched row sums exactly its own slots
            if o > 0:
                continue
            covered = set()
            for s_ in range(sb, se):
                b, e = group_of.get(s_, (s_, s_ + 1))
                covered |= set(range(b, e))
            assert set(pl.chunks[(pl.chunks[:, 0] == row), 3]) == covered
        fin = pl.finish
        assert (fin[:, 1] == fin[:, 0]).all() and (fin[:, 2] == fin[:, 0] + 1).all()
        np.testing.assert_array_equal(np.sort(fin[:, 0]), np.nonzero(g.in_deg_np > 0)[0])
    assert (cov == 1).all()


@pytest.mark.parametrize("world,chunks", [(1, 1), (2, 1), (3, 2), (8, 4)])
def test_owner_views_partition_the_nodes(world, chunks):
    g = _snapshot()
    V = g.number_of_nodes()
    lay = P.OwnerLayout(V, world, chunks)
    seen = []
    for rank in range(world):
        for j, (lo, hi) in enumerate(lay.ranges(rank)):
            assert (lo, hi) == lay.group(rank, j) and hi - lo <= lay.cr
            assert lo == hi or (lo // lay.cr == j * world + rank and (P.OwnerLayout(V, world, chunks).owner(
                np.arange(lo, hi)) == rank).all())
            v = P.OwnerView(g, lo, hi)
            rows = v.fw.host["rows"]
            assert ((rows >= lo) & (rows < hi)).all()
            assert v.n_pos == int((g.in_deg_np[rows] > 0).sum())
            # the view's items are exactly the in-edges of its inline rows
            n_inline = int(np.where(g.in_deg_np[rows[:v.n_pos]] > g.budget, 0, g.in_deg_np[rows[:v.n_pos]]).sum())
            assert v.fw.host["item_ptr"][-1] == n_inline
            seen += rows.tolist()
    assert sorted(seen) == list(range(V))
    # chunk j of every rank is one contiguous id range (its all-gather lands in place)
    for j in range(chunks):
        rs = [lay.group(k, j) for k in range(world)]
        for (a0, b0), (a1, b1) in zip(rs, rs[1:]):
            assert b0 == a1 or a1 == b1


def test_lpt_balances_and_respects_capacities():
    rng = np.random.default_rng(3)
    n = 80_000
    load = np.floor(1e6 / np.arange(1, n + 1) ** 1.1)[rng.permutation(n)]
    caps = np.array([n // 4] * 3 + [n - 3 * (n // 4)])
    g = P._lpt(load, caps, head=4000)
    assert (np.bincount(g, minlength=4) == caps).all()
    tot = np.bincount(g, weights=load, minlength=4)
    # the heaviest item is below a fair share here: every group within 2 % of the mean
    assert load.max() < load.sum() / 4 and tot.max() <= 1.02 * load.sum() / 4, tot / (load.sum() / 4)


@pytest.mark.parametrize("world", [2, 8])
def test_entity_relabel_balances_edges(world):
    """EntityRelabel.balanced: a permutation; per-rank in-edge loads of every snapshot within a
    few percent of the mean under Zipf(1.1) (equal contiguous id blocks are far off); the model
    tensors and triples relabel consistently (new row perm[i] = old row i)."""
    from regcn_amd.synthetic import snapshot_series
    V = 200_000
    snaps = snapshot_series(1, V, 16, 2, 400_000)
    rl = P.EntityRelabel.balanced(snaps, V, world)
    assert np.array_equal(np.sort(rl.perm), np.arange(V))
    for row in rl.loads(snaps, world):
        assert max(row) <= 1.03 * np.mean(row), row
    plain = P.EntityRelabel(np.arange(V)).loads(snaps, world)
    imb = lambda rows: max(max(r) / np.mean(r) for r in rows)  # noqa: E731
    assert imb(rl.loads(snaps, world)) < imb(plain) and (world < 8 or imb(plain) > 1.1)
    tr = rl.triples(snaps[0][:50])
    assert (tr[:, 0] == rl.perm[snaps[0][:50, 0]]).all() and (tr[:, 1] == snaps[0][:50, 1]).all()
    m = torch.nn.Module()
    m.dynamic_emb = torch.nn.Parameter(torch.arange(V, dtype=torch.float32).unsqueeze(1).repeat(1, 2))
    m.register_buffer("radius_target", torch.arange(V, dtype=torch.float32))
    rl.model(m)
    assert torch.equal(m.radius_target[torch.from_numpy(rl.perm)], torch.arange(V, dtype=torch.float32))
    assert torch.equal(m.dynamic_emb[torch.from_numpy(rl.perm), 0], torch.arange(V, dtype=torch.float32))


def test_owned_relation_spans_cover_each_pair_once():
    """The partitioned relation means: every forward (relation, entity) pair lies in exactly one
    rank's spans, each span inside its id range (the ranks' partial sums add up to the sums)."""
    rng = np.random.default_rng(0)
    R, V = 6, 500
    spans = [np.unique(rng.integers(0, V, rng.integers(0, 80))) for _ in range(R)]
    idx = torch.from_numpy(np.concatenate(spans + spans)).int()  # forward lists, then inverse copies
    cnt = torch.tensor([len(x) for x in spans], dtype=torch.float32)
    start = np.concatenate([[0], np.cumsum([len(x) for x in spans])])
    for world, chunks in ((2, 1), (3, 2), (8, 4)):
        lay = P.OwnerLayout(V, world, chunks)
        hit = np.zeros(int(cnt.sum()), np.int64)
        for k in range(world):
            ranges = lay.ranges(k)
            rows, beg, ln = P.owned_rel_spans(idx, cnt, ranges, lay.Vp)
            for row, b, n in zip(rows.tolist(), beg.tolist(), ln.tolist()):
                r, q = divmod(row, len(ranges))
                assert start[r] <= b and b + n <= start[r + 1]
                lo, hi = ranges[q]
                assert ((idx[b:b + n] >= lo) & (idx[b:b + n] < hi)).all()
                hit[b:b + n] += 1
        assert (hit == 1).all()


def _segment_sum_slice(g, pl, x, rel):
    """Test-local stand-in for the HIP partial kernels: raw Euclidean partial sums of the
    plan's edge slice, summed per row (what regcn_partial_sum_f32 leaves in P)."""
    src = torch.from_numpy(g._host["col_src"].astype(np.int64))
    typ = torch.from_numpy(g._host["col_type"].astype(np.int64))
    rowptr = g._host["rowptr"].astype(np.int64)
    dst = torch.from_numpy(np.repeat(np.arange(len(rowptr) - 1), np.diff(rowptr)))
    sl = slice(pl.e0, pl.e1)
    out = torch.zeros(x.shape[0], x.shape[1], dtype=torch.float64)
    out.index_add_(0, dst[sl], (x[src[sl]] + rel[typ[sl]]).double())
    return out


def _worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = _snapshot()
        V, d = g.number_of_nodes(), 12
        gen = torch.Generator().manual_seed(5)
        x = torch.randn(V, d, generator=gen)
        rel = torch.randn(2 * g.num_rels, d, generator=gen)
        # edge partition: every rank's partials, all-reduced, equal the full segment sum
        pl = P.EdgePlan(g, rank, world)
        part = _segment_sum_slice(g, pl, x, rel)
        P.allreduce_partials(part)
        full = _segment_sum_slice(g, P.EdgePlan(g, 0, 1), x, rel)
        err_edge = float((part - full).abs().max())
        # owner partition: each rank fills its node block, the all-gather rebuilds all rows
        per, bounds = P.owner_bounds(V, world)
        buf = torch.full((per * world, d), float("nan"))
        ref = torch.arange(V * d, dtype=torch.float32).view(V, d)
        buf[bounds[rank]:bounds[rank + 1]] = ref[bounds[rank]:bounds[rank + 1]]
        P.allgather_rows(buf, per)
        err_owner = float((buf[:V] - ref).abs().max())
        # the pipelined exchange of ShardedGraph.run_layer: OwnerLayout with 3 chunks per rank,
        # after each chunk the in-place all-gather of chunk j of every rank (x rows and radii)
        lay = P.OwnerLayout(V, world, 3)
        xx = torch.full((lay.Vp, d), float("nan"))
        rr = torch.full((lay.Vp,), float("nan"))
        cr = lay.cr
        for j, (lo, hi) in enumerate(lay.ranges(rank)):
            xx[lo:hi], rr[lo:hi] = -ref[lo:hi], ref[lo:hi, 0]
            a, b, k = j * world * cr, (j + 1) * world * cr, (j * world + rank) * cr
            P._all_gather_into(xx[a:b], xx[k:k + cr])
            P._all_gather_into(rr[a:b], rr[k:k + cr])
        err_owner = max(err_owner, float((xx[:V] + ref).abs().max()), float((rr[:V] - ref[:, 0]).abs().max()))
        # fetch_rows' exchange: the owner's rows in one all_reduce with zeros elsewhere
        ids = torch.tensor([0, V - 1, 17, 123, 17])
        got = torch.zeros(len(ids), d)
        mine = lay.owner(ids) == rank
        got[mine] = ref[ids[mine]]
        P.allreduce_partials(got)
        err_owner = max(err_owner, float((got - ref[ids]).abs().max()))
        result_q.put((rank, err_edge, err_owner))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_collectives_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(2))
    for rank, err_edge, err_owner in res:
        assert err_edge < 1e-9, (rank, err_edge)
        assert err_owner == 0.0, (rank, err_owner)


def _lse_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(0)
        S = torch.randn(5, 20, generator=g, dtype=torch.float64)
        sl = S[:, rank * 10:(rank + 1) * 10]
        lse = P.combine_lse(torch.logsumexp(sl, 1))
        cnt = P.combine_counts((sl > 0.1).sum(1))
        err = float((lse - torch.logsumexp(S, 1)).abs().max())
        q.put((rank, err, bool(torch.equal(cnt, (S > 0.1).sum(1)))))
    finally:
        dist.destroy_process_group()


def test_decoder_shard_collectives_gloo():
    """combine_lse / combine_counts (the B-sized exchanges of the candidate-sharded decoder,
    SURVEY.md §8(e)) over a world-2 gloo group equal the unsharded log-sum-exp and counts."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_lse_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, err, ok in sorted(q.get() for _ in range(2)):
        assert err < 1e-12 and ok, (rank, err, ok)


def test_shard_filters():
    ptr = np.array([0, 3, 3, 5], np.int32)
    idx = np.array([1, 7, 12, 0, 9], np.int32)
    p, i = P.shard_filters(ptr, idx, 5, 10)
    np.testing.assert_array_equal(p, [0, 1, 1, 2])
    np.testing.assert_array_equal(i, [2, 4])


def _replica_worker(rank, world, port, q):
    """Two replicas, different samples, one flattened gradient all-reduce per step: the
    parameters after three Adam steps equal one process stepping on the mean loss."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(1234 + rank)  # different init: broadcast_state must align them
        m = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
        m.register_buffer("unused_grad_holder", torch.zeros(1))
        extra = torch.nn.Parameter(torch.ones(2))  # never used: zero gradient on every rank
        P.broadcast_state(m)
        ref = [p.detach().clone() for p in m.parameters()]
        params = list(m.parameters()) + [extra]
        # weight decay on, as the CLI's Adam (hyperbolic_main.py:469): a parameter no rank
        # produced a gradient for must keep grad=None and so stay untouched
        opt = torch.optim.Adam(params, lr=1e-2, weight_decay=1e-5)
        g = torch.Generator().manual_seed(0)
        X = torch.randn(3, world, 4, 6, generator=g)
        for step in range(3):
            opt.zero_grad()
            m(X[step, rank]).pow(2).mean().backward()
            n = P.allreduce_gradients(params)
            assert extra.grad is None
            opt.step()
        assert torch.equal(extra.detach(), torch.ones(2))
        q.put((rank, n, [p.detach().numpy().copy() for p in m.parameters()], [r.numpy() for r in ref]))
    finally:
        dist.destroy_process_group()


def test_replica_gradients_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_replica_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted((q.get() for _ in range(2)), key=lambda t: t[0])
    (_, n0, p0, init), (_, n1, p1, _) = res
    assert n0 == n1 == 6 * 5 + 5 + 5 * 3 + 3 + 2
    for a, b in zip(p0, p1):
        np.testing.assert_array_equal(a, b)
    # single-process replay: mean of the two replicas' losses
    m = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
    with torch.no_grad():
        for p, v in zip(m.parameters(), init):
            p.copy_(torch.from_numpy(v))
    opt = torch.optim.Adam(m.parameters(), lr=1e-2, weight_decay=1e-5)
    g = torch.Generator().manual_seed(0)
    X = torch.randn(3, 2, 4, 6, generator=g)
    for step in range(3):
        opt.zero_grad()
        (0.5 * sum(m(X[step, r]).pow(2).mean() for r in range(2))).backward()
        opt.step()
    for a, b in zip(m.parameters(), p0):
        assert float((a.detach() - torch.from_numpy(b)).abs().max()) < 1e-6


def _pack_cpu(xn, rn, ids):  # torch stand-ins for regcn_pack_rows_f32 / regcn_unpack_rows_f32
    d = xn.shape[1]
    out = torch.zeros(ids.numel(), d + 4)
    out[:, :d], out[:, d] = xn[ids], rn[ids]
    return out


def _unpack_cpu(buf, ids, xn, rn):
    d = xn.shape[1]
    xn[ids], rn[ids] = buf[:, :d], buf[:, d]


def _exchange_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = _snapshot(V=400, T=3000, seed=world)
        V, d = g.number_of_nodes(), 6
        ref = torch.arange(V * d, dtype=torch.float32).view(V, d) + 0.5
        ok = True
        for chunks in (1, 3):
            lay = P.OwnerLayout(V, world, chunks)
            plan = P.ExchangePlan(g, lay, rank)
            xn = torch.full((lay.Vp, d), float("nan"))
            rn = torch.full((lay.Vp,), float("nan"))
            for j, (lo, hi) in enumerate(lay.ranges(rank)):
                xn[lo:hi], rn[lo:hi] = ref[lo:hi], -ref[lo:hi, 0]
                P.exchange_rows(plan.chunks[j], xn, rn, pack=_pack_cpu, unpack=_unpack_cpu)
            # every source of an in-edge of this rank's rows is valid, and nothing else arrived
            rowptr = g._host["rowptr"].astype(np.int64)
            src = g._host["col_src"].astype(np.int64)[:rowptr[-1]]
            dst = np.repeat(np.arange(V), np.diff(rowptr))
            mine = lay.owner(np.arange(V)) == rank
            need = np.zeros(V, bool)
            need[src[mine[dst]]] = True
            need |= mine
            got = ~torch.isnan(xn[:V, 0]).numpy()
            ok &= bool((got == need).all())
            ok &= bool(torch.equal(xn[:V][need], ref[need]) and torch.equal(rn[:V][need], -ref[need, 0]))
            ok &= plan.rows_received() == int((need & ~mine).sum())
            # the halo exchange: the received rows land at rows Vp + halo_off[j] .. in the plan's
            # halo order, and the remap sends every in-edge source of this rank's rows there
            H = plan.halo.numel()
            xh = torch.full((lay.Vp + H, d), float("nan"))
            rh = torch.full((lay.Vp + H,), float("nan"))
            for j, (lo, hi) in enumerate(lay.ranges(rank)):
                xh[lo:hi], rh[lo:hi] = ref[lo:hi], -ref[lo:hi, 0]
                P.exchange_halo(plan, j, xh, rh, lay.Vp, gather=lambda x_, r_, i_: (x_[i_], r_[i_]))
            m = plan.remap(V, lay.Vp).numpy()
            srcs = src[mine[dst]]
            ok &= bool(torch.equal(xh[torch.from_numpy(m[srcs])], ref[srcs]))
            ok &= bool(torch.equal(rh[torch.from_numpy(m[srcs])], -ref[srcs, 0]))
            ok &= bool((m[mine] == np.nonzero(mine)[0]).all()) and bool((m[need & ~mine] >= lay.Vp).all())
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sparse_exchange_gloo(world):
    """ExchangePlan + exchange_rows (the owner partition's per-chunk all_to_all): after every
    chunk's exchange a rank holds exactly its own rows and the sources of its rows' in-edges,
    with the owners' values; senders and receivers agree on the order.  The
    halo exchange (exchange_halo: two all_to_alls straight into the rows after Vp) delivers the
    same rows where ExchangePlan.remap points the consumer's source ids."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(world))
    assert all(ok for _, ok in res), res


def test_exposed_exchange_model():
    """The rank simulation's link model (parallel.exposed_after): exchanges shorter than the
    next chunk's compute hide except the last; longer ones queue on the link."""
    assert P.exposed_after([0.0, 1.0, 2.0, 3.0], [0.5] * 4) == pytest.approx(0.5)
    # 4 chunks of 0.09 ms compute, 0.164 ms exchanges: 0.657 - 3 * 0.09 exposed
    t = [0.0, 0.09, 0.18, 0.27]
    assert P.exposed_after(t, [0.164] * 4) == pytest.approx(4 * 0.164 - 0.27)
    assert P.exposed_after([0.0], [0.2]) == pytest.approx(0.2)
    assert P.exposed_after([0.0, 1.0], [0.0, 0.0]) == 0.0


@pytest.mark.parametrize("decoder", ["hyperbolic_convtranse", "roth"])
def test_entity_relabel_permutes_every_entity_tensor(decoder):
    """EntityRelabel.model permutes every parameter / buffer indexed by entity id of a real
    model -- incl. HyperbolicConvTransE's per-entity bias `decoder_ob.b` (hyperbolic_decoder.py
    :568) and RotH's Euclidean `decoder_ob.entity_bias` -- so a relabelled model scores entity
    perm[i] exactly as the original scores entity i; every other tensor is unchanged."""
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    V, R = 40, 3
    torch.manual_seed(0)
    m = HyperbolicRecurrentRGCN(decoder, "hyperbolic_uvrgcn", V, R, 0, 0, 8, "sub", 3, num_bases=4,
                                num_hidden_layers=2, self_loop=True, entity_prediction=True, relation_prediction=True,
                                use_entity_euclidean_bias=decoder == "roth")
    with torch.no_grad():
        for t in list(m.parameters()) + list(m.buffers()):
            if t.is_floating_point():
                t.copy_(torch.randn_like(t))
    before = {k: v.clone() for k, v in m.state_dict().items()}
    perm = np.random.default_rng(2).permutation(V)
    P.EntityRelabel(perm).model(m)
    after = m.state_dict()
    p = torch.from_numpy(perm)
    moved = set()
    for k, v in before.items():
        if k in P.EntityRelabel.ENTITY_TENSORS:
            assert torch.equal(after[k][p], v), k
            moved.add(k)
        else:
            assert torch.equal(after[k], v), k
    per_entity = {k for k, v in before.items() if v.dim() >= 1 and v.shape[0] == V}
    assert per_entity == moved, per_entity ^ moved
    assert ("decoder_ob.b" in moved) == (decoder == "hyperbolic_convtranse")


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 3), (4, 2)])
def test_send_slots_cover_the_send_list(world, chunks):
    """ExchangePlan.send_slots / send_block (the send block a chunk's tail writes itself,
    regcn_layer_desc.send_*): scattering every row of chunk j to its slots reproduces chunk j's
    send list gathered in order (one slot per receiver that reads the row), for every rank."""
    g = _snapshot(V=400, T=3000, seed=world)
    V, d = g.number_of_nodes(), 5
    ref = torch.arange(V * d, dtype=torch.float32).view(V, d) + 0.25
    lay = P.OwnerLayout(V, world, chunks)
    for rank in range(world):
        plan = P.ExchangePlan(g, lay, rank)
        for j, (lo, hi) in enumerate(lay.ranges(rank)):
            sidx = plan.chunks[j][0]
            sb = plan.send_block(j, lo, hi - lo, d)
            if sb is None:
                assert sidx.numel() == 0
                continue
            (lo_, n, ptr, pos, xs, r1), blk = sb
            assert (lo_, n) == (lo, hi - lo) and blk[0] is xs and blk[1] is r1
            assert ptr.dtype == torch.int32 and pos.dtype == torch.int32 and int(ptr[-1]) == sidx.numel()
            rows = lo + torch.repeat_interleave(torch.arange(n), (ptr[1:] - ptr[:-1]).long())
            xs[pos.long()] = ref[rows]
            r1[pos.long()] = -ref[rows, 0]
            assert torch.equal(xs, ref[sidx]) and torch.equal(r1, -ref[sidx, 0])
            assert sorted(pos.tolist()) == list(range(sidx.numel()))
