"""A whole sharded predict (-m gpu): two ranks launched like the driver launches bench.py
(torch.distributed.run), sharing the box's one GPU through a gloo group (on a node each rank
owns a GPU and the group is RCCL).  Both partitions of SURVEY.md §8(e) -- owner (with and
without the pipelined exchange: per chunk one all_to_all of the rows the next layer reads,
parallel.ExchangePlan) and edge -- against the same model unsharded: history
embeddings within 1e-4 * max(1, |ref|), relation states within 1e-5; the candidate-sharded
decoder on the unsharded embeddings gives the unsharded ranks bit for bit, and end to end the
entity ranks differ (near ties) for at most 1% of the queries, by at most 2."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag,rowtail", [("uvrgcn_roth_r512_d200", False), ("lgcn_roth_h7_d200", False),
                                         ("uvrgcn_roth_e80k_d200", True)])
def test_sharded_predict_world2(tmp_path, tag, rowtail):
    """rowtail: the large-snapshot layer path (REGCN_ROWTAIL_MIN_ROWS lowered in the ranks),
    where a rank's hub pass and gather run once and each chunk's tail is followed by its
    exchange (hyperbolic_layers.run_layer_chunked)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "res.json")
    env = dict(os.environ, PYTHONPATH=os.path.join(repo, "re-gcn_amd") + os.pathsep + repo,
               REGCN_DIST_BACKEND="gloo")
    if rowtail:
        env["REGCN_ROWTAIL_MIN_ROWS"] = "1"
        env["REGCN_ROWTAIL_MIN_VIEW_ROWS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(repo, "tests", "sharded_predict_job.py"), out, tag]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.load(open(out))
    assert res["world"] == 2
    for key in ("owner_1", "owner_3", "edge_1"):
        v = res[key]
        assert v["emb_err"] <= 1e-4, (key, v)
        assert v["h0_err"] <= 1e-5, (key, v)
        assert v["dec_ent_rank_equal"] and v["dec_rel_rank_equal"], (key, v)
        assert v["ent_rank_queries_differing"] <= 0.01 * v["queries"] and v["ent_rank_max_diff"] <= 2, (key, v)
    a = res["owner_analysis"]  # --run-analysis (the non-fused timestep) under the owner partition
    assert a["emb_err"] <= 1e-4 and a["hist_err"] <= 1e-4 and a["gate_err"] <= 1e-4, a
    print(res)


def test_cli_sharded_evaluation_world2():
    """`--test --shard owner` under torch.distributed.run (two ranks, gloo on the one GPU):
    every rank evaluates its partition and candidate slice; the logged MRRs match the
    single-process evaluation of the same seeded model within the north star's 0.002."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import re
    from regcn_amd import cli
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    argv = ["-d", "synthetic:icews14s_lgcn_roth", "--test", "--gpu", "0", "--encoder", "lgcn", "--decoder", "roth",
            "--n-hidden", "64", "--n-bases", "32", "--synthetic-snapshots", "8", "--test-history-len", "3",
            "--relation-prediction", "--entity-prediction", "--seed", "0"]
    single = cli.main(argv)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=os.path.join(repo, "re-gcn_amd"), REGCN_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "regcn_amd.cli"] + argv + ["--shard", "owner"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    found = re.findall(r"MRR raw ([0-9.]+) filter ([0-9.]+) \| relation raw ([0-9.]+) filter ([0-9.]+)",
                       r.stdout + r.stderr)
    assert len(found) == 2, (r.stdout + r.stderr)[-2000:]  # both ranks report the same pass
    for got in found:
        for a, b in zip((float(v) for v in got), single):
            assert abs(a - b) <= 0.002, (got, single)


@pytest.mark.parametrize("tag,world,chunks,rowtail", [("uvrgcn_roth_r512_d200", 8, 2, False),
                                                      ("lgcn_roth_h7_d200", 3, 1, False),
                                                      ("uvrgcn_roth_e80k_d200", 4, 3, False),
                                                      ("uvrgcn_roth_e80k_d200", 4, 3, True),
                                                      ("lgcn_roth_h7_d200", 2, 2, True)])
def test_rank_simulation_matches_unsharded(golden, tag, world, chunks, rowtail, monkeypatch):
    """The owner partition's per-rank work, all ranks run one after another on the GPU
    (parallel.RankSimulation, bench.py's owner_simulation): each rank's chunk views of every
    layer and its partial relation means, combined, give the unsharded history embeddings
    (1e-4 * max(1, |ref|)) and relation states; a balanced relabel of the entities
    (EntityRelabel) changes nothing but the row order.  rowtail: the large-snapshot layer path
    (threshold lowered), where a rank's hub pass and gather run once over all of its rows and
    only the tails per chunk (hyperbolic_layers.run_layer_chunked), and each chunk's tail also
    writes the send block of its halo exchange (regcn_layer_desc send_*): equal bit for bit to
    gathering the rows after it (regcn_gather_rows_f32)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    if rowtail:
        from regcn_amd import hyperbolic_layers as HL
        monkeypatch.setattr(HL, "ROWTAIL_MIN_ROWS", 1)
        monkeypatch.setattr(HL, "ROWTAIL_MIN_VIEW_ROWS", 1)
    import numpy as np
    from gpu_helpers import assert_close, build_hyperbolic_model
    from regcn_amd import graph as G
    from regcn_amd.parallel import EntityRelabel, RankSimulation
    dev = torch.device("cuda", 0)
    z = golden("model_%s.npz" % tag)
    m, glist, (V, R, d, T) = build_hyperbolic_model(z, tag, dev)
    with torch.no_grad():
        embs, _, h0, _, _ = m.forward(glist, None, True)
        ref = embs[-1].clone()
        sims = [RankSimulation(g, world, chunks) for g in glist]
        for sm in sims:
            sm.keep_sends = True
        e2, _, h02, _, _ = m.forward(sims, None, True)
        assert_close(e2[-1], ref, what="simulated ranks")
        sends = [s for sm in sims for s in sm.sends]
        assert bool(sends) == rowtail
        for (xs, r1), xn, rn, ids in sends:
            assert torch.equal(xs, xn.index_select(0, ids)) and torch.equal(r1, rn.index_select(0, ids))
        assert_close(h02, h0, 1e-5, "relation state")
        assert all(len(t) for sm in sims for t in sm.times)
        snaps = [z["snap%d" % t] for t in range(T)]
        rl = EntityRelabel.balanced(snaps, V, world, chunks)
        rl.model(m)
        gl = [G.build_sub_graph(V, R, rl.triples(s).astype(np.int64), True, dev) for s in snaps]
        e3 = m.forward([RankSimulation(g, world, chunks) for g in gl], None, True)[0]
        assert_close(e3[-1][torch.from_numpy(rl.perm).to(dev)], ref, what="relabelled simulated ranks")


def test_rccl_device_branches_world1(tmp_path):
    """The RCCL branches of the owner exchange (parallel._all_to_all_into's all_to_all_single
    and _all_gather_into's all_gather_into_tensor on device tensors, launched on the comm
    stream as ShardedGraph.run_layer launches them) in a one-rank "nccl" group: exact against
    the known one-rank result and equal bit for bit to the gloo branch of the same calls
    (tests/nccl_world1_job.py).  Two ranks cannot share the box's one GPU under RCCL."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "res.json")
    env = dict(os.environ, PYTHONPATH=os.path.join(repo, "re-gcn_amd") + os.pathsep + repo)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(repo, "tests", "nccl_world1_job.py"),
           out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.load(open(out))
    assert res["backend"] == "nccl" and res["world"] == 1, res
    assert res["nccl_exchange_exact"] and res["nccl_allgather_exact"] and res["nccl_equals_gloo"], res


@pytest.mark.parametrize("n,d", [(1, 200), (37, 200), (5000, 200), (129, 12)])
def test_gather_rows_matches_index_select(n, d):
    """The halo exchange's send-side gather (regcn_gather_rows_f32): rows `ids` of x and |h|,
    repeated and unsorted ids included, equal index_select bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from regcn_amd import parallel as P
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(n + d)
    V = 3 * n + 7
    x = torch.randn(V, d, generator=g).to(dev)
    r = torch.rand(V, generator=g).to(dev)
    ids = torch.randint(0, V, (n,), generator=g).to(dev)
    xs, r1 = P.gather_rows(x, r, ids)
    torch.cuda.synchronize()
    assert torch.equal(xs, x.index_select(0, ids)) and torch.equal(r1, r.index_select(0, ids))


@pytest.mark.parametrize("ln,d", [(0, 200), (1, 200), (0, 37)])
def test_init_entity_rows_match_the_full_map(ln, d):
    """regcn_init_entity_rows_f32 (the owner partition's initial rows: a rank's own rows at
    their ids, its halo compacted at rows Vp..): every listed row equal bit for bit to the same
    row of regcn_init_entities_f32 over all rows; unlisted rows untouched; h may be skipped."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from regcn_amd import _lib
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(d + ln)
    V, c = 5003, 0.7
    dyn = (0.3 * torch.randn(V, d, generator=g)).to(dev)
    rs = (0.2 + torch.rand(V, generator=g)).to(dev)
    f, i = _lib.fptr, _lib.iptr
    h, x, r = torch.empty(V, d, device=dev), torch.empty(V, d, device=dev), torch.empty(V, device=dev)
    _lib.call("regcn_init_entities_f32", f(dyn), f(rs), V, d, c, ln, f(h), f(x), f(r), _lib.stream())
    ids = torch.randperm(V, generator=g)[:1777].to(torch.int32).to(dev)
    h2, x2 = torch.full_like(h, float("nan")), torch.full_like(x, float("nan"))
    r2 = torch.full_like(r, float("nan"))
    _lib.call("regcn_init_entity_rows_f32", f(dyn), f(rs), i(ids), i(ids), ids.numel(), d, c, ln, f(h2), f(x2),
              f(r2), _lib.stream())
    xc, rc = torch.empty(ids.numel(), d, device=dev), torch.empty(ids.numel(), device=dev)
    _lib.call("regcn_init_entity_rows_f32", f(dyn), f(rs), i(ids), None, ids.numel(), d, c, ln, None, f(xc),
              f(rc), _lib.stream())
    torch.cuda.synchronize()
    li = ids.long()
    assert torch.equal(h2[li], h[li]) and torch.equal(x2[li], x[li]) and torch.equal(r2[li], r[li])
    rest = torch.ones(V, dtype=torch.bool, device=dev)
    rest[li] = False
    assert bool(torch.isnan(h2[rest]).all() and torch.isnan(x2[rest]).all() and torch.isnan(r2[rest]).all())
    assert torch.equal(xc, x[li]) and torch.equal(rc, r[li])
