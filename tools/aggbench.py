"""Aggregation at the HBM-roofline stress scale (|V| = 1M,
|E| = 50M directed edges per snapshot, R = 256, d = 200) on one GPU.

Times, as graph-replayed launches between HIP events (bench.event_time):
  union aggregation alone   regcn_union_aggregate_f32 over every chunk of the snapshot
  lorentz aggregation alone regcn_lorentz_aggregate_f32 (2x2 block messages + centroid)
  fused layers              HyperbolicUnionRGCNLayer / LorentzRGCNLayer forward (gather + GEMMs)
and reports algorithmic bytes B_agg = E (4d + 12) + V (4d + 12) per aggregation over the time,
as GB/s and as a fraction of the 8 TB/s HBM peak.  The Lorentz aggregation reads the
row/type edge order (graph.row_type_cols); `lorentz_aggregate_csr` times the edge-id order.
--cpu adds the CPU oracle's layers at |V| = 1M, |E| = 5M.

  python tools/aggbench.py [--V 1000000] [--triples 25000000] [--reps 3] [--cpu] [--which ...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
sys.path.insert(0, REPO)
from bench import HBM_PEAK_GBS, event_time  # noqa: E402
from regcn_amd import _lib  # noqa: E402
from regcn_amd import graph as G  # noqa: E402
from regcn_amd.hyperbolic_layers import HyperbolicUnionRGCNLayer, LorentzRGCNLayer  # noqa: E402
from regcn_amd.hyperbolic_ops import HyperbolicOps as H  # noqa: E402
from regcn_amd.synthetic import snapshot_series  # noqa: E402

C = 0.01


def measure(V=1_000_000, R=256, triples=25_000_000, d=200, reps=3, dev=None,
            which=("union_aggregate", "union_layer", "lorentz_aggregate", "lorentz_layer"), log=print,
            uniform_s=False):
    """Times the named launches on a synthetic config-5 snapshot; returns the result dict.
    uniform_s: subjects uniform (objects Zipf), so the hub rows' gathered sources are spread
    over the whole table and really come from HBM."""
    dev = dev or torch.device("cuda", 0)
    t0 = time.time()
    snap = snapshot_series(0, V, R, 1, triples, uniform_s=uniform_s)[0]
    g = G.build_sub_graph(V, R, snap, True, dev)
    del snap
    E = g.number_of_edges()
    wk = g.work()
    log("graph: V=%d E=%d pos=%d tiles=%d heavy=%d chunks=%d built in %.1f s"
        % (V, E, g.n_pos, g.n_pos_tiles, g.n_heavy, wk["chunks"].shape[0], time.time() - t0))
    torch.manual_seed(0)
    h = H.apply_radius(H.exp_map_zero(torch.randn(V, d, device=dev), C),
                       torch.rand(V, 1, device=dev) * 2.5 + 0.5, C)
    x = H.log_map_zero(h, C).contiguous()
    r = h.norm(dim=1).clamp_min(1e-6).contiguous()
    rel = (torch.randn(2 * R, d, device=dev) * 0.1).contiguous()
    ch, fx = wk["chunks"], wk["fixups"]
    stride = d + 4
    part = torch.empty(max(g.n_slots, 1), stride, device=dev, dtype=torch.float32)
    out = torch.empty(V, d, device=dev, dtype=torch.float32)
    f, i = _lib.fptr, _lib.iptr
    lor = LorentzRGCNLayer(d, d, 2 * R, 100, c=C, activation=F.rrelu, self_loop=True).to(dev).eval()
    uni = HyperbolicUnionRGCNLayer(d, d, 2 * R, c=C, activation=F.rrelu, self_loop=True,
                                   radius_msg_gamma=0.15).to(dev).eval()
    w_rel = lor.weight.detach().contiguous()

    t0 = time.time()
    cs, ct = g.row_type_cols()  # the product order of the chunked edge lists (same-type runs)
    torch.cuda.synchronize()
    log("row/type edge order built in %.1f ms" % ((time.time() - t0) * 1e3))

    def union_agg(src=cs, typ=ct):
        _lib.call("regcn_union_aggregate_f32", f(x), f(r), f(rel), i(src), i(typ),
                  f(wk["norm"]), i(ch), ch.shape[0], i(fx), fx.shape[0], 0.15, d, f(part), stride, f(out),
                  _lib.stream())

    ss = g.row_src_cols()  # the source half's order (duplicate sources adjacent)

    def union_agg_src_runs():
        _lib.call("regcn_union_aggregate_src_runs_f32", f(x), f(r), f(rel), i(cs), i(ct), i(ss),
                  f(wk["norm"]), i(ch), ch.shape[0], i(fx), fx.shape[0], 0.15, 0, d, f(part), stride, f(out),
                  _lib.stream())

    def lorentz_agg(src=cs, typ=ct):
        _lib.call("regcn_lorentz_aggregate_f32", f(x), f(rel), f(w_rel), i(src), i(typ),
                  i(ch), ch.shape[0], i(fx), fx.shape[0], 100, float(C), d, f(part), stride, f(out), _lib.stream())

    fns = {"union_aggregate": union_agg, "union_layer": lambda: uni(g, h, rel),
           "lorentz_aggregate": lorentz_agg, "lorentz_layer": lambda: lor(g, h, rel),
           "lorentz_aggregate_csr": lambda: lorentz_agg(wk["col_src"], wk["col_type"]),  # edge-id order, for comparison
           "union_aggregate_csr": lambda: union_agg(wk["col_src"], wk["col_type"]),
           "union_aggregate_src_runs": union_agg_src_runs}
    st = torch.cuda.Stream(dev)
    b_agg = E * (4 * d + 12) + V * (4 * d + 12)
    # distinct (row, source) pairs: the source half's gathered rows with source runs
    s_np = ss.cpu().numpy()
    rp = wk["rowptr"].cpu().numpy()
    head = np.ones(len(s_np), bool)
    head[1:] = s_np[1:] != s_np[:-1]
    head[rp[:-1][rp[:-1] < len(s_np)]] = True
    n_distinct = int(head.sum())
    res = {"V": V, "E": E, "R2": 2 * R, "d": d, "b_agg_bytes": b_agg, "hbm_peak_gbs": HBM_PEAK_GBS,
           "distinct_row_sources": n_distinct,
           "b_agg_src_runs_bytes": n_distinct * 4 * d + E * 24 + V * (4 * d + 12),
           "sources": "uniform subjects, Zipf objects" if uniform_s else "Zipf subjects and objects"}
    log("distinct (row, source) pairs: %d of %d edges" % (n_distinct, E))
    with torch.no_grad():
        for name in which:
            ms = event_time(fns[name], reps, st, replays=3)
            gbs = b_agg / (ms * 1e-3) / 1e9
            res[name] = {"ms": round(ms, 4), "edges_per_s_G": round(E / (ms * 1e-3) / 1e9, 3),
                         "algorithmic_GBps": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
            log("%-18s %8.3f ms  %6.3f G edges/s  %7.1f GB/s  %.1f%% of HBM peak"
                % (name, ms, E / (ms * 1e-3) / 1e9, gbs, 100 * gbs / HBM_PEAK_GBS))
    return res


def cpu_layers(V=1_000_000, R=256, triples=2_500_000, d=200, log=print):
    """The CPU baseline of config 5 (full size is infeasible on CPU, so
    |V| = 1M with |E| = 5M): the oracle's Union and Lorentz layers (oracle/layers.py, test
    infrastructure) timed on the host cores.  Returns {layer: M edges/s}."""
    from oracle import graph as og
    from oracle import layers as ol
    threads = int(os.environ.get("OMP_NUM_THREADS", "8"))
    torch.set_num_threads(threads)
    snap = snapshot_series(0, V, R, 1, triples)[0]
    g = og.build_sub_graph(V, R, snap)
    E = 2 * triples
    gen = torch.Generator().manual_seed(0)
    h = torch.randn(V, d, generator=gen)
    h = h / h.norm(dim=1, keepdim=True) * (torch.rand(V, 1, generator=gen) * 2.5 + 0.5) * 0.1
    rel = torch.randn(2 * R, d, generator=gen) * 0.1
    w = lambda *s: torch.randn(*s, generator=gen) * 0.05  # noqa: E731
    out = {"V": V, "E": E, "d": d, "threads": threads}
    with torch.no_grad():
        for name, fn in (("union_layer", lambda: ol.union_layer(g, h, rel, w(d, d), w(d, d), w(d, d), C, 0.15)),
                         ("lorentz_layer", lambda: ol.lorentz_layer(g, h, rel, w(2 * R, 100 * 4), w(d, d), w(d, d),
                                                                    C, 100))):
            t0 = time.perf_counter()
            fn()
            dt = time.perf_counter() - t0
            out[name] = {"s": round(dt, 2), "M_edges_per_s": round(E / dt / 1e6, 3)}
            log("cpu %-14s %7.2f s  %.3f M edges/s (%d threads)" % (name, dt, E / dt / 1e6, threads))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--V", type=int, default=1_000_000)
    ap.add_argument("--R", type=int, default=256)
    ap.add_argument("--triples", type=int, default=25_000_000)
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--json", default=None, help="write the results here as well")
    ap.add_argument("--which", default="union_aggregate,union_layer,lorentz_aggregate,lorentz_layer")
    ap.add_argument("--cpu", action="store_true", help="also time the oracle layers at |V|=1M, |E|=5M on the host")
    ap.add_argument("--uniform-src", action="store_true", help="uniform subjects (objects stay Zipf)")
    a = ap.parse_args()
    res = measure(a.V, a.R, a.triples, a.d, a.reps, which=a.which.split(","), log=lambda m: print(m, flush=True),
                  uniform_s=a.uniform_src)
    if a.cpu:
        res["cpu_oracle_E5M"] = cpu_layers(a.V, a.R, 2_500_000, a.d, log=lambda m: print(m, flush=True))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
