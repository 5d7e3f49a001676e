#!/usr/bin/env python
"""Benchmark of the RE-GCN hot path on MI355X (contract: one JSON line on rank 0).

A step is one pass of the hot path over one batch of synthetic input: the
`HyperbolicRecurrentRGCN.predict` of one sample = the recurrent encoder over a
history_len=3 window of snapshots (relation context, relation GRU, 2 message-passing
layers, time gate + radius evolution per snapshot) followed by all-entity RotH scoring
of the target snapshot's queries (entity and relation decoders).  The default workload
is BASELINE.json configs[1] (ICEWS14s-shaped, encoder=lgcn, decoder=roth, c=0.01,
d=200) on synthetic snapshots (the datasets are absent).

metric = million directed message edges aggregated per second (edges after inverse
doubling x GCN layers x history snapshots), whole job.
Multi-GPU: one process per GPU, each rank runs its own independent samples (replicas:
the path has no exchange step at this size); scaling = weak.

The timed region replays one captured HIP graph per pool sample (inputs resident in
HBM).  `roofline` reports the dominant kernel, timed live with HIP events on its own
stream; `cpu_baseline` times the CPU oracle (oracle/, a restatement of the reference
op sequence) on the same workload on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))

METRIC = "million edges aggregated/sec at d=200 history_len=3; MRR parity vs ref"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFLOPS = 157.3  # dense fp32 matrix peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="icews14s_lgcn_roth")
    ap.add_argument("--pool", type=int, default=4, help="distinct samples cycled through the timed steps")
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of HIP graph replay")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU-oracle work")
    return ap.parse_args()


def build_model(cfg, d, device, seed):
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    torch.manual_seed(seed)
    V, R = cfg["V"], cfg["R"]
    rng = np.random.default_rng(seed)
    m = HyperbolicRecurrentRGCN(cfg["decoder"], cfg["encoder"], V, R, 0, 0, d, "sub", cfg["T"],
                                num_bases=cfg["n_bases"], num_hidden_layers=2, dropout=0.2, c=0.01, self_loop=True,
                                layer_norm=False, input_dropout=0.2, hidden_dropout=0.2, feat_dropout=0.2,
                                entity_prediction=True, relation_prediction=True, use_cuda=True, gpu=0,
                                radius_target=rng.uniform(0.5, 3.0, V).astype(np.float32), radius_msg_gamma=0.15)
    return m.to(device).eval()


def make_samples(cfg, pool, device, seed):
    from regcn_amd import graph as G
    from regcn_amd.synthetic import snapshot_series
    V, R, T = cfg["V"], cfg["R"], cfg["T"]
    snaps = snapshot_series(seed, V, R, T + pool, cfg["per_snap"])
    out = []
    for i in range(pool):
        hist = snaps[i:i + T]
        glist = [G.build_sub_graph(V, R, s, True, device) for s in hist]
        test = torch.from_numpy(snaps[i + T]).to(device)
        out.append((hist, glist, test, snaps[i + T]))
    return out


def edges_per_step(glist, n_layers=2):
    return n_layers * sum(g.number_of_edges() for g in glist)


def event_time(fn, reps, stream, replays=5):
    """Average device time of one fn() launch in ms: `reps` launches captured into a HIP
    graph on `stream`, replayed `replays` times between HIP events recorded on `stream`
    (graph replay removes the per-call host launch cost, which would otherwise dominate
    these 5-50 us kernels)."""
    with torch.cuda.stream(stream):
        fn()
        torch.cuda.synchronize()
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph, stream=stream):
            for _ in range(reps):
                fn()
        gph.replay()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(replays):
            gph.replay()
        e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) / (reps * replays)


def kernel_profile(model, sample, d, device):
    """Live HIP-event timing of each hot-path kernel on the bench workload (first history
    snapshot of sample 0 for the per-layer kernels, the sample's queries for the scorer).
    Returns {name: dict(ms, launches_per_step, work, unit, bound)}."""
    from regcn_amd import _lib
    from regcn_amd.hyperbolic_decoder import _chunked_hyperbolic_dist_score
    from regcn_amd.tangent import tangent_of
    hist, glist, test, _ = sample
    g = glist[0]
    wk = g.work()
    V = g.number_of_nodes()
    T = len(glist)
    st = torch.cuda.Stream(device)
    res = {}
    with torch.no_grad(), torch.cuda.stream(st):
        embs, _, h0, _, _ = model.forward(glist, None, True)
        h = embs[-1]
        x, r = tangent_of(h, 0.01)
        rel = h0.contiguous()
        agg = torch.empty_like(x)
        lay = model.rgcn.layers[0]
        ch, fx = wk["chunks"], wk["fixups"]
        E = g.number_of_edges()
        n_rows = int(ch.shape[0])  # single-chunk rows written (no long rows at this size)
        agg_bytes = E * (4 * d + 12) + n_rows * (4 * d + 12)
        if model.encoder_name == "lgcn":
            part = torch.empty(max(g.n_slots, 1), d + 4, device=device)
            W = lay.weight.detach().contiguous()
            name = "k_lorentz_sum"

            def agg_fn():
                _lib.call("regcn_lorentz_aggregate_f32", _lib.fptr(x), _lib.fptr(rel), _lib.fptr(W),
                          _lib.iptr(wk["col_src"]), _lib.iptr(wk["col_type"]), _lib.iptr(ch), ch.shape[0],
                          _lib.iptr(fx), fx.shape[0], lay.num_bases, 0.01, d, _lib.fptr(part), d + 4,
                          _lib.fptr(agg), _lib.stream())
        else:
            part = torch.empty(max(g.n_slots, 1), d, device=device)
            name = "k_gather_sum"

            def agg_fn():
                _lib.call("regcn_union_aggregate_f32", _lib.fptr(x), _lib.fptr(r), _lib.fptr(rel),
                          _lib.iptr(wk["col_src"]), _lib.iptr(wk["col_type"]), _lib.fptr(wk["norm"]),
                          _lib.iptr(ch), ch.shape[0], _lib.iptr(fx), fx.shape[0], 0.15, d, _lib.fptr(part), d,
                          _lib.fptr(agg), _lib.stream())
        res[name] = dict(ms=event_time(agg_fn, 200, st), launches_per_step=2 * T, work=agg_bytes, unit="GB/s",
                         bound="hbm", what="E*(4d+12) + rows*(4d+12) bytes, E=%d, rows=%d" % (E, n_rows))
        from regcn_amd.hyperbolic_layers import layer_tail
        wl, we = lay.loop_weight.detach(), lay.evolve_loop_weight.detach()
        wn = getattr(lay, "weight_neighbor", None)
        wn = wn.detach() if wn is not None else None

        def tail_fn():
            layer_tail(agg, wn, x, wl, we, None, None, None, None, g, 0.01, False)
        tail_flops = 2.0 * d * d * (V + (g.n_pos if wn is not None else 0))
        res["k_layer_tail"] = dict(ms=event_time(tail_fn, 200, st), launches_per_step=2 * T, work=tail_flops,
                                   unit="TFLOP/s", bound="mfma",
                                   what="2*d*d*(V%s) flops" % (" + n_pos" if wn is not None else ""))
        trev = model.temporal_radius_evolution
        from regcn_amd.weights import packed
        wg, bg = packed(model.time_gate_weight), model.time_gate_bias.detach().contiguous()
        w_r = trev.radius_mlp.weight.detach().reshape(-1).contiguous()
        b_r = trev.radius_mlp.bias.detach().reshape(-1).contiguous()
        rs = model._static_radius(0.01).contiguous()
        hn, xn, rn = torch.empty_like(x), torch.empty_like(x), torch.empty_like(r)
        hc = h.contiguous()

        def step_fn():
            _lib.call("regcn_timestep_f32", _lib.fptr(hc), _lib.fptr(x), _lib.fptr(wg), _lib.fptr(bg), _lib.fptr(rs),
                      _lib.fptr(w_r), _lib.fptr(b_r), 0.1, 1.0, 0, 1, V, d, 0.01, 0.01, _lib.fptr(hn), _lib.fptr(xn),
                      _lib.fptr(rn), _lib.stream())
        res["k_timestep"] = dict(ms=event_time(step_fn, 200, st), launches_per_step=T, work=2.0 * d * d * V,
                                 unit="TFLOP/s", bound="mfma", what="2*d*d*V flops")
        B = 2 * test.shape[0]
        q = torch.randn(B, d, device=device) * 0.05
        cand = h.contiguous()
        sc = torch.ones(1, device=device)

        def score_fn():
            _chunked_hyperbolic_dist_score(q, cand, None, 0.01, 128, 256, score_scale=sc, score_margin=sc)
        res["k_score"] = dict(ms=event_time(score_fn, 200, st), launches_per_step=1, work=2.0 * B * V * d,
                              unit="TFLOP/s", bound="mfma", what="2*B*N*d flops, B=%d, N=%d" % (B, V))
    torch.cuda.synchronize()
    return res


def cpu_baseline(cfg, d, model, sample, budget):
    """Time the CPU oracle (restatement of the reference op sequence) on one sample."""
    sys.path.insert(0, REPO)
    from oracle import graph as OG
    from oracle import model as OM
    hist, glist, _, test_np = sample
    V, R = cfg["V"], cfg["R"]
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    ocfg = dict(c=0.01, n_layers=2, n_bases=cfg["n_bases"], radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
                radius_anchor_beta=1.0, radius_msg_gamma=0.15, use_residual_evolution=True, layer_norm=False,
                encoder=cfg["encoder"], decoder=cfg["decoder"])
    og = [OG.build_sub_graph(V, R, s) for s in hist]
    test = torch.from_numpy(test_np)
    times = []
    t_end = time.time() + budget
    with torch.no_grad():
        while True:
            t0 = time.time()
            OM.hyperbolic_predict(sd, ocfg, og, test)
            times.append(time.time() - t0)
            if time.time() > t_end or len(times) >= 5:
                break
    per = float(np.mean(times))
    return dict(value=edges_per_step(glist) / per / 1e6, unit="M edges/s", cores=torch.get_num_threads(),
                kind="port",
                sample="%d x oracle predict (%s, history %d, %d queries) on host CPU; %.2f s each"
                       % (len(times), cfg["label"], cfg["T"], 2 * len(test_np), per))


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)
    from regcn_amd.synthetic import CONFIGS
    cfg = CONFIGS[args.config]
    d = args.d
    model = build_model(cfg, d, device, seed=1234)          # same weights on every rank
    samples = make_samples(cfg, args.pool, device, seed=100 + 7919 * rank)  # independent data per rank
    R = cfg["R"]

    def eager(i):
        _, glist, test, _ = samples[i]
        return model.predict(glist, R, None, test, True)

    with torch.no_grad():
        for w in range(max(args.warmup, 1)):
            eager(w % len(samples))
    torch.cuda.synchronize()
    graphs = []
    if not args.no_graph:
        cap = torch.cuda.Stream(device)
        with torch.no_grad():
            for i in range(len(samples)):
                gph = torch.cuda.CUDAGraph()
                with torch.cuda.stream(cap):
                    eager(i)  # warm the capture stream's allocator pool
                    torch.cuda.synchronize()
                    with torch.cuda.graph(gph, stream=cap):
                        eager(i)
                graphs.append(gph)
        for gph in graphs:
            gph.replay()
        torch.cuda.synchronize()

    def step(k):
        i = k % len(samples)
        if graphs:
            graphs[i].replay()
        else:
            with torch.no_grad():
                eager(i)

    epw = [edges_per_step(s[1]) for s in samples]
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    edges_local = sum(epw[k % len(samples)] for k in range(args.steps))
    if world > 1:
        t = torch.tensor([elapsed, float(edges_local)], device=device, dtype=torch.float64)
        tm = t.clone()
        dist.all_reduce(tm[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, edges_total = float(tm[0]), float(t[1])
    else:
        edges_total = float(edges_local)
    value = edges_total / elapsed / 1e6

    kern = kernel_profile(model, samples[0], d, device) if rank == 0 else {}
    out = None
    if rank == 0:
        shares = {k: v["ms"] * v["launches_per_step"] for k, v in kern.items()}
        dom = max(shares, key=shares.get)
        kd = kern[dom]
        if kd["unit"] == "GB/s":
            ach, peak = kd["work"] / (kd["ms"] * 1e-3) / 1e9, HBM_PEAK_GBS
        else:
            ach, peak = kd["work"] / (kd["ms"] * 1e-3) / 1e12, FP32_MFMA_PEAK_TFLOPS
        roof = dict(bound=kd["bound"], kernel=dom, achieved=round(ach, 3), peak=peak, unit=kd["unit"],
                    frac=round(ach / peak, 4), traffic=None, work_per_launch=kd["what"],
                    avg_launch_us=round(kd["ms"] * 1e3, 3))
        kernels = {k: dict(avg_us=round(v["ms"] * 1e3, 3), per_step=v["launches_per_step"],
                           achieved=round(v["work"] / (v["ms"] * 1e-3) / (1e9 if v["unit"] == "GB/s" else 1e12), 3),
                           unit=v["unit"]) for k, v in kern.items()}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(cfg, d, model, samples[0], args.cpu_budget)
        ms = elapsed / args.steps * 1e3
        out = {"metric": METRIC, "value": round(value, 3), "unit": "M edges/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic (%s-shaped snapshots, random-init weights)" % args.config.split("_")[0],
               "config": {"workload": cfg["label"], "V": cfg["V"], "R": cfg["R"], "triples_per_snapshot":
                          cfg["per_snap"], "history_len": cfg["T"], "n_layers": 2, "d": d,
                          "edges_per_step": int(np.mean(epw)), "queries_per_step": 2 * cfg["per_snap"],
                          "hip_graph": bool(graphs), "parallelism": "replicas x%d" % world},
               "roofline": roof, "kernels": kernels, "cpu_baseline": cpu}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
