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

Every step computes everything from the parameters and its snapshots: no state is kept
across steps except the weights' MFMA fragment packing (a layout of each weight, redone
when the weight changes).  `--serving-cache` keeps the parameter-only states (initial
entity state, the pristine-row memo) across steps instead; it is reported separately.
Predicts of different test snapshots are independent (hyperbolic_main.py:100-149 without
--multi-step), so `--concurrent` (default 4) of the pool's samples run together, one
stream each, inside one captured HIP graph of the whole pool (inputs resident in HBM);
`latency_ms_per_predict` is one sample's predict alone.  `roofline` reports the dominant kernel, timed live with HIP events on its own
stream; `cpu_baseline` times the CPU oracle (oracle/, a restatement of the reference
op sequence) on the same workload on rank 0.  `aggregation_roofline` (N=1) is the
north-star HBM check: the d=200 aggregation kernels on a config-5 snapshot
(|V|=1M, |E|=50M), algorithmic bytes over the HIP-event launch time.
"""
import argparse
import contextlib
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
    ap.add_argument("--pool", type=int, default=16,
                    help="distinct samples cycled through the timed steps; one pool pass is one batch of "
                         "independent predicts (ICEWS14s has 31 test snapshots)")
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of HIP graph replay")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="steps captured per HIP graph (default: the whole pool, replayed as one launch; "
                         "1 = one graph per step)")
    ap.add_argument("--concurrent", type=int, default=4,
                    help="independent samples in flight together (one stream each inside the pool's HIP "
                         "graph): predicts of different test snapshots are independent (hyperbolic_main.py "
                         ":100-149 without --multi-step), so a server may overlap them")
    ap.add_argument("--per-layer", action="store_true",
                    help="run the encoder as per-layer launches instead of the timestep phase launches")
    ap.add_argument("--serving-cache", action="store_true",
                    help="keep parameter-only states across steps (initial entity state, timestep 0's GRU "
                         "pre-half, and the memoised state of rows without an in-edge so far in the window, "
                         "copied instead of recomputed); default: every step computes everything from the "
                         "parameters and its snapshots")
    ap.add_argument("--no-memo", action="store_true", help=argparse.SUPPRESS)  # the default now
    ap.add_argument("--no-batch-share", action="store_true",
                    help="each predict computes its own parameter-only states (default: a pool pass = one "
                         "batch of independent predicts computes them once, inside the timed region, and its "
                         "predicts copy the pristine rows' states, HyperbolicRecurrentRGCN.shared_parameter_states)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU-oracle work")
    ap.add_argument("--no-scale", action="store_true",
                    help="skip the config-5 aggregation roofline (|V|=1M, |E|=50M; ~20 s, N=1 only)")
    ap.add_argument("--shard", default="replica", choices=["replica", "edge", "owner"],
                    help="multi-GPU: independent samples per rank (weak scaling), or every snapshot "
                         "partitioned across the ranks by edges (all-reduce) / destination owner "
                         "(all-gather) (strong scaling, SURVEY.md §8(e))")
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


def make_samples(cfg, pool, device, seed, shard="replica"):
    from regcn_amd import graph as G
    from regcn_amd.parallel import ShardedGraph
    from regcn_amd.synthetic import snapshot_series
    V, R, T = cfg["V"], cfg["R"], cfg["T"]
    snaps = snapshot_series(seed, V, R, T + pool, cfg["per_snap"])
    out = []
    for i in range(pool):
        hist = snaps[i:i + T]
        glist = [G.build_sub_graph(V, R, s, True, device) for s in hist]
        if shard != "replica":
            glist = [ShardedGraph(g, shard) for g in glist]
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


def sequence_times(fns, reps, stream, replays=3):
    """Average device time of each launch in ms when the launches run in their pipeline order
    (each one after its real predecessor, so caches hold what the pipeline leaves them): the
    prefix fns[0..i] captured `reps` times into a HIP graph on `stream`, replayed between HIP
    events on that stream, and launch i timed as the prefix-to-prefix difference.  (Events
    recorded inside a captured graph cannot be timed on this runtime.)"""
    totals = [0.0]
    with torch.cuda.stream(stream):
        for fn in fns:
            fn()
        torch.cuda.synchronize()
        for i in range(1, len(fns) + 1):
            gph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gph, stream=stream):
                for _ in range(reps):
                    for fn in fns[:i]:
                        fn()
            gph.replay()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            for _ in range(replays):
                gph.replay()
            e.record(stream)
            e.synchronize()
            totals.append(s.elapsed_time(e) / (reps * replays))
            del gph
    torch.cuda.synchronize()
    return [max(totals[i + 1] - totals[i], 1e-6) for i in range(len(fns))]


def pmc_traffic(kernel, config, d):
    """HBM bytes per launch of `kernel` from the committed PMC summary of this same bench
    command (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes).  (None, reason) if absent."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, "no profiles/pmc_traffic.json"
    with open(path) as f:
        pm = json.load(f)
    if pm.get("config") != config or int(pm.get("d", -1)) != d:
        return None, "pmc_traffic.json is for another workload"
    k = pm["kernels"].get(kernel.split(" ")[0] if kernel.startswith("k_query<1>") else kernel)
    if k is None:
        return None, "kernel not in pmc_traffic.json"
    return k["hbm_bytes"], "profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, %d launches)" % \
        k["launches"]


def _work(flops, nbytes, ms):
    """Roofline bound of a launch: whichever of its MFMA flops / HBM bytes takes longer at
    peak.  Returns dict(bound, unit, work, achieved, frac)."""
    t_mfma = flops / (FP32_MFMA_PEAK_TFLOPS * 1e12)
    t_hbm = nbytes / (HBM_PEAK_GBS * 1e9)
    if t_mfma >= t_hbm:
        ach = flops / (ms * 1e-3) / 1e12
        return dict(bound="mfma", unit="TFLOP/s", work=flops, achieved=ach, peak=FP32_MFMA_PEAK_TFLOPS,
                    frac=ach / FP32_MFMA_PEAK_TFLOPS)
    ach = nbytes / (ms * 1e-3) / 1e9
    return dict(bound="hbm", unit="GB/s", work=nbytes, achieved=ach, peak=HBM_PEAK_GBS, frac=ach / HBM_PEAK_GBS)


def kernel_profile(model, sample, d, device, share=False, pool=1):
    """Live HIP-event timing of each launch of the hot path on the bench workload: the batch's
    cold chain, the timestep phase launches (csrc/timestep.hip) of the sample's last history
    snapshot and the two decoders on its queries, in pipeline order (sequence_times: one
    HIP graph on a stream of its own, a HIP event between consecutive launches).  Returns
    {kernel: dict(ms, per_step, flops, bytes, ...)}."""
    from regcn_amd import hyperbolic_model as HM
    from regcn_amd.hyperbolic_decoder import (_chunked_hyperbolic_dist_score, roth_pair_fusable, roth_pair_queries,
                                              roth_pair_scores)
    hist, glist, test, _ = sample
    glist = [getattr(g, "g", g) for g in glist]  # rank 0 alone: unpartitioned (no collectives)
    g = glist[-1]
    V = g.number_of_nodes()
    E = g.number_of_edges()
    T = len(glist)
    n_pos = g.n_pos
    # rows without in-edges that the captured launches (the window's last timestep) run: all
    # of them, or with the pristine memo only the earlier snapshots' in-edge rows (the
    # kernel's grid bound; an upper bound of the rows it runs)
    memo = share or (model.memo_pristine and model.param_caches)
    split = not memo and model.split_zero_rows  # the rows without in-edges in k_zero_step
    n_zero = sum(x.n_pos for x in glist[:-1]) if memo else 0 if split else V - n_pos
    n_zs = V - n_pos if split else 0
    st = torch.cuda.Stream(device)
    res = {}
    c = model._c_float()
    R2 = model.emb_rel.shape[0]
    lorentz = model.encoder_name == "lgcn"
    lay0, lay1 = model.rgcn.layers[0], model.rgcn.layers[1]
    tag = "3, %d" % (d // lay0.num_bases if d // lay0.num_bases in (1, 2, 4) else 0) if lorentz else "0, 1"
    gemm = 2.0 * d * d  # flops per row of one d x d product
    wn = 0 if lorentz else gemm * n_pos  # union: agg @ W_n
    skip = 2 if getattr(lay1, "skip_connect", False) else 1
    gather_b = E * (4 * d + 8 + (0 if lorentz else 4)) + V * 4 * 2
    row_b = 4.0 * d  # bytes of one fp32 row
    gru_w = 4.0 * 3 * d * d  # one 3d x d GRU weight half
    with torch.no_grad(), torch.cuda.stream(st):
        HM.PHASE_CAPTURE = {}
        try:
            with model.shared_parameter_states(T) if share else contextlib.nullcontext():
                embs, _, h0, _, _ = model.forward(glist, None, True)
            cap = HM.PHASE_CAPTURE
        finally:
            HM.PHASE_CAPTURE = None
        stages = []
        if cap:
            # per launch: A = in-edge rows' self-loop + time-gate GEMMs, layer 0 of the other
            # rows, the GRU x-half (R2 x 3d x d); B = layer-0 gathers (+ W_n), layer 1's
            # self-loop GEMM of the in-edge rows, layer 1 of the other rows (the last
            # timestep's B has no next GRU pre-half); C = layer-1 gathers (+ W_n), the time
            # gate of the other rows (the in-edge rows' ran in A)
            stages += [
                ("k_phase_a", cap["A"][0],
                 2 * gemm * n_pos + gemm * n_zero + 2.0 * R2 * 3 * d * d,
                 row_b * (4 * n_pos + 2 * n_zero) + 4.0 * R2 * d * 3 + gru_w),
                ("k_phase_b<%s>" % tag, cap["B"][0],
                 wn + gemm * n_pos + skip * gemm * n_zero,
                 gather_b + row_b * (3 * n_pos + (1 + skip) * n_zero)),
                ("k_phase_c<%s>" % tag, cap["C"][0],
                 wn + gemm * n_zero,
                 gather_b + row_b * ((4 + skip) * n_pos + 4 * n_zero)),
            ]
            if "chain" in cap:  # the batch's pristine states: all rows x T timesteps, once per pool pass
                stages.insert(0, ("k_cold_chain", cap["chain"][0], (2 + skip) * gemm * V * T,
                                  row_b * V * (1 + 2 * T)))
            if "Z" in cap:  # rows without in-edges: W_evolve[0], W_evolve[1] (+ skip), W_g; x0 in, h, x out
                stages.append(("k_zero_step", cap["Z"][0], (2 + skip) * gemm * n_zs, row_b * 3 * n_zs))
        at = torch.cat([test, torch.stack([test[:, 2], test[:, 1] + model.num_rels, test[:, 0]], 1)])
        B = at.shape[0]
        emb = model._final_embedding(embs[-1], c).contiguous()
        dec, rdec = model.decoder_ob, model.rdecoder
        fdec = dec
        if model.fused_decoders and roth_pair_fusable(dec, rdec, emb):
            # the predict's two decoder launches (csrc/queries.hip, score.hip jobs)
            rel = h0.detach().contiguous()
            _, qe, qr, cand = roth_pair_queries(fdec, rdec, emb, rel, test, model.num_rels)
            stages.append(("k_queries4", lambda: roth_pair_queries(fdec, rdec, emb, rel, test, model.num_rels),
                           2.0 * B * 5.5 * d * d, 4.0 * (B * d * 5 + R2 * d * 2)))
            stages.append(("k_score_f32_jobs", lambda: roth_pair_scores(fdec, rdec, emb, qe, qr, cand),
                           2.0 * B * (V + R2) * d, 4.0 * (B * d * 2 + (V + R2) * d + B * (V + R2))))
            dec = None
        q = dec._query(emb, h0, at) if dec is not None else None
        if dec is not None and type(dec).__name__ == "HyperbolicRotH":
            stages.append(("k_query<0>", lambda: dec._query(emb, h0, at), 2.0 * B * 3.5 * d * d,
                           4.0 * B * d * 3))
        if dec is not None:
            stages.append(("k_score_f32<0>", lambda: _chunked_hyperbolic_dist_score(
                q, emb, dec.entity_bias, dec.c, 128, 256, score_scale=dec.score_scale_raw,
                score_margin=dec.score_margin, _raw_scale=True), 2.0 * B * V * d, 4.0 * (B * d + V * d + B * V)))
        if dec is not None and type(rdec).__name__ == "HyperbolicRotHRel":
            stages.append(("k_query<1> + k_score (relations)", lambda: rdec.forward(emb, h0, at),
                           2.0 * B * 2 * d * d + 2.0 * B * R2 * d, 4.0 * (B * d * 3 + B * R2)))
        seq = sequence_times([fn for _, fn, _, _ in stages], 30, st)
        for (name, fn, flops, nbytes), ms in zip(stages, seq):
            per_step = T if name.startswith(("k_phase", "k_zero")) else 1.0 / pool if name == "k_cold_chain" else 1
            res[name] = dict(ms=ms, per_step=per_step, flops=flops, bytes=nbytes, **_work(flops, nbytes, ms))
    torch.cuda.synchronize()
    return res


def decoder_at_scale():
    """Config-5 decoder: all-entity scoring of B = 1024 queries against
    N = 1M candidates at d = 200, MFMA-bound; flops 2 B N d per launch over the HIP-event
    launch time against the dense fp32 MFMA peak (tools/scorebench.py)."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from scorebench import measure
    r = measure(1024, 1_000_000, 200, reps=3, modes="score,ce", verbose=False)
    torch.cuda.empty_cache()
    return {"bound": "mfma", "unit": "TFLOP/s", "peak": FP32_MFMA_PEAK_TFLOPS,
            "config": "B=1024 queries x N=1000000 candidates, d=200", "flops_per_launch": r["flops_per_launch"],
            "score": {"achieved": r["score"]["tflops"], "frac": r["score"]["frac"], "avg_launch_us":
                      round(r["score"]["ms"] * 1e3, 1), "kernel": "k_score_f32<0>"},
            "cross_entropy": {"achieved": r["ce"]["tflops"], "frac": r["ce"]["frac"], "avg_launch_us":
                              round(r["ce"]["ms"] * 1e3, 1), "kernel": "k_score_f32<1>"}}


def aggregation_at_scale(device):
    """North-star roofline check: the d=200 union and Lorentz
    aggregations over one |V|=1M, |E|=50M synthetic snapshot (Zipf destinations), timed
    live with HIP events; algorithmic bytes E (4d + 12) + V (4d + 12) per launch."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from aggbench import measure
    res = measure(dev=device, which=("union_aggregate", "lorentz_aggregate"), log=lambda m: None)
    out = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS, "config": "synthetic |V|=%d |E|=%d R2=%d d=%d"
           % (res["V"], res["E"], res["R2"], res["d"]), "bytes_per_launch": res["b_agg_bytes"]}
    try:  # HBM bytes per launch from the committed PMC passes of tools/aggbench.py
        with open(os.path.join(REPO, "profiles", "pmc_traffic_agg.json")) as fh:
            pmc = json.load(fh)["kernels"]
    except (OSError, ValueError, KeyError):
        pmc = {}
    for k, kern in (("union_aggregate", "k_gather_sum<0>"), ("lorentz_aggregate", "k_lorentz_sum<2>")):
        tr = pmc.get(kern, {}).get("hbm_bytes")
        out[k] = {"achieved": res[k]["algorithmic_GBps"], "frac": res[k]["hbm_frac"], "avg_launch_us":
                  round(res[k]["ms"] * 1e3, 1), "G_edges_per_s": res[k]["edges_per_s_G"], "kernel": kern,
                  "traffic": tr, "traffic_source": "profiles/pmc_traffic_agg.json (rocprofv3 FETCH_SIZE x2 + "
                  "WRITE_SIZE of tools/aggbench.py)" if tr else None}
    torch.cuda.empty_cache()
    return out


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
            o_tr, o_score, o_score_rel = OM.hyperbolic_predict(sd, ocfg, og, test)[:3]
            times.append(time.time() - t0)
            if time.time() > t_end or len(times) >= 5:
                break
        # MRR parity (the metric's second half): the HIP predict and the oracle on the same
        # sample and weights, raw and time-filtered (rgcn/utils.py:136-166), entity and relation
        dev = next(model.parameters()).device
        all_tr, score, score_rel = model.predict(glist, R, None, test.to(dev), True)
        ans_e = OM.answers_for_filter(test_np, R)
        ans_r = OM.answers_for_filter(test_np, R, rel_p=True)
        mrr = {}
        for name, got, ref, rel in (("entity", score, o_score, False), ("relation", score_rel, o_score_rel, True)):
            f_g, r_g = OM.total_rank(o_tr, got.float().cpu(), ans_r if rel else ans_e, rel)[:2]
            f_o, r_o = OM.total_rank(o_tr, ref.float(), ans_r if rel else ans_e, rel)[:2]
            mrr[name] = {"raw_hip": round(r_g, 6), "raw_oracle": round(r_o, 6), "filtered_hip": round(f_g, 6),
                         "filtered_oracle": round(f_o, 6), "max_abs_delta": round(max(abs(r_g - r_o), abs(f_g - f_o)), 6)}
        mrr["tolerance"] = 0.002
        mrr["note"] = "random-init weights on synthetic snapshots: absolute MRR is near chance; the delta is the check"
    per = float(np.mean(times))
    return dict(value=edges_per_step(glist) / per / 1e6, unit="M edges/s", cores=torch.get_num_threads(),
                kind="port",
                sample="%d x oracle predict (%s, history %d, %d queries) on host CPU; %.2f s each"
                       % (len(times), cfg["label"], cfg["T"], 2 * len(test_np), per)), mrr


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; BENCH_DIST_BACKEND=gloo rehearses several ranks on one card
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    from regcn_amd.synthetic import CONFIGS
    cfg = CONFIGS[args.config]
    d = args.d
    model = build_model(cfg, d, device, seed=1234)          # same weights on every rank
    model.use_phases = not args.per_layer
    model.memo_pristine = model.param_caches = args.serving_cache
    sharded = args.shard != "replica" and world > 1
    # replicas: independent data per rank; sharded: every rank holds the same snapshots
    samples = make_samples(cfg, args.pool, device, seed=100 if sharded else 100 + 7919 * rank,
                           shard=args.shard if sharded else "replica")
    if sharded:
        args.no_graph = True  # collectives between the launches: eager
    R = cfg["R"]

    def eager(i):
        _, glist, test, _ = samples[i]
        return model.predict(glist, R, None, test, True)

    conc = max(1, min(args.concurrent, len(samples)))
    lanes = [torch.cuda.Stream(device) for _ in range(conc)] if conc > 1 else []

    share = not args.no_batch_share and not args.serving_cache

    def pool_pass(origin):
        """Every pool sample once, as one batch: the batch's parameter-only states computed
        once on `origin` (share), then with lanes sample i on lane i % conc, forked from and
        joined back into `origin` (a fork/join in the captured graph)."""
        with model.shared_parameter_states(cfg["T"]) if share else contextlib.nullcontext():
            if not lanes:
                for i in range(len(samples)):
                    eager(i)
                return
            for ln in lanes:
                ln.wait_stream(origin)
            for i in range(len(samples)):
                with torch.cuda.stream(lanes[i % conc]):
                    eager(i)
            for ln in lanes:
                origin.wait_stream(ln)

    with torch.no_grad():
        for w in range(max(args.warmup, 1)):
            eager(w % len(samples))
        if lanes:
            pool_pass(torch.cuda.current_stream(device))
    torch.cuda.synchronize()
    # HIP graphs: one per step (graph_steps = 1), and one holding the whole pool's steps in
    # sequence, so consecutive steps do not pay a graph launch each (~20 us on this runtime)
    graphs, pool_graph = [], None
    gs = args.graph_steps or len(samples)
    if lanes and (args.no_graph or gs != len(samples)):
        raise SystemExit("--concurrent needs the whole-pool HIP graph (no --no-graph / --graph-steps)")
    if not args.no_graph:
        cap = torch.cuda.Stream(device)
        # one predict alone (the per-sample graphs: latency, --graph-steps 1) keeps its rows
        # without in-edges inside the phase launches, beside the in-edge tiles' latency
        # chains; with several predicts in flight they run as their own launch
        # (regcn_zero_step_f32), whose workgroups the other predicts' chains overlap.  Both
        # are bit for bit the same values (tests/test_gpu_parity.py).
        split_many = model.split_zero_rows
        model.split_zero_rows = False
        with torch.no_grad():
            for i in range(len(samples)):
                gph = torch.cuda.CUDAGraph()
                with torch.cuda.stream(cap):
                    eager(i)  # warm the capture stream's allocator pool
                    torch.cuda.synchronize()
                    with torch.cuda.graph(gph, stream=cap):
                        eager(i)
                graphs.append(gph)
            model.split_zero_rows = split_many and bool(lanes)
            if gs > 1 and gs == len(samples):
                pool_graph = torch.cuda.CUDAGraph()
                with torch.cuda.stream(cap):
                    with torch.cuda.graph(pool_graph, stream=cap):
                        pool_pass(cap)
        for gph in graphs:
            gph.replay()
        if pool_graph is not None:
            pool_graph.replay()
        torch.cuda.synchronize()

    def run_steps(k0, n):
        """Steps k0 .. k0 + n - 1 (sample k % pool): whole-pool graph launches where aligned."""
        k = k0
        while k < k0 + n:
            if pool_graph is not None and k % len(samples) == 0 and k + len(samples) <= k0 + n:
                pool_graph.replay()
                k += len(samples)
            elif graphs:
                graphs[k % len(samples)].replay()
                k += 1
            else:
                with torch.no_grad():
                    eager(k % len(samples))
                k += 1

    epw = [edges_per_step(s[1]) for s in samples]
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(0, args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    edges_local = sum(epw[k % len(samples)] for k in range(args.steps))
    if world > 1:
        t = torch.tensor([elapsed, float(edges_local)], dtype=torch.float64,
                         device=device if backend == "nccl" else "cpu")
        tm = t.clone()
        dist.all_reduce(tm[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, edges_total = float(tm[0]), float(t[1])
        if sharded:  # every rank processed the same edges: count them once
            edges_total = float(edges_local)
    else:
        edges_total = float(edges_local)
    value = edges_total / elapsed / 1e6

    # latency of one predict alone (concurrency 1): its HIP graph replayed and waited for
    lat_ms = None
    if graphs and rank == 0:
        lat = []
        for k in range(40):
            t1 = time.perf_counter()
            graphs[k % len(graphs)].replay()
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t1)
        lat_ms = float(np.median(lat)) * 1e3

    kern = kernel_profile(model, samples[0], d, device, share=share, pool=len(samples)) if rank == 0 else {}
    out = None
    if rank == 0:
        shares = {k: v["ms"] * v["per_step"] for k, v in kern.items()}
        dom = max(shares, key=shares.get)
        kd = kern[dom]
        traffic, tsrc = pmc_traffic(dom, args.config, d)
        roof = dict(bound=kd["bound"], kernel=dom, achieved=round(kd["achieved"], 3), peak=kd["peak"],
                    unit=kd["unit"], frac=round(kd["frac"], 4), traffic=traffic, traffic_source=tsrc,
                    flops_per_launch=kd["flops"], algorithmic_bytes_per_launch=kd["bytes"],
                    avg_launch_us=round(kd["ms"] * 1e3, 3))
        if kd["frac"] < 0.1:  # the ICEWS-size launches move <= a few MB each
            roof["note"] = ("latency-bound at this size (a few MB and ~20 in-edge tiles per launch, one "
                            "gather -> GEMM -> epilogue chain per tile); the HBM and MFMA rooflines of the "
                            "same kernels are aggregation_roofline (config 5) and decoder_roofline")
        kernels = {k: dict(avg_us=round(v["ms"] * 1e3, 3), per_step=v["per_step"], bound=v["bound"],
                           achieved=round(v["achieved"], 3), unit=v["unit"], frac=round(v["frac"], 4))
                   for k, v in kern.items()}
        # SURVEY.md §8(d) asks for edges/s per layer and per encoder forward besides the
        # end-to-end step: from the live kernel times (sum of per-step kernel time, no gaps)
        enc_us = sum(v["ms"] * 1e3 * v["per_step"] for k, v in kern.items() if k.startswith(("k_phase", "k_zero", "k_cold")))
        e_step = float(np.mean(epw))
        breakdown = {"encoder_kernels_us_per_step": round(enc_us, 2),
                     "encoder_M_edges_per_s": round(e_step / enc_us, 3) if enc_us else None,
                     "note": "kernel time only (sum of the stage launches' HIP-event averages, the phase "
                             "launches of one timestep x history_len); value is end to end"}
        scale = dec = None
        if not args.no_scale and world == 1:
            scale = aggregation_at_scale(device)
            dec = decoder_at_scale()
        cpu = mrr = None
        if not args.no_cpu_baseline and world == 1:
            cpu, mrr = cpu_baseline(cfg, d, model, samples[0], args.cpu_budget)
        ms = elapsed / args.steps * 1e3
        out = {"metric": METRIC, "value": round(value, 3), "unit": "M edges/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
               "scaling": "strong" if sharded else "weak", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic (%s-shaped snapshots, random-init weights)" % args.config.split("_")[0],
               "config": {"workload": cfg["label"], "V": cfg["V"], "R": cfg["R"], "triples_per_snapshot":
                          cfg["per_snap"], "history_len": cfg["T"], "n_layers": 2, "d": d,
                          "edges_per_step": int(np.mean(epw)), "queries_per_step": 2 * cfg["per_snap"],
                          "hip_graph": bool(graphs), "steps_per_graph_launch": len(samples) if pool_graph else 1,
                          "concurrent_samples": conc, "encoder_launches": "per-layer" if args.per_layer
                          else "timestep phases", "serving_cache": bool(args.serving_cache),
                          "batch_shared_states": share,
                          "parallelism": ("%s-partitioned snapshots x%d" % (args.shard, world)) if sharded
                          else "replicas x%d" % world},
               "latency_ms_per_predict": round(lat_ms, 4) if lat_ms else None,
               "roofline": roof, "kernels": kernels, "breakdown": breakdown, "aggregation_roofline": scale,
               "decoder_roofline": dec, "cpu_baseline": cpu, "mrr_parity": mrr}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
