#!/usr/bin/env python
"""Benchmark of the RE-GCN hot path on MI355X (contract: one JSON line on rank 0).

Headline workload (default `--config synthetic_1m`): BASELINE.json configs[4], the
north-star stress snapshot shape on ONE GPU -- |V| = 1M entities, |E| = 50M directed
message edges per snapshot (25M triples + inverses), |R| = 256 (R2 = 512), d = 200,
history_len = 3, encoder hyperbolic_uvrgcn (2 layers), decoder RotH.  A step is one
`HyperbolicRecurrentRGCN.predict` (hyperbolic_model.py:892-939): the full recurrent
forward over a 3-snapshot window (hyperbolic_model.py:797-884: relation context, relation
GRU, 2 message-passing layers, time gate + radius evolution per snapshot) followed by the
entity (RotH) and relation (RotHRel) decoders on a 1,024-query chunk (512 test triples
and their inverses) scored against all 1M entities.  Every step computes everything from
the parameters and its snapshots (no state kept across steps except the weights' MFMA
fragment packing); the snapshot graphs are built once, in HBM, before the timed region.

metric = million directed message edges aggregated per second (edges after inverse
doubling x GCN layers x history snapshots = 300M per step), whole job:
K steps timed exactly, between barriers + device synchronisation, max over ranks.
Multi-GPU: one process per GPU.  The default (--gpus > 1) is replicas: independent predicts are
the data-parallel unit (hyperbolic_main.py's test loop predicts every test snapshot from its own
window), so each rank runs its own windows with no data-path collective (weak scaling; value =
all ranks' edges over the max-over-ranks time).  `--shard owner` (or `--owner-leg` beside the
replicas) partitions every snapshot instead (SURVEY.md §8(e) partitioning 2, strong scaling of one
predict): the entity ids are relabelled so each rank's rows carry an equal share of the edges
(parallel.EntityRelabel), every rank runs its rows of every layer and sends the rows the other
ranks read (halo all_to_all, 804 B per row) on a side stream while its next row chunk computes,
the relation means are partitioned (one all_reduce of R x d), and the step ends in the
candidate-sharded decoder (predict_ranks).  At N = 1 the line carries `owner_simulation`: the 8
ranks' launches run one after another on the one GPU, each rank's device time measured, plus the
replicated work and the exchange volume.

Per-call device times come from HIP events recorded on the launching stream after every
library call during the timed steps (`_lib.EVENT_TRACE`); `roofline` reports the call
with the largest time per step against its algorithmic bytes (or flops), with the HBM
traffic of its kernel from the committed rocprofv3 PMC passes (profiles/).
`cpu_baseline` times the CPU oracle's encoder forward on a bounded sample on rank 0.

The dataset-sized configs (ICEWS14s lgcn+roth, ICEWS14s RE-GCN uvrgcn+convtranse, ICEWS18 roth,
GDELT for both encoders) run with `--config` (latency-bound: pools of 48 independent predicts, 24
in flight, in one HIP graph, whole pool passes timed); the headline line carries them as `legs`
(value, roofline fraction, CPU baseline, MRR parity of the HIP predict against the oracle).
The printed line is compact (<= 8 KB, compact_line); the full record goes to BENCH_DETAIL
(default gpurun_out/bench_detail.json).
"""
import argparse
import contextlib
import gc
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
HBM_COPY_GBS = 6300.0          # measured device copy rate (uniform-source aggregation)
LINK_DERATE = 0.8              # owner simulation: the peer links at 80 % of nominal (the derated prediction)
SIM_BLOCKER_CYCLES = int(os.environ.get("BENCH_SIM_BLOCKER_CYCLES", str(1_200_000_000)))  # ~0.5 s device wait
FP32_MFMA_PEAK_TFLOPS = 157.3  # dense fp32 matrix peak (MI355X_MICROARCH.md)


_T0 = time.time()


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print("[bench %6.1f s] %s" % (time.time() - _T0, msg), file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="synthetic_1m")
    ap.add_argument("--pool", type=int, default=0,
                    help="distinct samples cycled through the timed steps (default: 2 windows at config 5; 48 "
                         "for the dataset configs, where one pool pass is one batch of independent predicts)")
    ap.add_argument("--queries", type=int, default=1024,
                    help="config 5: queries per step (half test triples, half their inverses)")
    ap.add_argument("--encoder-launches", default="auto", choices=["auto", "phases", "layers"],
                    help="timestep phase launches or per-layer launches (auto: layers at config 5, phases "
                         "for the dataset configs); both give the same values bit for bit")
    ap.add_argument("--no-extras", action="store_true",
                    help="config 5: skip the ICEWS14s / ICEWS18 sub-benchmarks and the MRR parity leg")
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of HIP graph replay")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="steps captured per HIP graph (default: the whole pool, replayed as one launch; "
                         "1 = one graph per step)")
    ap.add_argument("--concurrent", type=int, default=24,
                    help="independent samples in flight together (one stream each inside the pool's HIP "
                         "graph): predicts of different test snapshots are independent (hyperbolic_main.py "
                         ":100-149 without --multi-step), so a server may overlap them.  Default 16 with "
                         "pools of 48 (profiles/r6_concurrency_sweep.txt: ICEWS14s 27.9 -> 31.7, GDELT "
                         "65.6 -> 69.6, ICEWS18 31.7 -> 34.4 M edges/s against 4 with pools of 16)")
    ap.add_argument("--per-layer", action="store_true", help=argparse.SUPPRESS)  # = --encoder-launches layers
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
                    help="skip the config-5 aggregation and decoder rooflines (N=1 only)")
    ap.add_argument("--shard", default="auto", choices=["auto", "replica", "edge", "owner"],
                    help="multi-GPU: independent samples per rank (weak scaling, no data-path collective), "
                         "or every snapshot partitioned across the ranks by edges (all-reduce) / destination "
                         "owner (halo all_to_all) (strong scaling, SURVEY.md §8(e)); auto: replica")
    ap.add_argument("--owner-leg", action="store_true",
                    help="config 5, N > 1: also run the owner partition (every snapshot split across the "
                         "ranks by destination rows, halo exchange over RCCL) beside the replica headline")
    ap.add_argument("--sim-ranks", type=int, default=8,
                    help="config 5 at N = 1: ranks of the one-GPU owner-partition simulation (0: skip)")
    a = ap.parse_args(argv)
    if a.per_layer:
        a.encoder_launches = "layers"
    return a


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
    w_dd = 4.0 * d * d  # one d x d weight
    # per-launch tables every in-edge tile reads: the relation rows (h_0) and the Lorentz block
    # table (R2 x num_bases s^2) or the union W_n
    tables = 4.0 * R2 * d + (4.0 * lay0.weight.numel() if lorentz else w_dd)
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
            # bytes: the rows each launch moves plus every weight / table it reads once (the
            # GRU halves, W_loop / W_evolve / W_g, the relation and Lorentz block tables)
            stages += [
                ("k_phase_a", cap["A"][0],
                 2 * gemm * n_pos + gemm * n_zero + 2.0 * R2 * 3 * d * d,
                 row_b * (4 * n_pos + 2 * n_zero) + 4.0 * R2 * d * 3 + gru_w + 3 * w_dd),
                ("k_phase_b<%s>" % tag, cap["B"][0],
                 wn + gemm * n_pos + skip * gemm * n_zero,
                 gather_b + row_b * (3 * n_pos + (1 + skip) * n_zero) + tables + 2 * w_dd
                 + 2 * gru_w + 4.0 * 2 * R2 * d),
                ("k_phase_c<%s>" % tag, cap["C"][0],
                 wn + gemm * n_zero,
                 gather_b + row_b * ((4 + skip) * n_pos + 4 * n_zero) + tables + w_dd),
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
    aggregations over one |V|=1M, |E|=50M synthetic snapshot, timed live with HIP events;
    algorithmic bytes E (4d + 12) + V (4d + 12) per launch.  Two source distributions:
    Zipf(1.1) subjects and objects (the headline's snapshots: the hub rows' sources are hot
    rows that L2 / the Infinity Cache serve, so the algorithmic rate can pass the HBM peak),
    and uniform subjects with Zipf objects (the hub rows' sources spread over the whole
    800 MB table: the gathers really stream from HBM).  `traffic` is the rocprofv3
    FETCH_SIZE x2 + WRITE_SIZE bytes per launch of the same command (profiles/), and
    `traffic_frac` those bytes over the launch time against the 8 TB/s peak."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from aggbench import measure
    out = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS}
    for tag, uniform, pmc_file in (("zipf_src", False, "pmc_traffic_agg.json"),
                                   ("uniform_src", True, "pmc_traffic_agg_uniform.json")):
        res = measure(dev=device, which=("union_aggregate", "union_aggregate_src_runs", "lorentz_aggregate"),
                      log=lambda m: None, uniform_s=uniform)
        try:  # HBM bytes per launch from the committed PMC passes of tools/aggbench.py
            with open(os.path.join(REPO, "profiles", pmc_file)) as fh:
                pmc = json.load(fh)["kernels"]
        except (OSError, ValueError, KeyError):
            pmc = {}
        sub = {"config": "synthetic |V|=%d |E|=%d R2=%d d=%d, %s" % (res["V"], res["E"], res["R2"], res["d"],
                                                                   res["sources"]),
               "bytes_per_launch": res["b_agg_bytes"]}
        for k, kern in (("union_aggregate", "k_union_runs<false, false>"),
                        ("union_aggregate_src_runs", "k_union_runs<false, true>"),
                        ("lorentz_aggregate", "k_lorentz_sum<2>")):
            tr = pmc.get(kern, {}).get("hbm_bytes")
            e = {"achieved": res[k]["algorithmic_GBps"], "frac": res[k]["hbm_frac"],
                 "avg_launch_us": round(res[k]["ms"] * 1e3, 1), "G_edges_per_s": res[k]["edges_per_s_G"],
                 "kernel": kern, "traffic": tr}
            if k == "union_aggregate_src_runs":  # its own algorithm's bytes: one row per distinct (row, source)
                b = res["b_agg_src_runs_bytes"]
                e["bytes_per_launch"] = b
                e["distinct_row_sources"] = res["distinct_row_sources"]
                e["achieved"] = round(b / (res[k]["ms"] * 1e-3) / 1e9, 1)
                e["frac"] = round(e["achieved"] / HBM_PEAK_GBS, 4)
            if tr:
                e["traffic_GBps"] = round(tr / (res[k]["ms"] * 1e-3) / 1e9, 1)
                e["traffic_frac"] = round(e["traffic_GBps"] / HBM_PEAK_GBS, 4)
                e["traffic_source"] = "profiles/%s (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE of tools/aggbench.py%s)" % (
                    pmc_file, " --uniform-src" if uniform else "")
            sub[k] = e
        out[tag] = sub
        torch.cuda.empty_cache()
    return out


CPU_MAX_TRIPLES = 256


def cpu_baseline(cfg, d, model, sample, budget):
    """Time the CPU oracle (restatement of the reference op sequence) on one sample."""
    log("  cpu baseline (%s)" % cfg["label"])
    sys.path.insert(0, REPO)
    from oracle import graph as OG
    from oracle import model as OM
    hist, glist, _, test_np = sample
    V, R = cfg["V"], cfg["R"]
    torch.set_num_threads(cpu_threads())
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    ocfg = dict(c=0.01, n_layers=2, n_bases=cfg["n_bases"], radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
                radius_anchor_beta=1.0, radius_msg_gamma=0.15, use_residual_evolution=True, layer_norm=False,
                encoder=cfg["encoder"], decoder=cfg["decoder"])
    og = [OG.build_sub_graph(V, R, s) for s in hist]
    # a bounded sample: the full encoder over the window, the decoders on at most 256 test
    # triples (512 queries; ICEWS18's 3,080 queries x 23k candidates take the per-pair oracle
    # minutes), the same queries for the MRR parity below
    test_np = test_np[:CPU_MAX_TRIPLES]
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
                kind="port", **cpu_info(),
                sample="%d x oracle predict (%s, history %d, %d queries) on host CPU; %.2f s each"
                       % (len(times), cfg["label"], cfg["T"], 2 * len(test_np), per)), mrr


def _ctx():
    """(world, rank, device, backend): one process per GPU; BENCH_DIST_BACKEND=gloo rehearses
    several ranks on one card."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=device)
            else:
                dist.init_process_group(backend)
    return world, rank, device, backend


def _timed(world, device, backend, run, edges_local):
    """Barrier + synchronise, run(), synchronise + barrier; returns (elapsed max over ranks,
    edges summed over ranks)."""
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed, float(edges_local)], dtype=torch.float64,
                         device=device if backend == "nccl" else "cpu")
        tm = t.clone()
        dist.all_reduce(tm[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        return float(tm[0]), float(t[1])
    return elapsed, float(edges_local)


def cpu_threads():
    """Threads for the CPU baseline: every core this process may use.  On the GPU box one
    GPU's job gets a share of the host (the harness sets OMP_NUM_THREADS to it, 16 per GPU)
    while os.cpu_count() reports the whole machine, which the other GPUs' jobs share."""
    share = os.environ.get("OMP_NUM_THREADS")
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    return max(1, min(aff, int(share))) if share and share.isdigit() else aff


def cpu_info():
    """Host CPU model and the threads the CPU baseline used (lscpu model
    and core count)."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "host_logical_cpus": os.cpu_count(),
            "threads_note": "cores = the CPU share this process is given (OMP_NUM_THREADS / affinity); the "
                            "host's logical CPUs serve all of its GPUs' jobs"}


# ------------------------------------------------------------------------- dataset configs
def run_small(args, cfg, world, rank, device, backend, extras=True):
    """The dataset-sized configs: pools of independent predicts (see the module docstring).
    Whole pool passes are timed (steps rounded up to a multiple of the pool when the pool
    runs as one HIP graph), so the value does not depend on the step count."""
    d = args.d
    pool_n = args.pool or 48
    model = build_model(cfg, d, device, seed=1234)          # same weights on every rank
    model.use_phases = args.encoder_launches != "layers"
    model.memo_pristine = model.param_caches = args.serving_cache
    sharded = args.shard != "replica" and world > 1
    # replicas: independent data per rank; sharded: every rank holds the same snapshots
    samples = make_samples(cfg, pool_n, device, seed=100 if sharded else 100 + 7919 * rank,
                           shard=args.shard if sharded else "replica")
    no_graph = args.no_graph or sharded  # sharded: collectives between the launches, eager
    R = cfg["R"]

    def eager(i):
        _, glist, test, _ = samples[i]
        return model.predict(glist, R, None, test, True)

    conc = max(1, min(args.concurrent, len(samples)))
    lanes = [torch.cuda.Stream(device) for _ in range(conc)] if conc > 1 and not no_graph else []
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
    if lanes and gs != len(samples):
        raise SystemExit("--concurrent needs the whole-pool HIP graph (no --graph-steps)")
    if not no_graph:
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

    # whole pool passes only when the pool is one graph launch (the value would otherwise
    # depend on steps mod pool: the remainder would replay single-predict latency graphs)
    steps = args.steps
    if pool_graph is not None:
        steps = -(-steps // len(samples)) * len(samples)

    def run_steps():
        k = 0
        while k < steps:
            if pool_graph is not None:
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
    edges_local = sum(epw[k % len(samples)] for k in range(steps))
    elapsed, edges_total = _timed(world, device, backend, run_steps, edges_local)
    if sharded:  # every rank processed the same edges: count them once
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
                            "same kernels are the config-5 headline's")
        kernels = {k: dict(avg_us=round(v["ms"] * 1e3, 3), per_step=v["per_step"], bound=v["bound"],
                           achieved=round(v["achieved"], 3), unit=v["unit"], frac=round(v["frac"], 4))
                   for k, v in kern.items()}
        enc_us = sum(v["ms"] * 1e3 * v["per_step"] for k, v in kern.items() if k.startswith(("k_phase", "k_zero", "k_cold")))
        e_step = float(np.mean(epw))
        breakdown = {"encoder_kernels_us_per_step": round(enc_us, 2),
                     "encoder_M_edges_per_s": round(e_step / enc_us, 3) if enc_us else None,
                     "note": "kernel time only (sum of the stage launches' HIP-event averages, the phase "
                             "launches of one timestep x history_len); value is end to end"}
        cpu = mrr = None
        if extras and not args.no_cpu_baseline and world == 1:
            cpu, mrr = cpu_baseline(cfg, d, model, samples[0], args.cpu_budget)
        ms = elapsed / steps * 1e3
        out = {"metric": METRIC, "value": round(value, 3), "unit": "M edges/s", "n_gpus": world,
               "steps": steps, "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
               "scaling": "strong" if sharded else "weak", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic (%s-shaped snapshots, random-init weights)" % args.config.split("_")[0],
               "config": {"workload": cfg["label"], "V": cfg["V"], "R": cfg["R"], "triples_per_snapshot":
                          cfg["per_snap"], "history_len": cfg["T"], "n_layers": 2, "d": d,
                          "edges_per_step": int(np.mean(epw)), "queries_per_step": 2 * cfg["per_snap"],
                          "hip_graph": bool(graphs), "steps_per_graph_launch": len(samples) if pool_graph else 1,
                          "concurrent_samples": conc if lanes else 1,
                          "encoder_launches": "per-layer" if not model.use_phases else "timestep phases",
                          "serving_cache": bool(args.serving_cache), "batch_shared_states": share,
                          "parallelism": ("%s-partitioned snapshots x%d" % (args.shard, world)) if sharded
                          else "replicas x%d" % world},
               "latency_ms_per_predict": round(lat_ms, 4) if lat_ms else None,
               "roofline": roof, "kernels": kernels, "breakdown": breakdown,
               "cpu_baseline": cpu, "mrr_parity": mrr}
    del graphs, pool_graph, samples, model
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def run_regcn(args, cfg, world, rank, device, backend):
    """BASELINE.json configs[0]: the Euclidean RE-GCN (`RecurrentRGCN` + ConvTransE / ConvTransR,
    src/rrgcn.py:142-194, src/decoder.py:10-100) at ICEWS14s' shape (|V| = 7,128, R = 230, 246
    triples per snapshot, history 3, d = 200, the reference's ICEWS14s command: self-loop, layer
    norm).  A step is one `predict`; a pool of 16 independent predicts is captured into one HIP
    graph and whole pool passes are timed.  The CPU baseline is the oracle's `euclid_predict`
    (oracle/model.py:330) on the host cores, and the MRR of both on the same sample is compared."""
    from regcn_amd import graph as G
    from regcn_amd.rrgcn import RecurrentRGCN
    from regcn_amd.synthetic import snapshot_series
    d, V, R, T = args.d, cfg["V"], cfg["R"], cfg["T"]
    pool_n = args.pool or 48
    torch.manual_seed(1234)
    model = RecurrentRGCN("convtranse", "uvrgcn", V, R, 0, 0, d, "sub", T, num_bases=cfg["n_bases"],
                          num_basis=cfg["n_bases"], num_hidden_layers=2, dropout=0.2, self_loop=True,
                          layer_norm=True, input_dropout=0.2, hidden_dropout=0.2, feat_dropout=0.2,
                          entity_prediction=True, relation_prediction=True, use_cuda=True, gpu=0)
    model = model.to(device).eval()
    snaps = snapshot_series(100 + 7919 * rank, V, R, T + pool_n, cfg["per_snap"])
    samples = []
    for i in range(pool_n):
        glist = [G.build_sub_graph(V, R, s, True, device) for s in snaps[i:i + T]]
        samples.append((snaps[i:i + T], glist, torch.from_numpy(snaps[i + T]).to(device), snaps[i + T]))

    def eager(i):
        _, glist, test, _ = samples[i]
        return model.predict(glist, R, None, test, True)

    cap = torch.cuda.Stream(device)
    conc = max(1, min(args.concurrent, len(samples)))
    lanes = [torch.cuda.Stream(device) for _ in range(conc)] if conc > 1 else []

    def pool_pass(origin):  # sample i on lane i % conc, forked from and joined back into origin
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
        for i in range(len(samples)):
            eager(i)
        torch.cuda.synchronize()
        pool_graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(cap):
            pool_pass(cap)  # warm the capture streams' allocator pools
            torch.cuda.synchronize()
            with torch.cuda.graph(pool_graph, stream=cap):
                pool_pass(cap)
    pool_graph.replay()
    torch.cuda.synchronize()
    steps = -(-args.steps // len(samples)) * len(samples)
    epw = [edges_per_step(s[1]) for s in samples]
    edges_local = sum(epw) * (steps // len(samples))

    def run_steps():
        for _ in range(steps // len(samples)):
            pool_graph.replay()

    elapsed, edges_total = _timed(world, device, backend, run_steps, edges_local)
    value = edges_total / elapsed / 1e6
    out = None
    if rank == 0:
        cpu = mrr = None
        if not args.no_cpu_baseline and world == 1:
            log("  cpu baseline (%s)" % cfg["label"])
            sys.path.insert(0, REPO)
            from oracle import graph as OG
            from oracle import model as OM
            torch.set_num_threads(cpu_threads())
            hist, glist, test, test_np = samples[0]
            sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
            og = [OG.build_sub_graph(V, R, s) for s in hist]
            times = []
            t_end = time.time() + args.cpu_budget
            with torch.no_grad():
                while True:
                    t0 = time.time()
                    o_tr, o_score, o_score_rel = OM.euclid_predict(sd, dict(layer_norm=True, n_layers=2), og,
                                                                    torch.from_numpy(test_np))[:3]
                    times.append(time.time() - t0)
                    if time.time() > t_end or len(times) >= 5:
                        break
                _, score, score_rel = model.predict(glist, R, None, test, True)
            per = float(np.mean(times))
            cpu = dict(value=epw[0] / per / 1e6, unit="M edges/s", cores=torch.get_num_threads(), kind="port",
                       **cpu_info(), sample="%d x oracle euclid_predict (%s, history %d, %d queries); %.3f s each"
                       % (len(times), cfg["label"], T, 2 * len(test_np), per))
            mrr = {}
            for name, got, ref, rel in (("entity", score, o_score, False), ("relation", score_rel, o_score_rel, True)):
                ans = OM.answers_for_filter(test_np, R, rel_p=rel)
                f_g, r_g = OM.total_rank(o_tr, got.float().cpu(), ans, rel)[:2]
                f_o, r_o = OM.total_rank(o_tr, ref.float(), ans, rel)[:2]
                mrr[name] = {"raw_hip": round(r_g, 6), "raw_oracle": round(r_o, 6), "filtered_hip": round(f_g, 6),
                             "filtered_oracle": round(f_o, 6),
                             "max_abs_delta": round(max(abs(r_g - r_o), abs(f_g - f_o)), 6)}
            mrr["tolerance"] = 0.002
        out = {"metric": METRIC, "value": round(value, 3), "unit": "M edges/s", "n_gpus": world, "steps": steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed / steps * 1e3, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic (ICEWS14s-shaped snapshots, random-init weights)",
               "config": {"workload": cfg["label"] + " (BASELINE.json configs[0]): RecurrentRGCN.predict, "
                          "layer norm, self-loop, ConvTransE + ConvTransR", "V": V, "R": R,
                          "triples_per_snapshot": cfg["per_snap"], "history_len": T, "n_layers": 2, "d": d,
                          "edges_per_step": int(np.mean(epw)), "queries_per_step": 2 * cfg["per_snap"],
                          "hip_graph": True, "steps_per_graph_launch": len(samples), "concurrent_samples": conc,
                          "parallelism": "replicas x%d" % world},
               "cpu_baseline": cpu, "mrr_parity": mrr}
    del pool_graph, samples, model
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


# ------------------------------------------------------------------------ the printed line
LINE_LIMIT = 8192  # bytes: the driver parses the last stdout line from a bounded tail


def _rnd(x, n=4):
    return None if x is None else round(float(x), n)


def _cpu_short(c):
    if not c:
        return None
    return {"value": _rnd(c["value"], 6), "unit": c["unit"], "cores": c["cores"], "kind": c["kind"],
            "sample": c["sample"][:160], "cpu_model": c.get("cpu_model")}


def _roof_short(r, kernels=None):
    if not r:
        return None
    keep = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "traffic_GBps", "traffic_frac",
            "avg_launch_us", "launches_per_step", "algorithmic_bytes_per_launch", "flops_per_launch")
    s = {k: r[k] for k in keep if r.get(k) is not None}
    for k in ("algorithmic_bytes_per_launch", "flops_per_launch"):
        if k in s:
            s[k] = float("%.4g" % s[k])
    if s.get("traffic"):
        s["traffic_unit"] = "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, %s)" % (
            (r.get("traffic_source") or "profiles/").split(" ")[0])
    l2 = (kernels or {}).get(r.get("call"), {}).get("l2_request_stream")
    if l2:
        s["l2_request_stream"] = {"requests_per_launch": float("%.4g" % l2["requests_per_launch"]),
                                  "achieved_TBps": l2["achieved_TBps"], "ceiling_TBps": l2["ceiling_TBps"],
                                  "frac": l2["frac"]}
    return s


def _leg_short(r):
    s = {k: r.get(k) for k in ("value", "ms_per_step", "latency_ms_per_predict") if r.get(k) is not None}
    rf = r.get("roofline")
    if rf:
        s["roofline"] = {k: rf.get(k) for k in ("kernel", "bound", "frac", "avg_launch_us")}
    c = r.get("cpu_baseline")
    if c:
        s["cpu_baseline"] = {"value": _rnd(c["value"], 7), "cores": c["cores"], "kind": c["kind"]}
    m = r.get("mrr_parity")
    if m:
        s["mrr_max_abs_delta"] = max(m[k]["max_abs_delta"] for k in ("entity", "relation") if k in m)
    return s


def compact_line(out, detail_path=None):
    """The bench line the driver parses (<= LINE_LIMIT bytes): the contract keys, the headline's
    roofline and cpu_baseline, a one-line owner simulation, each dataset leg's value, roofline
    fraction and cpu_baseline.  The full record (per-call kernels, rooflines at scale, per-rank
    arrays) goes to `detail_path`."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    line = {k: out.get(k) for k in keep}
    cfg = {k: v for k, v in (out.get("config") or {}).items() if k != "snapshot_stats"}
    if isinstance(cfg.get("workload"), str):
        cfg["workload"] = cfg["workload"][:220]
    line["config"] = cfg
    line["roofline"] = _roof_short(out.get("roofline"), out.get("kernels"))
    line["cpu_baseline"] = _cpu_short(out.get("cpu_baseline"))
    if out.get("latency_ms_per_predict") is not None:
        line["latency_ms_per_predict"] = out["latency_ms_per_predict"]
    b = out.get("breakdown") or {}
    if "encoder_ms_per_step" in b:
        line["breakdown"] = {"encoder_ms_per_step": b["encoder_ms_per_step"],
                             "decoder_ms_per_step": b.get("decoder_ms_per_step")}
    kern = out.get("kernels") or {}
    if kern and "avg_us" in next(iter(kern.values())):
        top = sorted(kern.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1].get("per_step", 1))[:6]
        line["top_calls_us"] = {k: [v["avg_us"], v.get("per_step"), v.get("frac")] for k, v in top}
    sim = out.get("owner_simulation")
    if sim:
        line["owner_simulation"] = {
            "world": sim["world"], "predicted_step_ms": sim["predicted_step_ms"],
            "speedup_vs_headline": sim.get("predicted_speedup_vs_headline"), "max_rank_ms": sim["max_rank_ms"],
            "mean_rank_ms": sim["mean_rank_ms"], "sum_rank_ms": round(sim["mean_rank_ms"] * sim["world"], 3),
            "exposed_exchange_ms": sim["exposed_exchange_ms_per_step"], "replicated_ms": sim["replicated_ms"],
            "receive_ms_max": max(sim.get("receive_ms_per_rank") or [0.0]),
            "predicted_step_ms_links_derated": sim.get("predicted_step_ms_links_derated"),
            "blocker_margin_ms": sim.get("blocker_margin_ms")}
    ag = out.get("aggregation_roofline")
    if ag:
        u = ag.get("uniform_src", {}).get("union_aggregate", {})
        z = ag.get("zipf_src", {}).get("union_aggregate", {})
        line["aggregation_roofline"] = {"union_uniform_src": {"frac": u.get("frac"), "traffic_frac": u.get("traffic_frac"),
                                                              "avg_launch_us": u.get("avg_launch_us")},
                                        "union_zipf_src": {"frac": z.get("frac"), "traffic_frac": z.get("traffic_frac"),
                                                           "avg_launch_us": z.get("avg_launch_us")}}
    dr = out.get("decoder_roofline")
    if dr:
        line["decoder_roofline"] = {"score_frac": dr["score"]["frac"], "ce_frac": dr["cross_entropy"]["frac"],
                                    "score_us": dr["score"]["avg_launch_us"]}
    for k in ("owner_partition", "edge_partition"):
        if out.get(k):
            line[k] = {kk: out[k][kk] for kk in ("value", "ms_per_step", "scaling", "parallelism") if kk in out[k]}
    if out.get("mrr_parity"):
        m = out["mrr_parity"]
        line["mrr_parity"] = {"max_abs_delta": max(m[k]["max_abs_delta"] for k in ("entity", "relation") if k in m),
                              "tolerance": m.get("tolerance"), "workload": (m.get("workload") or "")[:60]}
    legs = {k: _leg_short(out[k]) for k in LEGS if isinstance(out.get(k), dict)}
    if legs:
        line["legs"] = legs
    if detail_path:
        line["detail"] = detail_path
    s = json.dumps(line, separators=(",", ":"))
    for drop in ("top_calls_us", "aggregation_roofline", "decoder_roofline", "breakdown"):
        if len(s) <= LINE_LIMIT:
            break
        line.pop(drop, None)
        s = json.dumps(line, separators=(",", ":"))
    return s


def write_detail(out):
    """The full record beside the line (BENCH_DETAIL, default gpurun_out/bench_detail.json)."""
    path = os.environ.get("BENCH_DETAIL", os.path.join("gpurun_out", "bench_detail.json"))
    try:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as fh:
            json.dump(out, fh)
        return path
    except OSError:
        return None


LEGS = ("icews14s", "icews14s_regcn", "icews18", "gdelt", "gdelt_lgcn")


# --------------------------------------------------------------------------- config 5
SCALE_KERNEL = {  # library call -> its main kernel (rocprof / PMC name)
    "regcn_union_aggregate_f32": "k_union_runs<false, false>",
    "regcn_union_aggregate_src_runs_f32": "k_union_runs<false, true>",
    "regcn_segment_mean_f32": "k_gather_sum<1>",
    "regcn_layer_f32": "k_layer<0, 1, false>",
    "regcn_layer_f32(step)": "k_layer<0, 1, true>",
    # one call = the crel gather over the big tiles + the plain gather over the rest
    "regcn_layer_rowtail_f32(gather)": "k_gather_crel<0, 32> + k_gather_agg<0, 1>",
    "regcn_layer_rowtail_f32": "k_rowtail2<13, 1>",
    "regcn_layer_rowtail_f32(step)": "k_rowtail3<13, 3>",
    "regcn_timestep_phase_f32(A)": "k_phase_a",
    "regcn_timestep_phase_f32(B)": "k_phase_b<0, 1>",
    "regcn_timestep_phase_f32(C)": "k_phase_c<0, 1>",
    "regcn_zero_step_f32": "k_zero_step",
    "regcn_hyp_score_jobs_f32": "k_score_f32_jobs",
    "regcn_roth_queries_f32": "k_queries4",
    "regcn_relation_gru_x_f32": "k_rel_gru_x",
    "regcn_relation_gru_pre_f32": "k_rel_gru_pre",
    "regcn_init_entities_f32": "k_init_rows4<11>",
}


def heavy_distinct_sources(g):
    """Distinct (row, source) pairs over the hub rows (the pre-aggregated rows): the source
    rows regcn_union_aggregate_src_runs_f32 gathers."""
    wk = g.work()
    hc = wk["heavy_chunks"]
    if not hc.numel():
        return 0
    ss = g.row_src_cols()
    rp = wk["rowptr"].long()
    E, V = ss.numel(), rp.numel() - 1
    head = torch.ones(E, dtype=torch.bool, device=ss.device)
    head[1:] = ss[1:] != ss[:-1]
    starts = rp[:-1]
    head[starts[starts < E]] = True
    mark = torch.zeros(V, dtype=torch.bool, device=ss.device)
    mark[hc[:, 0].long()] = True
    dst = torch.repeat_interleave(torch.arange(V, device=ss.device), rp[1:] - rp[:-1])
    return int((head & mark[dst]).sum())


def scale_work(model, glist, B):
    """Algorithmic (flops, bytes) per launch of each library call of one config-5 predict,
    averaged over the window's snapshots (gathered source row + indices +
    radius per edge; row reads/writes per node; d x d products 2 d^2 flops per row)."""
    d = model.dynamic_emb.shape[1]
    V = model.num_ents
    R2 = 2 * model.num_rels
    gemm = 2.0 * d * d
    row = 4.0 * d
    st = []
    for g in glist:
        wk = g.work()
        hc = wk["heavy_chunks"]
        e_heavy = int((hc[:, 2] - hc[:, 1]).sum()) if hc.numel() else 0
        st.append(dict(n_pos=g.n_pos, items=int(wk["item_src"].numel()), e_heavy=e_heavy, n_heavy=g.n_heavy,
                       pairs=int(wk["rel_idx"].numel()) // 2, heavy_sources=heavy_distinct_sources(g)))
    m = {k: float(np.mean([x[k] for x in st])) for k in st[0]}
    per_edge = row + 12.0  # source row + col_src + col_type + radius[src]
    io_layer = V * (row + 4) + V * (2 * row + 4) + V * 4.0  # x, r in; h, x', r' out; norm
    w = {
        "regcn_union_aggregate_f32": (0.0, m["e_heavy"] * per_edge + m["n_heavy"] * (row + 12)),
        # source runs: one gathered row per distinct (row, source); per edge (src, type) and
        # radius[src] in type order, src and radius[src] in source order
        "regcn_union_aggregate_src_runs_f32": (0.0, m["heavy_sources"] * row + m["e_heavy"] * 20.0
                                               + m["n_heavy"] * (row + 12)),
        "regcn_segment_mean_f32": (0.0, m["pairs"] * (row + 4) + R2 * row),
        "regcn_layer_f32": (gemm * (m["n_pos"] + V), m["items"] * per_edge + m["n_heavy"] * row + io_layer),
        "regcn_layer_f32(step)": (gemm * (m["n_pos"] + 2 * V),
                                  m["items"] * per_edge + m["n_heavy"] * row + io_layer + V * (2 * row + 4)),
        # the large-snapshot layer as two launches (csrc/rowtail.hip): the inline rows' gather
        # into the agg buffer, then the 64-row tail (the first layer also computes the time-gate
        # product and writes it; the step layer reads it back with x_prev for the blend)
        "regcn_layer_rowtail_f32(gather)": (0.0, m["items"] * per_edge + (m["n_pos"] - m["n_heavy"]) * (row + 8)),
        "regcn_layer_rowtail_f32": (gemm * (m["n_pos"] + 2 * V), m["n_pos"] * row + V * (row + 4) + V * row
                                    + V * (2 * row + 4)),
        "regcn_layer_rowtail_f32(step)": (gemm * (m["n_pos"] + V), m["n_pos"] * row + V * (row + 4) + 2 * V * row
                                          + V * (2 * row + 8)),
        "regcn_timestep_phase_f32(A)": (2 * gemm * m["n_pos"] + 2.0 * R2 * 3 * d * d,
                                        V * row + 2 * m["n_pos"] * row + 4.0 * R2 * d * 3 + 4.0 * 3 * d * d),
        "regcn_timestep_phase_f32(B)": (2 * gemm * m["n_pos"], m["items"] * per_edge + m["n_heavy"] * row
                                        + m["n_pos"] * 3 * row),
        "regcn_timestep_phase_f32(C)": (gemm * m["n_pos"], m["items"] * per_edge + m["n_heavy"] * row
                                        + m["n_pos"] * 5 * row),
        "regcn_zero_step_f32": (3 * gemm * (V - m["n_pos"]), (V - m["n_pos"]) * 3 * row),
        "regcn_hyp_score_jobs_f32": (2.0 * B * (V + R2) * d, 4.0 * (B * (V + R2) + (V + R2) * d)),
        "regcn_roth_queries_f32": (2.0 * B * 5.5 * d * d, 4.0 * (B * d * 5 + R2 * d * 2)),
        "regcn_init_entities_f32": (0.0, V * (3 * row + 8)),
    }
    return w, m


def summarize_trace(trace, steps):
    """Per library call: launches per step and mean device ms per launch, from the events
    recorded after each call (the interval since the previous event on the same stream)."""
    per = {}
    prev = None
    for name, ev in trace:
        if prev is not None and name != "__step__":
            per.setdefault(name, []).append(prev.elapsed_time(ev))
        prev = ev
    return {k: dict(ms=float(np.mean(v)), per_step=len(v) / steps) for k, v in per.items()}


def pmc_for(kernel, config, d):
    path = os.path.join(REPO, "profiles", "pmc_traffic_%s.json" % config)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        pm = json.load(f)
    if pm.get("config") != config or int(pm.get("d", -1)) != d:
        return None, None
    names = kernel.split(" + ")  # a call of several kernels: their bytes per launch summed
    ks = [pm["kernels"].get(n) for n in names]
    if any(k is None for k in ks):
        return None, None
    return sum(k["hbm_bytes"] for k in ks), "profiles/pmc_traffic_%s.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, %s launches)" % (
        config, " + ".join(str(k["launches"]) for k in ks))


L2_GATHER_CEILING_TBPS = 16.8  # rows gathered from the XCD's L2, chip-wide (MI355X_MICROARCH.md, lower end)


def l2_request_stream(config, ms):
    """The inline gather against the L2-gather ceiling: L1 <- L2 read requests per launch of its
    kernels (rocprofv3 TCP_TCC_READ_REQ_sum, summed over the gather's kernels, from
    profiles/pmc_l2req_<config>.json) x 128 B over the call's measured time."""
    path = os.path.join(REPO, "profiles", "pmc_l2req_%s.json" % config)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        pm = json.load(f)
    req = float(pm["gather_requests_per_launch"])
    tbps = req * 128.0 / (ms * 1e-3) / 1e12
    return {"requests_per_launch": req, "bytes_per_launch": req * 128.0, "achieved_TBps": round(tbps, 2),
            "ceiling_TBps": L2_GATHER_CEILING_TBPS, "frac": round(tbps / L2_GATHER_CEILING_TBPS, 4),
            "kernels": pm.get("kernels"), "source": "profiles/pmc_l2req_%s.json" % config}


def cpu_baseline_scale(cfg, d, budget):
    """The CPU oracle's encoder forward (oracle/model.py hyperbolic_forward, the reference op
    sequence with per-edge message materialisation) over ONE snapshot at |V| = 1M with a
    bounded edge count (full |E| = 50M is infeasible on the host)."""
    sys.path.insert(0, REPO)
    from oracle import graph as OG
    from oracle import model as OM
    from regcn_amd.synthetic import snapshot_series
    torch.set_num_threads(cpu_threads())
    V, R = cfg["V"], cfg["R"]
    triples = 2_500_000
    snap = snapshot_series(7, V, R, 1, triples)[0]
    g = OG.build_sub_graph(V, R, snap)
    del snap
    m = build_model(dict(cfg, V=V), d, torch.device("cpu"), seed=1234)
    sd = {k: v.detach() for k, v in m.state_dict().items()}
    del m
    ocfg = dict(c=0.01, n_layers=2, n_bases=cfg["n_bases"], radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
                radius_anchor_beta=1.0, radius_msg_gamma=0.15, use_residual_evolution=True, layer_norm=False,
                encoder=cfg["encoder"], decoder=cfg["decoder"])
    times = []
    t_end = time.time() + budget
    with torch.no_grad():
        while True:
            t0 = time.time()
            OM.hyperbolic_forward(sd, ocfg, [g])
            times.append(time.time() - t0)
            if time.time() > t_end or len(times) >= 3:
                break
    per = float(np.mean(times))
    edges = 2 * 2 * triples  # directed edges x 2 layers
    return dict(value=round(edges / per / 1e6, 4), unit="M edges/s", cores=torch.get_num_threads(), kind="port",
                sample="%d x oracle encoder forward (1 snapshot, |V|=%d, |E|=%d directed, R2=%d, d=%d, 2 layers: "
                       "%d message edges; the full |E|=50M window is infeasible on the host), %.2f s each"
                       % (len(times), V, 2 * triples, 2 * R, d, edges, per), **cpu_info())


def prepare_snapshot(V, R, triples, device, prep=None):
    """One config-5 snapshot in HBM with every list a predict reads (graph build on the device,
    then the row/type and row/source orders, inline items in source order, the entity-block
    relation and hub lists -- otherwise built lazily by the first predict); `prep` collects
    the build and list times in ms (synchronised)."""
    from regcn_amd import graph as G
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = G.build_sub_graph(V, R, triples, True, device)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    g.row_type_cols()
    g.row_src_cols()
    if g.use_item_src_runs():
        g.item_src_cols()
    G.rel_block_work(g, R)
    G.hub_block_work(g)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if prep is not None:
        prep.append((1e3 * (t1 - t0), 1e3 * (t2 - t1)))
    return g


def owner_simulation(args, cfg, device, world):
    """The config-5 owner partition for `world` GPUs, simulated on this one:
    entity ids relabelled for equal edge loads (EntityRelabel.balanced), every snapshot a
    parallel.RankSimulation, so each layer runs rank 0's chunk launches, then rank 1's, ...
    (each rank's device time from HIP events around its launches), the relation means sum the
    ranks' partials, and the decoder scores each rank's own rows as its candidates.  Reports
    the per-rank device ms per step, the replicated ms (what every rank runs: initial state,
    relation GRU, queries, target scores, relation decoder), the all-gather volume, and the
    step a rank would take with the exchange hidden under its compute."""
    from regcn_amd.graph import hub_block_work  # noqa: F401
    from regcn_amd.parallel import SIM_MARKERS, CandidateShard, EntityRelabel, RankSimulation
    from regcn_amd.synthetic import snapshot_series
    d, T, V, R = args.d, cfg["T"], cfg["V"], cfg["R"]
    snaps = snapshot_series(100, V, R, T + 1, cfg["per_snap"])
    rl = EntityRelabel.balanced(snaps[:T], V, world)
    loads = rl.loads(snaps[:T], world)
    loads_plain = EntityRelabel(np.arange(V)).loads(snaps[:T], world)
    snaps = [rl.triples(x) for x in snaps]
    t0 = time.time()
    sims = [RankSimulation(prepare_snapshot(V, R, x, device), world) for x in snaps[:T]]
    setup_s = time.time() - t0
    test = torch.from_numpy(np.ascontiguousarray(snaps[T][:args.queries // 2])).to(device)
    del snaps
    model = build_model(cfg, d, device, seed=1234)
    rl.model(model)
    model.memo_pristine = model.param_caches = False
    dec = model.decoder_ob
    lay = sims[-1].layout
    shards = [CandidateShard(V, k, world, None, ranges=lay.ranges(k)) for k in range(world)]
    kw = dict(scale=dec.score_scale_raw, margin=dec.score_margin, raw_scale=True)
    dec_times = [[] for _ in range(world)]

    def step():
        model.__dict__["_owner_rows_only"] = True  # as predict_ranks: no exchange after the last layer
        try:
            embs, _, r_emb, _, _ = model.forward(sims, None, True)
        finally:
            model.__dict__.pop("_owner_rows_only", None)
        inv = test.flip(1)
        inv[:, 1] = inv[:, 1] + R
        at = torch.cat([test, inv])
        emb = embs[-1]
        q = dec._query(emb, r_emb, at)
        ts = shards[0].target_scores(q, emb, None, at[:, 2], dec.c, **kw)
        for k, sh in enumerate(shards):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if SIM_MARKERS:
                torch.cuda._sleep(1)
            a.record()
            sh.range_ranks(q, emb, None, dec.c, ts, **kw)
            b.record()
            if SIM_MARKERS:
                torch.cuda._sleep(1)
            dec_times[k].append((a, b))
        model.rdecoder.forward(emb, r_emb, at, mode="test")

    reps = 3

    def reset():
        for sm in sims:
            sm.times = [[] for _ in range(world)]
            sm.chunk_marks = [[] for _ in range(world)]
            sm.delivery = []
            for sg in sm.ranks:
                sg.exchanged_bytes = 0
        for k in range(world):
            dec_times[k].clear()

    def timed(blocker):
        """reps simulated steps; blocker: a device-side wait before each step, during which
        the host enqueues the whole step, so the step's launches run back to back (device
        time, no host-issue gaps).  Returns the mean ms per step."""
        reset()
        tot = 0.0
        gc_on = gc.isenabled()
        gc.disable()  # a collector pause while the host enqueues must not outlast the blocker
        try:
            for _ in range(reps):
                t0 = time.perf_counter()
                if blocker:
                    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s0.record()
                    torch.cuda._sleep(SIM_BLOCKER_CYCLES)
                    s1.record()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                step()
                b.record()
                if not blocker:
                    continue
                host_ms = (time.perf_counter() - t0) * 1e3
                torch.cuda.synchronize()
                tot += a.elapsed_time(b)
                # device time only if the whole step was enqueued before the wait ended
                margin[0] = min(margin[0], s0.elapsed_time(s1) - host_ms)
        finally:
            if gc_on:
                gc.enable()
        torch.cuda.synchronize()
        return tot / reps if blocker else a.elapsed_time(b)

    margin = [float("inf")]

    with torch.no_grad():
        step()
        torch.cuda.synchronize()
        t_host = time.perf_counter()
        timed(False)  # as issued (the host's launch rate included): reported beside
        host_issued_ms = (time.perf_counter() - t_host) * 1e3 / reps
        issued_rank = np.sum([sm.per_rank_ms() for sm in sims], axis=0) / reps
        issued_dec = np.array([sum(a.elapsed_time(b) for a, b in t) for t in dec_times]) / reps
        total = timed(True)
    enc = np.sum([sm.per_rank_ms() for sm in sims], axis=0) / reps
    dec_ms = np.array([sum(a.elapsed_time(b) for a, b in t) for t in dec_times]) / reps
    per_rank = enc + dec_ms
    delivery = sum(sm.delivery_ms() for sm in sims) / reps
    replicated = total - float(per_rank.sum()) - delivery
    layers = 2 * T
    link_gbs, links = 153.0, world - 1  # xGMI: 7 links x ~153 GB/s per MI355X
    # received per rank per step (the sparse exchange: the rows the next layer reads; none
    # after the last layer), and the all-gather it replaces
    recv = np.array([sum(sm.ranks[k].exchanged_bytes for sm in sims) for k in range(world)]) / reps
    full_bytes = (world - 1) * lay.cr * lay.chunks * (d + 1) * 4
    xbytes = float(recv.max()) / layers
    xchg_ms = xbytes / (links * link_gbs * 1e9) * 1e3
    edges = 2 * sum(sm.number_of_edges() for sm in sims)
    # per rank: chunk j's exchange starts when chunk j's rows are final and the link is free;
    # the next layer waits for the last one (RankSimulation.exposed_exchange_ms)
    exp_k = np.sum([sm.exposed_exchange_ms(link_gbs) for sm in sims], axis=0) / reps
    # the receive side on a real node: RCCL's copy kernels land each received row in a FIFO in
    # the receiver's HBM and copy it to the halo rows (a read + a write of the bytes through HBM),
    # charged to the receiving rank at the measured 6.3 TB/s copy rate as if serialised with its
    # compute (an upper bound: the copies run on a few CUs beside the layer kernels)
    recv_ms = 2.0 * recv / (HBM_COPY_GBS * 1e9) * 1e3
    exposed = float(exp_k[int(np.argmax(per_rank + exp_k + recv_ms))])
    pred = float((per_rank + exp_k + recv_ms).max()) + replicated
    # the same with the peer links derated to LINK_DERATE of their nominal 153 GB/s
    exp_d = np.sum([sm.exposed_exchange_ms(link_gbs * LINK_DERATE) for sm in sims], axis=0) / reps
    pred_derated = float((per_rank + exp_d + recv_ms).max()) + replicated
    return {
        "world": world, "chunks_per_rank": lay.chunks, "rows_per_chunk": lay.cr,
        "per_rank_ms": [round(float(x), 3) for x in per_rank],
        "per_rank_encoder_ms": [round(float(x), 3) for x in enc],
        "per_rank_decoder_ms": [round(float(x), 3) for x in dec_ms],
        "max_rank_ms": round(float(per_rank.max()), 3), "mean_rank_ms": round(float(per_rank.mean()), 3),
        "replicated_ms": round(replicated, 3), "single_gpu_equivalent_ms": round(total, 3),
        "exchange_bytes_per_layer_per_rank": int(xbytes), "exchange_gb_per_step_per_rank": round(float(recv.max()) / 1e9, 3),
        "allgather_bytes_per_layer_per_rank": int(full_bytes),
        "exchange_ms_per_layer_at_7_links": round(xchg_ms, 3),
        "exposed_exchange_ms_per_rank": [round(float(x), 3) for x in exp_k],
        "exposed_exchange_ms_per_step": round(exposed, 3),
        "edge_loads_per_rank": loads, "edge_loads_contiguous_ids": loads_plain,
        "receive_ms_per_rank": [round(float(x), 3) for x in recv_ms],
        "predicted_step_ms": round(pred, 3),
        "predicted_M_edges_per_s": round(edges / pred / 1e3, 1),
        "predicted_step_ms_links_derated": round(pred_derated, 3),
        "link_derate": LINK_DERATE,
        "halo_delivery_ms_simulated": round(delivery, 3),
        "blocker_margin_ms": round(margin[0], 1),  # > 0: every timed step was enqueued before its wait ended
        "as_issued": {"host_ms_per_step": round(host_issued_ms, 3),
                      "max_rank_ms": round(float((issued_rank + issued_dec).max()), 3),
                      "note": "the same steps without the device-side wait: the one host issues all 8 ranks' "
                              "launches (~8x a real rank's), so ranks see its launch-rate gaps"},
        "setup_s": round(setup_s, 1),
        "note": "ranks run one after another on one MI355X (parallel.RankSimulation); per-rank = device time "
                "of its own launches (layer chunks incl. hub pass, relation-mean partials, its candidate "
                "slice with the fused score + rank count; the send-side gather of its exchanges); "
                "replicated = the rest of the step (initial state, relation GRU, queries, relation "
                "decoder; the halo delivery of the simulated all_to_alls, RCCL's work on a node, is in it "
                "too); each timed step starts behind a device-side wait so that its launches run back to "
                "back (device time; `as_issued` without it); predicted step = max over ranks of (rank + "
                "its exposed exchange) + replicated.  Exchange: per chunk two all_to_alls (x rows, |h|) of "
                "the rows the next layer reads (ExchangePlan) into the receivers' halo rows, its time = the "
                "busiest peer link's bytes at the nominal 153 GB/s, starting when the chunk's rows are final "
                "and the previous chunk's exchange is done; a layer exposes what runs past its last chunk.  "
                "Receive side: each rank's received bytes cross its HBM twice (RCCL's FIFO, then the halo "
                "rows) at the 6.3 TB/s copy rate, added to the rank as serialised time; the simulation's "
                "own delivery copies (one GPU scattering all 8 ranks' halos) are reported, not used",
    }


def run_scale(args, cfg, world, rank, device, backend):
    """Config 5 headline (see the module docstring)."""
    from regcn_amd import _lib
    from regcn_amd import graph as G
    from regcn_amd.synthetic import snapshot_series
    from regcn_amd.parallel import EntityRelabel, ShardedGraph
    d, T, V, R = args.d, cfg["T"], cfg["V"], cfg["R"]
    n_win = args.pool or 2
    t_setup = time.time()
    # replicas: own data per rank; --shard edge|owner: every rank holds the same snapshots and
    # processes its partition of each (strong scaling)
    sharded = args.shard != "replica" and world > 1
    snaps = snapshot_series(100 if sharded else 100 + 7919 * rank, V, R, T + n_win, cfg["per_snap"])
    relabel = None
    if sharded and args.shard == "owner":  # equal edge loads per rank (parallel.EntityRelabel)
        relabel = EntityRelabel.balanced(snaps[:T + n_win - 1], V, world)
        snaps = [relabel.triples(s) for s in snaps]
    graphs, prep = [], []
    for s in snaps[:T + n_win - 1]:
        graphs.append(prepare_snapshot(V, R, s, device, prep))
    if sharded:
        graphs = [ShardedGraph(g, args.shard) for g in graphs]
    tests = [torch.from_numpy(np.ascontiguousarray(snaps[T + i][:args.queries // 2])).to(device)
             for i in range(n_win)]
    del snaps
    windows = [graphs[i:i + T] for i in range(n_win)]
    model = build_model(cfg, d, device, seed=1234)
    if relabel is not None:
        relabel.model(model)
    model.use_phases = args.encoder_launches == "phases"
    model.memo_pristine = model.param_caches = False  # every step computes everything
    B = 2 * tests[0].shape[0]

    def step(k):
        i = k % n_win
        _lib.trace_mark("__step__")
        if sharded:  # the candidate-sharded decoder: every rank ranks its own candidates
            return model.predict_ranks(windows[i], R, None, tests[i], True)
        return model.predict(windows[i], R, None, tests[i], True)

    with torch.no_grad():
        for k in range(max(args.warmup, 1)):
            step(k)
    torch.cuda.synchronize()
    setup_s = time.time() - t_setup
    epw = [edges_per_step(w) for w in windows]
    edges_local = sum(epw[k % n_win] for k in range(args.steps))
    trace = []

    def run():
        _lib.EVENT_TRACE = trace
        try:
            with torch.no_grad():
                for k in range(args.steps):
                    step(k)
        finally:
            _lib.EVENT_TRACE = None

    for g in graphs if sharded else ():
        g.exchanged_bytes = 0
    elapsed, edges_total = _timed(world, device, backend, run, edges_local)
    xbytes = sum(getattr(g, "exchanged_bytes", 0) for g in graphs) / max(args.steps, 1) if sharded else 0
    if sharded:  # every rank processed its part of the same edges: count them once
        edges_total = float(edges_local)
    value = edges_total / elapsed / 1e6
    out = None
    if rank == 0:
        calls = summarize_trace(trace, args.steps)
        work, stats = scale_work(model, [getattr(g, "g", g) for g in windows[0]], B)
        if sharded:  # a rank's launches do its partition's share: no per-launch roofline
            work = {k: (0.0, 0.0) for k in work}
        kernels = {}
        for name, v in calls.items():
            flops, nbytes = work.get(name, (0.0, 0.0))
            e = dict(avg_us=round(v["ms"] * 1e3, 1), per_step=round(v["per_step"], 3),
                     kernel=SCALE_KERNEL.get(name, name))
            if flops or nbytes:
                wv = _work(flops, nbytes, v["ms"])
                e.update(bound=wv["bound"], achieved=round(wv["achieved"], 1), unit=wv["unit"],
                         frac=round(wv["frac"], 4))
            kernels[name] = e
        dom = max(calls, key=lambda k: calls[k]["ms"] * calls[k]["per_step"])
        flops, nbytes = work.get(dom, (0.0, 0.0))
        wv = _work(flops, nbytes, calls[dom]["ms"])
        kname = SCALE_KERNEL.get(dom, dom)
        traffic, tsrc = pmc_for(kname, args.config, d)
        roof = dict(bound=wv["bound"], kernel=kname, call=dom, achieved=round(wv["achieved"], 1),
                    peak=wv["peak"], unit=wv["unit"], frac=round(wv["frac"], 4), traffic=traffic,
                    traffic_source=tsrc, flops_per_launch=flops, algorithmic_bytes_per_launch=nbytes,
                    avg_launch_us=round(calls[dom]["ms"] * 1e3, 1), launches_per_step=calls[dom]["per_step"])
        if traffic:
            roof["traffic_GBps"] = round(traffic / (calls[dom]["ms"] * 1e-3) / 1e9, 1)
            roof["traffic_frac"] = round(roof["traffic_GBps"] / HBM_PEAK_GBS, 4)
        if roof["bound"] == "hbm" and roof["frac"] > 1.0:
            roof["note"] = ("achieved counts SURVEY.md §8(d)'s algorithmic bytes (a gathered 800-B source row per "
                            "edge); with Zipf(1.1) sources most of those rows are L2 / Infinity-Cache hits, so it "
                            "passes the HBM peak: the HBM figure is `traffic` (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE "
                            "of the same launch) and aggregation_roofline.uniform_src")
        gname = "regcn_layer_rowtail_f32(gather)"
        if gname in calls and not sharded:
            # the aggregation launch under SURVEY.md §8(d)'s count: 812 B per unit x its units
            # (inline in-edges + the rows it finishes)
            units = stats["items"] + stats["n_pos"] - stats["n_heavy"]
            b8 = units * (4.0 * d + 12)
            kernels[gname].update(s8d_bytes_per_launch=b8, s8d_units_per_launch=units,
                                  s8d_achieved_GBps=round(b8 / (calls[gname]["ms"] * 1e-3) / 1e9, 1))
            kernels[gname]["s8d_frac"] = round(kernels[gname]["s8d_achieved_GBps"] / HBM_PEAK_GBS, 4)
            l2 = l2_request_stream(args.config, calls[gname]["ms"])
            if l2:  # the bound that applies: rows gathered from the XCD's L2 (MI355X_MICROARCH.md)
                kernels[gname]["l2_request_stream"] = l2
        if dom.startswith("regcn_layer_f32") and not sharded:
            # SURVEY.md §8(d)'s count alone: 812 B per unit (gathered row + col_src + col_type +
            # radius per edge; row write + rowptr + norm + radius per node) x the launch's units
            # (its inline in-edges + every row); `achieved` above adds the timestep's row I/O
            units = stats["items"] + V
            b8 = units * (4.0 * d + 12)
            roof["s8d_bytes_per_launch"] = b8
            roof["s8d_units_per_launch"] = units
            roof["s8d_achieved_GBps"] = round(b8 / (calls[dom]["ms"] * 1e-3) / 1e9, 1)
            roof["s8d_frac"] = round(roof["s8d_achieved_GBps"] / HBM_PEAK_GBS, 4)
        ms = elapsed / args.steps * 1e3
        enc_ms = sum(v["ms"] * v["per_step"] for k, v in calls.items()
                     if k not in ("regcn_hyp_score_jobs_f32", "regcn_roth_queries_f32"))
        out = {"metric": METRIC, "value": round(value, 3), "unit": "M edges/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
               "scaling": "strong" if sharded else "weak", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic (config-5 snapshots: Zipf(1.1) subjects/objects, uniform relations, 60% "
                       "recurring triples; random-init weights)",
               "config": {"workload": cfg["label"] + " (BASELINE.json configs[4]) on 1 GPU per rank: "
                          "HyperbolicRecurrentRGCN.predict, encoder hyperbolic_uvrgcn x2 layers, RotH + RotHRel "
                          "decoders on a %d-query chunk" % B,
                          "V": V, "R": R, "R2": 2 * R, "triples_per_snapshot": cfg["per_snap"],
                          "edges_per_snapshot": 2 * cfg["per_snap"], "history_len": T, "n_layers": 2, "d": d,
                          "edges_per_step": int(np.mean(epw)), "queries_per_step": B, "windows": n_win,
                          "encoder_launches": "timestep phases" if model.use_phases else "per-layer",
                          "hip_graph": False,
                          "parallelism": ("%s-partitioned snapshots x%d" % (args.shard, world)) if sharded
                          else "replicas x%d" % world,
                          "snapshot_stats": {k: round(v) for k, v in stats.items()}},
               "exchange_gb_per_step_rank0": round(xbytes / 1e9, 3) if sharded else None,
               "roofline": roof, "kernels": kernels,
               "breakdown": {"encoder_ms_per_step": round(enc_ms, 3),
                             "encoder_M_edges_per_s": round(np.mean(epw) / enc_ms / 1e3, 1),
                             "decoder_ms_per_step": round(sum(calls[k]["ms"] * calls[k]["per_step"] for k in calls
                                                              if k in ("regcn_hyp_score_jobs_f32",
                                                                       "regcn_roth_queries_f32")), 3),
                             "encoder_M_edges_per_s_note": "with Zipf(1.1) sources the hub rows' gathered "
                                 "rows are L2 / MALL hits (830 rows hold ~65 % of the edges): this rate is cache "
                                 "reuse on top of HBM streaming; the HBM figure is aggregation_roofline.uniform_src "
                                 "(fabric traffic with uniformly spread sources)",
                             "setup_s": round(setup_s, 1),
                             "snapshot_prep_ms": {
                                 "graph_build": round(float(np.mean([p[0] for p in prep])), 1),
                                 "lists": round(float(np.mean([p[1] for p in prep])), 1),
                                 "note": "per snapshot, once (cached for every predict that reads it): the device "
                                         "CSR / r2e / tile build, then the row/type and row/source orders, inline "
                                         "items in source order and the entity-block relation and hub lists"},
                             "note": "per-call device time from HIP events recorded after each library call on "
                                     "the launching stream during the timed steps"}}
    del windows, graphs, tests, model, trace
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    world, rank, device, backend = _ctx()
    from regcn_amd.synthetic import CONFIGS
    cfg = CONFIGS[args.config]
    if args.shard == "auto":
        # independent predicts (windows) are the data-parallel unit: one per rank, no data-path
        # collective, weak scaling; --shard owner|edge partitions every snapshot across the
        # ranks instead (strong scaling of one predict; --owner-leg runs it beside the replicas)
        args.shard = "replica"
    if args.encoder_launches == "auto":
        args.encoder_launches = "layers" if cfg.get("scale") else "phases"
    if cfg.get("scale"):
        log("config 5: %d steps" % args.steps)
        out = run_scale(args, cfg, world, rank, device, backend)
        if rank == 0:
            log("config 5 done: %.1f M edges/s" % out["value"])
        if world > 1 and args.shard == "replica" and args.owner_leg:
            # the owner partition beside the replicas: every rank the same windows, its rows of
            # every snapshot (strong scaling of one predict, SURVEY.md §8(e) partitioning 2)
            log("owner-partition leg")
            own_args = parse(["--shard", "owner", "--steps", str(max(4, args.steps // 2)), "--warmup", "1",
                              "--no-extras"])
            r = run_scale(own_args, cfg, world, rank, device, backend)
            if rank == 0:
                out["owner_partition"] = {k: r[k] for k in ("value", "unit", "ms_per_step", "steps", "scaling")}
                out["owner_partition"]["parallelism"] = r["config"]["parallelism"]
                out["owner_partition"]["exchange_gb_per_step_rank0"] = r.get("exchange_gb_per_step_rank0")
        if rank == 0 and world == 1 and args.sim_ranks > 1 and not args.no_extras:
            log("owner simulation, %d ranks" % args.sim_ranks)
            sim = owner_simulation(args, cfg, device, args.sim_ranks)
            # against this run's measured one-GPU step (the simulation's own sum of the ranks'
            # launches is larger: many short launches)
            sim["predicted_speedup_vs_headline"] = round(out["ms_per_step"] / sim["predicted_step_ms"], 2)
            out["owner_simulation"] = sim
        if rank == 0 and world == 1:
            if not args.no_cpu_baseline:
                log("cpu baseline")
                out["cpu_baseline"] = cpu_baseline_scale(cfg, args.d, args.cpu_budget)
            if not args.no_scale:
                log("aggregation and decoder rooflines")
                out["aggregation_roofline"] = aggregation_at_scale(device)
                out["decoder_roofline"] = decoder_at_scale()
        if world == 1 and not args.no_extras:
            # the dataset configs (BASELINE.json configs[1..3]) as legs of the N = 1 line; GDELT
            # (configs[3], history 7) for both encoders, each with its CPU baseline
            for key, name, enc in (("icews14s", "icews14s_lgcn_roth", None),
                                   ("icews14s_regcn", "icews14s_uvrgcn_convtranse", None),
                                   ("icews18", "icews18_roth", None),
                                   ("gdelt", "gdelt", None), ("gdelt_lgcn", "gdelt", "lgcn")):
                sub = parse(["--config", name, "--steps", "64", "--warmup", "4", "--cpu-budget", "10"])
                c = dict(CONFIGS[name])
                if enc:
                    c.update(encoder=enc, label=c["label"] + ", encoder=" + enc)
                log("leg %s" % key)
                if key == "icews14s_regcn":
                    r = run_regcn(sub, c, world, rank, device, backend)
                    if rank == 0:
                        out[key] = r
                    continue
                r = run_small(sub, c, world, rank, device, backend)
                if rank == 0:
                    out[key] = {k: r[k] for k in ("value", "unit", "ms_per_step", "latency_ms_per_predict",
                                                  "steps", "config", "roofline", "kernels", "breakdown")}
                    if r.get("cpu_baseline"):
                        out[key]["cpu_baseline"] = r["cpu_baseline"]
                    if r.get("mrr_parity"):
                        mp = dict(r["mrr_parity"], workload=c["label"])
                        if key == "icews14s":
                            out["mrr_parity"] = mp
                        else:
                            out[key]["mrr_parity"] = mp
    elif cfg["decoder"] == "convtranse":
        out = run_regcn(args, cfg, world, rank, device, backend)
    else:
        out = run_small(args, cfg, world, rank, device, backend)
        if world > 1 and args.shard == "replica" and not args.no_extras:
            # the north star's literal scheme beside the replicas: every snapshot's edges split
            # across the ranks, one all_reduce of the destination partials per layer (SURVEY.md
            # §8(e) partitioning 1; latency-bound at dataset sizes, reported as measured)
            sub = parse(["--config", args.config, "--shard", "edge", "--steps", str(max(8, args.steps // 4)),
                         "--warmup", "2", "--no-cpu-baseline", "--pool", "4"])
            r = run_small(sub, cfg, world, rank, device, backend, extras=False)
            if rank == 0:
                out["edge_partition"] = {k: r[k] for k in ("value", "unit", "ms_per_step", "steps", "scaling")}
                out["edge_partition"]["parallelism"] = r["config"]["parallelism"]
        if rank == 0 and world == 1 and not args.no_scale:
            out["aggregation_roofline"] = aggregation_at_scale(device)
            out["decoder_roofline"] = decoder_at_scale()
    if rank == 0:
        print(compact_line(out, write_detail(out)), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
