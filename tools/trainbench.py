"""Training-step benchmark on the BASELINE.json configs[1] shape.

One training sample = hyperbolic_main.py:547-628 for one target snapshot: its ~246 triples in
`--triple-batch-size` (64) mini-batches, each a get_loss (recurrent encoder over the
history_len=3 window + RotH entity/relation cross entropy + radius loss) and a backward,
then gradient clipping and one Adam step.  Snapshot graphs are built once (device build) and
reused, as the CLI does.  Reports ms per sample, samples/s and forward message edges/s
(edges x layers x snapshots x mini-batches, the encoder is recomputed per mini-batch as in
the reference), next to the CPU oracle's get_loss + backward on the same sample.

  python tools/trainbench.py [--steps 20] [--encoder lgcn] [--cpu-budget 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--encoder", default="lgcn", choices=["lgcn", "hyperbolic_uvrgcn"])
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="capture each sample's whole step (forward, backward, clip, Adam) in a HIP graph once "
                         "and replay it (Adam capturable; the step has no host synchronisation)")
    ap.add_argument("--per-batch-encoder", action="store_true",
                    help="recompute the encoder per mini-batch (the reference loop) instead of once per sample")
    a = ap.parse_args()
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    from regcn_amd.synthetic import CONFIGS, snapshot_series
    from regcn_amd.weights import bump_versions
    cfg = CONFIGS["icews14s_lgcn_roth"]
    V, R, T, per = cfg["V"], cfg["R"], cfg["T"], cfg["per_snap"]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    rng = np.random.default_rng(0)
    rt = rng.uniform(0.5, 3.0, V).astype(np.float32)
    m = HyperbolicRecurrentRGCN("roth", a.encoder, V, R, 0, 0, a.d, "sub", T, num_bases=100, num_hidden_layers=2,
                                dropout=0.2, c=0.01, self_loop=True, layer_norm=False, input_dropout=0.2,
                                hidden_dropout=0.2, feat_dropout=0.2, entity_prediction=True, relation_prediction=True,
                                use_cuda=True, gpu=0, radius_target=rt, radius_msg_gamma=0.15).to(dev).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5, capturable=a.graph, fused=True)
    snaps = snapshot_series(1, V, R, T + 8, per)
    graphs = [G.build_sub_graph(V, R, s, True, dev) for s in snaps]
    samples = [(graphs[i:i + T], torch.from_numpy(snaps[i + T]).to(dev)) for i in range(8)]
    edges_fwd = [sum(g.number_of_edges() for g in gl) * 2 for gl, _ in samples]  # x 2 layers

    def step(k):
        glist, tr = samples[k % len(samples)]
        opt.zero_grad()
        nb = 0
        if a.per_batch_encoder:  # hyperbolic_main.py:585-598 as written
            for b in range(0, tr.shape[0], a.batch):
                le, lr, ls, lrad = m.get_loss(glist, tr[b:b + a.batch], None, True)
                (0.7 * le + 0.3 * lr + ls.sum() + lrad).backward()
                nb += 1
        else:  # the CLI default: one encoder pass per sample, same gradients
            m.get_loss_batches(glist, tr, None, True, a.batch,
                               combine=lambda le, lr, ls, lrad: 0.7 * le + 0.3 * lr + ls.sum() + lrad)
            nb = 1
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
        bump_versions(m.parameters())  # as the CLI: the fused step leaves the version counters
        return nb

    cap = torch.cuda.Stream(dev) if a.graph else torch.cuda.current_stream(dev)
    cap.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cap):  # with --graph every step runs on the capture stream
        for k in range(max(a.warmup, len(samples) if a.graph else 0)):
            step(k)
    torch.cuda.synchronize()
    graphs = []
    if a.graph:  # one graph per sample (its snapshot shapes), captured after an eager warmup
        with torch.cuda.stream(cap):
            for k in range(len(samples)):
                opt.zero_grad(set_to_none=True)
                gph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gph, stream=cap):
                    step(k)
                graphs.append(gph)
        torch.cuda.synchronize()
        for gph in graphs:
            gph.replay()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    edges = 0
    for k in range(a.steps):
        if graphs:
            graphs[k % len(samples)].replay()
            nb = 1 if not a.per_batch_encoder else (samples[k % len(samples)][1].shape[0] + a.batch - 1) // a.batch
        else:
            nb = step(k)
        edges += edges_fwd[k % len(samples)] * nb
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"workload": "ICEWS14s-shaped training sample, encoder=%s, decoder=roth, d=%d, history 3, "
                       "mini-batch %d (reference defaults, dropout 0.2), encoder %s%s" % (
                           a.encoder, a.d, a.batch, "per mini-batch" if a.per_batch_encoder else "once per sample",
                           ", HIP graph per sample" if a.graph else ""),
           "ms_per_sample": round(dt / a.steps * 1e3, 3), "samples_per_s": round(a.steps / dt, 2),
           "fwd_M_edges_per_s": round(edges / dt / 1e6, 3), "triples_per_sample": per}
    if not a.no_cpu:
        from oracle import graph as OG
        from oracle import model as OM
        # the box's CPU share (OMP_NUM_THREADS=16 there; nproc shows the whole machine)
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", min(16, os.cpu_count() or 1))))
        print("gpu leg done: %s; cpu oracle leg (%.0f s budget)" % (json.dumps(out), a.cpu_budget),
              file=sys.stderr, flush=True)
        sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        names = [k for k, _ in m.named_parameters()]
        for k in names:
            sd[k].requires_grad_(True)
        ocfg = dict(c=0.01, n_layers=2, n_bases=100, radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
                    radius_anchor_beta=1.0, radius_msg_gamma=0.15, use_residual_evolution=True, encoder=a.encoder,
                    decoder="roth", layer_norm=False)
        og = [OG.build_sub_graph(V, R, s) for s in snaps[:T]]
        tr = torch.from_numpy(snaps[T])
        n_mb, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < a.cpu_budget or n_mb == 0:
            b = (n_mb * a.batch) % len(tr)
            le, lr, ls, lrad = OM.hyperbolic_get_loss(sd, ocfg, og, tr[b:b + a.batch], rt)
            (0.7 * le + 0.3 * lr + ls.sum() + lrad).backward()
            n_mb += 1
        cdt = (time.perf_counter() - t0) / n_mb
        mb_per_sample = (per + a.batch - 1) // a.batch
        out["cpu_baseline"] = {"ms_per_sample": round(cdt * mb_per_sample * 1e3, 1),
                               "samples_per_s": round(1.0 / (cdt * mb_per_sample), 4),
                               "cores": torch.get_num_threads(), "kind": "port",
                               "sample": "%d oracle get_loss+backward mini-batches (%.2f s each)" % (n_mb, cdt)}
        out["speedup_vs_cpu"] = round(out["samples_per_s"] / out["cpu_baseline"]["samples_per_s"], 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
