"""Config-5 probe (|V| = 1M, |E| = 50M per snapshot, R = 256, d = 200,
history 3): one HyperbolicRecurrentRGCN.predict on 512 test triples (1,024 queries), phase
launches vs per-layer launches, wall time per predict and peak memory.

  python tools/c5probe.py [--V 1000000] [--triples 25000000] [--reps 5] [--modes phases,layers]
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
sys.path.insert(0, REPO)
from bench import build_model  # noqa: E402
from regcn_amd import graph as G  # noqa: E402
from regcn_amd.synthetic import CONFIGS, snapshot_series  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--V", type=int, default=1_000_000)
    ap.add_argument("--triples", type=int, default=25_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="phases,layers")
    ap.add_argument("--encoder", default="hyperbolic_uvrgcn")
    ap.add_argument("--budgets", default="0", help="fused-layer edge budgets to compare (0: the default)")
    ap.add_argument("--rt-stamps", action="store_true",
                    help="step-tail phase cycles (a library built with -DREGCN_RT_STAMPS=1 as REGCN_HIP_LIB)")
    ap.add_argument("--streams", type=int, default=1,
                    help="independent predicts in flight on this many streams (two windows alternate)")
    a = ap.parse_args()
    cfg = dict(CONFIGS["synthetic_1m"], V=a.V, per_snap=a.triples, encoder=a.encoder)
    dev = torch.device("cuda", 0)
    t0 = time.time()
    snaps = snapshot_series(100, cfg["V"], cfg["R"], cfg["T"] + (2 if a.streams > 1 else 1), cfg["per_snap"])
    print("generated %d snapshots in %.1f s" % (len(snaps), time.time() - t0), flush=True)
    for budget in [int(b) for b in a.budgets.split(",")]:
        run(a, cfg, snaps, dev, budget)


def run(a, cfg, snaps, dev, budget):
    t0 = time.time()
    glist = [G.build_sub_graph(cfg["V"], cfg["R"], s, True, dev, tile_budget=budget or None) for s in snaps[:cfg["T"]]]
    if a.streams > 1:
        return run_streams(a, cfg, snaps, dev, glist)
    torch.cuda.synchronize()
    print("built in %.2f s (budget %s)" % (time.time() - t0, budget or "default"), flush=True)
    for g in glist:
        print("  E=%d n_pos=%d tiles=%d heavy=%d budget=%d chunk=%d rel_max_span=%d items=%d heavy_chunks=%d"
              % (g.number_of_edges(), g.n_pos, g.n_pos_tiles, g.n_heavy, g.budget, g.chunk_edges,
                 g.rel_max_span, g.work()["item_src"].numel(), g.work()["heavy_chunks"].shape[0]), flush=True)
    model = build_model(cfg, 200, dev, seed=1234)
    model.param_caches = False
    model.memo_pristine = False
    test = torch.from_numpy(snaps[cfg["T"]][:512]).to(dev)
    edges = 2 * sum(g.number_of_edges() for g in glist)
    outs = {}
    if a.rt_stamps:
        rt_stamps(model, glist, cfg, test, dev)
        return
    for mode in a.modes.split(","):
        model.use_phases = mode == "phases"
        with torch.no_grad():
            for _ in range(2):
                r = model.predict(glist, cfg["R"], None, test, True)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.time()
            s.record()
            for _ in range(a.reps):
                r = model.predict(glist, cfg["R"], None, test, True)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.reps
        outs[mode] = [t.clone() for t in r]
        print("%-7s %9.3f ms per predict (wall %.3f)  %.1f M edges/s   peak mem %.1f GB"
              % (mode, ms, (time.time() - t0) / a.reps * 1e3, edges / ms / 1e3,
                 torch.cuda.max_memory_allocated() / 1e9), flush=True)
    del glist
    torch.cuda.empty_cache()
    if len(outs) == 2:
        p, l = outs["phases"], outs["layers"]
        for name, x, y in (("score", p[1], l[1]), ("score_rel", p[2], l[2])):
            print("%s equal=%s max|d|=%.3g finite=%s" % (name, bool(torch.equal(x, y)), float((x - y).abs().max()),
                                                        bool(torch.isfinite(x).all())), flush=True)


def rt_stamps(model, glist, cfg, test, dev):
    """Wave 0's s_memtime cycles per phase of the last step-tail launch (k_rowtail3, the
    diagnostic build's trace[16 b + 8 ..]): products, row maps, blend-stage waits, blend, the
    maps after it, the radius stores, the x stores;
    mean over its workgroups and fractions."""
    from regcn_amd import _lib
    model.use_phases = False
    with torch.no_grad():
        for _ in range(2):
            model.predict(glist, cfg["R"], None, test, True)
        torch.cuda.synchronize()
        buf = torch.zeros(1 << 20, 16, dtype=torch.int64, device=dev)
        _lib.call("regcn_set_trace", _lib.addr(buf, torch.int64))
        model.predict(glist, cfg["R"], None, test, True)
        torch.cuda.synchronize()
        _lib.call("regcn_set_trace", None)
    ph = buf[:, 8:15].double().cpu()
    used = ph.sum(1) > 0
    mean = ph[used].mean(0)
    names = ["products", "row_maps", "stage_waits", "blend", "maps_after", "radius_stores", "x_stores"]
    print(json.dumps({"workgroups": int(used.sum()), "cycles_mean": {n: round(float(v)) for n, v in zip(names, mean)},
                      "frac": {n: round(float(v / mean.sum()), 4) for n, v in zip(names, mean)}}), flush=True)


def run_streams(a, cfg, snaps, dev, glist):
    """Independent predicts on a.streams streams (windows: the first T snapshots and the next
    T, alternating): the memory-bound aggregations of one overlap the MFMA-bound decoder and
    the fused layers of another."""
    T, R = cfg["T"], cfg["R"]
    g2 = [G.build_sub_graph(cfg["V"], R, s, True, dev) for s in snaps[1:T + 1]]
    wins = [glist, g2]
    tests = [torch.from_numpy(snaps[T][:512]).to(dev), torch.from_numpy(snaps[T + 1][:512]).to(dev)]
    model = build_model(cfg, 200, dev, seed=1234)
    model.param_caches = False
    model.memo_pristine = False
    model.use_phases = False
    streams = [torch.cuda.Stream(dev) for _ in range(a.streams)]
    edges = 2 * sum(g.number_of_edges() for g in glist)
    main = torch.cuda.current_stream(dev)

    def run(n):
        for k in range(n):
            st = streams[k % len(streams)]
            st.wait_stream(main) if k < len(streams) else None
            with torch.cuda.stream(st):
                model.predict(wins[k % 2], R, None, tests[k % 2], True)
        for st in streams:
            main.wait_stream(st)

    with torch.no_grad():
        run(2 * len(streams))
        torch.cuda.synchronize()
        for reps in (4 * len(streams),):
            t0 = time.time()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            run(reps)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / reps
            print("streams %d: %9.3f ms per predict (wall %.3f)  %.1f M edges/s   peak mem %.1f GB"
                  % (len(streams), ms, (time.time() - t0) / reps * 1e3, edges / ms / 1e3,
                     torch.cuda.max_memory_allocated() / 1e9), flush=True)


if __name__ == "__main__":
    main()
