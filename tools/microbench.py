"""Kernel microbenchmarks on the GPU box (graph-replayed launches timed with HIP events)."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
from regcn_amd import _lib, graph as G  # noqa: E402
from regcn_amd.synthetic import snapshot_series  # noqa: E402

dev = torch.device("cuda", 0)


def timeit(fn, reps=50):
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st)
        for _ in range(5):
            g.replay()
        e.record(st)
        e.synchronize()
    return s.elapsed_time(e) / (5 * reps) * 1e3  # us per launch


def run(V, R, per_snap, d=200, nb=100, chunk=None):
    snaps = snapshot_series(0, V, R, 1, per_snap)
    g = G.build_sub_graph(V, R, snaps[0], True, dev, chunk_edges=chunk)
    wk = g.work()
    E = g.number_of_edges()
    x = torch.randn(V, d, device=dev) * 0.1
    r = x.norm(dim=1).contiguous()
    rel = torch.randn(2 * R, d, device=dev) * 0.1
    W = torch.randn(2 * R, nb * (d // nb) ** 2, device=dev) * 0.1
    out = torch.empty_like(x)
    ch, fx = wk["chunks"], wk["fixups"]
    part = torch.empty(max(g.n_slots, 1), d + 4, device=dev)
    f, i = _lib.fptr, _lib.iptr

    def lor():
        _lib.call("regcn_lorentz_aggregate_f32", f(x), f(rel), f(W), i(wk["col_src"]), i(wk["col_type"]), i(ch),
                  ch.shape[0], i(fx), fx.shape[0], nb, 0.01, d, f(part), d + 4, f(out), _lib.stream())

    def uni():
        _lib.call("regcn_union_aggregate_f32", f(x), f(r), f(rel), i(wk["col_src"]), i(wk["col_type"]),
                  f(wk["norm"]), i(ch), ch.shape[0], i(fx), fx.shape[0], 0.15, d, f(part), d + 4, f(out),
                  _lib.stream())

    def pro():
        _lib.call("regcn_prologue_f32", f(x), V, d, 0.01, f(out), f(r), _lib.stream())
    from regcn_amd.hyperbolic_layers import layer_tail
    from regcn_amd.weights import packed
    Wl = torch.randn(d, d, device=dev) * 0.05
    We = torch.randn(d, d, device=dev) * 0.05
    Wn = torch.randn(d, d, device=dev) * 0.05

    def tail():
        layer_tail(out, Wn, x, Wl, We, None, None, None, None, g, 0.01, False)
    Wg = packed(torch.randn(d, d, device=dev) * 0.05)
    bg = torch.zeros(d, device=dev)
    rs = torch.rand(V, device=dev) + 0.5
    wr = torch.randn(d, device=dev) * 0.01
    br = torch.zeros(1, device=dev)
    hn, xn, rn = torch.empty_like(x), torch.empty_like(x), torch.empty_like(r)

    def step():
        _lib.call("regcn_timestep_f32", f(x), f(x), f(Wg), f(bg), f(rs), f(wr), f(br), 0.1, 1.0, 0, 1, V, d, 0.01,
                  0.01, f(hn), f(xn), f(rn), _lib.stream())
    tl, tu, tp, tt, ts = timeit(lor), timeit(uni), timeit(pro), timeit(tail), timeit(step)
    byts = E * (4 * d + 12) + ch.shape[0] * (4 * d + 12)
    fl_tail = 2.0 * d * d * (V + g.n_pos)
    print("V=%d E=%d chunks=%d (chunk_edges=%d) lorentz %.1f us (%.1f GB/s)  union %.1f us (%.1f GB/s)  "
          "prologue %.1f us  layer_tail %.1f us (%.1f TF)  timestep %.1f us (%.1f TF)"
          % (V, E, ch.shape[0], g.chunk_edges, tl, byts / tl / 1e3, tu, byts / tu / 1e3, tp, tt,
             fl_tail / tt / 1e6, ts, 2.0 * d * d * V / ts / 1e6), flush=True)


if __name__ == "__main__":
    for V, R, ps in [(7128, 230, 246), (23033, 256, 1540), (100000, 256, 250000), (1000000, 256, 2500000)]:
        run(V, R, ps)
