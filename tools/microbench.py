"""Kernel microbenchmarks on the GPU box: the fused per-layer kernel (Lorentz and Union,
with and without the fused timestep) and the relation GRU at four snapshot sizes, timed
as graph-replayed launches between HIP events (bench.event_time)."""
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
sys.path.insert(0, REPO)
from bench import FP32_MFMA_PEAK_TFLOPS, HBM_PEAK_GBS, event_time  # noqa: E402
from regcn_amd import graph as G  # noqa: E402
from regcn_amd.hyperbolic_layers import HyperbolicUnionRGCNLayer, LorentzRGCNLayer, StepSpec  # noqa: E402
from regcn_amd.hyperbolic_model import relation_gru_step  # noqa: E402
from regcn_amd.hyperbolic_ops import HyperbolicOps as H  # noqa: E402
from regcn_amd.synthetic import snapshot_series  # noqa: E402
from regcn_amd.weights import packed  # noqa: E402

dev = torch.device("cuda", 0)
C = 0.01


def run(V, R, per_snap, d=200, nb=100):
    snaps = snapshot_series(0, V, R, 1, per_snap)
    g = G.build_sub_graph(V, R, snaps[0], True, dev)
    E = g.number_of_edges()
    torch.manual_seed(0)
    h = H.exp_map_zero(torch.randn(V, d, device=dev) * 0.3, C)
    rel = torch.randn(2 * R, d, device=dev) * 0.1
    lor = LorentzRGCNLayer(d, d, 2 * R, nb, c=C, activation=F.rrelu, self_loop=True).to(dev).eval()
    uni = HyperbolicUnionRGCNLayer(d, d, 2 * R, c=C, activation=F.rrelu, self_loop=True,
                                   radius_msg_gamma=0.15).to(dev).eval()
    gru = torch.nn.GRUCell(2 * d, d).to(dev)
    xp = torch.randn(V, d, device=dev) * 0.1
    step = StepSpec(xp, packed(torch.randn(d, d, device=dev) * 0.05), torch.zeros(d, device=dev),
                    torch.rand(V, device=dev) + 0.5, torch.randn(d, device=dev) * 0.01, torch.zeros(1, device=dev),
                    0.1, 1.0, False, True, C)
    x = H.log_map_zero(h, C)
    st = torch.cuda.Stream(dev)
    with torch.no_grad():
        t_lor = event_time(lambda: lor(g, h, rel), 20, st)
        t_lors = event_time(lambda: lor(g, h, rel, step=step), 20, st)
        t_uni = event_time(lambda: uni(g, h, rel), 20, st)
        t_gru = event_time(lambda: relation_gru_step(gru, rel, x, g, rel), 20, st)
    gather = E * (4 * d + 8) + 8 * V
    io = 4.0 * V * d * 3 + 4 * V
    fl = 2.0 * d * d * V
    print("V=%d E=%d pos=%d tiles=%d heavy=%d | lorentz layer %.1f us (%.1f TF, %.0f GB/s) | +step %.1f us "
          "(%.1f TF) | union layer %.1f us (%.1f TF) | rel GRU %.1f us"
          % (V, E, g.n_pos, g.n_pos_tiles, g.n_heavy, t_lor * 1e3, fl / t_lor / 1e9, (gather + io) / t_lor / 1e6,
             t_lors * 1e3, 2 * fl / t_lors / 1e9, t_uni * 1e3, (fl + 2.0 * d * d * g.n_pos) / t_uni / 1e9,
             t_gru * 1e3), flush=True)


def trace(V=7128, R=230, per_snap=246, d=200, nb=100):
    """Per-workgroup phase stamps (s_memrealtime, 10 ns) of the fused Lorentz layer + step
    kernel (layer.hip trace_mark): where the critical path of a small snapshot goes."""
    from regcn_amd import hyperbolic_layers as HL
    snaps = snapshot_series(0, V, R, 1, per_snap)
    g = G.build_sub_graph(V, R, snaps[0], True, dev)
    torch.manual_seed(0)
    h = H.exp_map_zero(torch.randn(V, d, device=dev) * 0.3, C)
    rel = torch.randn(2 * R, d, device=dev) * 0.1
    lor = LorentzRGCNLayer(d, d, 2 * R, nb, c=C, activation=F.rrelu, self_loop=True).to(dev).eval()
    xp = torch.randn(V, d, device=dev) * 0.1
    step = StepSpec(xp, packed(torch.randn(d, d, device=dev) * 0.05), torch.zeros(d, device=dev),
                    torch.rand(V, device=dev) + 0.5, torch.randn(d, device=dev) * 0.01, torch.zeros(1, device=dev),
                    0.1, 1.0, False, True, C)
    n_wg = g.n_pos_tiles + (V - g.n_pos + 15) // 16
    for name, kw in (("layer", {}), ("layer+step", {"step": step})):
        with torch.no_grad():
            for _ in range(3):
                lor(g, h, rel, **kw)
            HL.TRACE = torch.zeros(n_wg * 16, dtype=torch.int64, device=dev)
            lor(g, h, rel, **kw)
            torch.cuda.synchronize()
            t = HL.TRACE.view(n_wg, 16).cpu().double()
            HL.TRACE = None
        t0 = t[:, 0].min()
        us = lambda a, b, sel: ((t[sel, b] - t[sel, a]) / 100.0)  # 100 MHz -> us
        pos = torch.arange(n_wg) < g.n_pos_tiles
        print("%s V=%d pos tiles=%d zero tiles=%d total %.1f us (first start -> last end)"
              % (name, V, int(pos.sum()), int((~pos).sum()), float((t[:, 5].max() - t0) / 100.0)))
        for label, sel in (("pos", pos), ("zero", ~pos)):
            if not sel.any():
                continue
            start = (t[sel, 0] - t0) / 100.0
            ph = [("start", start), ("rows", us(0, 1, sel)), ("operands", us(1, 2, sel)), ("gemm", us(2, 3, sel)),
                  ("act", us(3, 4, sel)), ("epilogue", us(4, 5, sel))]
            if label == "pos":
                ph += [("g.idx", us(8, 9, sel)), ("g.loop", us(9, 11, sel)), ("g.sync", us(11, 12, sel)),
                       ("g.finish", us(12, 13, sel))]
            if name == "layer+step":
                ph += [("s.gemm", us(4, 14, sel)), ("s.gate", us(14, 15, sel)), ("s.radius", us(15, 5, sel))]
            print("  %-4s " % label + " ".join("%s %.2f/%.2f" % (k, float(v.median()), float(v.max())) for k, v in ph))
        clk = (t[:, 7] - t[:, 6]) / ((t[:, 5] - t[:, 0]).clamp(min=1) / 100.0)
        print("  shader clock ~%.0f MHz (median over workgroups)" % float(clk.median()))


def trace_pos(V=7128, R=230, per_snap=246, d=200, nb=100):
    """The in-edge tiles alone (run_layer pos_only): per-phase stamps and launch times of the
    layer and layer+step kernels over rows[:n_pos], and of the in-degree-0 chain kernel."""
    from regcn_amd import hyperbolic_layers as HL
    snaps = snapshot_series(0, V, R, 1, per_snap)
    g = G.build_sub_graph(V, R, snaps[0], True, dev)
    torch.manual_seed(0)
    h = H.exp_map_zero(torch.randn(V, d, device=dev) * 0.3, C)
    rel = torch.randn(2 * R, d, device=dev) * 0.1
    lor = LorentzRGCNLayer(d, d, 2 * R, nb, c=C, activation=F.rrelu, self_loop=True).to(dev).eval()
    lor2 = LorentzRGCNLayer(d, d, 2 * R, nb, c=C, activation=F.rrelu, self_loop=True).to(dev).eval()
    xp = torch.randn(V, d, device=dev) * 0.1
    step = StepSpec(xp, packed(torch.randn(d, d, device=dev) * 0.05), torch.zeros(d, device=dev),
                    torch.rand(V, device=dev) + 0.5, torch.randn(d, device=dev) * 0.01, torch.zeros(1, device=dev),
                    0.1, 1.0, False, True, C)
    out = (torch.empty(V, d, device=dev), torch.empty(V, d, device=dev), torch.empty(V, device=dev))
    st = torch.cuda.Stream(dev)
    n_wg = g.n_pos_tiles
    with torch.no_grad():
        for name, fn in (("pos layer", lambda: lor(g, h, rel, pos_only=True)),
                         ("pos layer+step", lambda: lor(g, h, rel, step=step, pos_only=True, out=out))):
            ms = event_time(fn, 20, st)
            for _ in range(2):
                fn()
            HL.TRACE = torch.zeros(max(n_wg, 1) * 16, dtype=torch.int64, device=dev)
            fn()
            torch.cuda.synchronize()
            t = HL.TRACE.view(-1, 16).cpu().double()
            HL.TRACE = None
            t0 = t[:, 0].min()
            us = lambda a, b: ((t[:, b] - t[:, a]) / 100.0)  # noqa: E731
            ph = [("start", (t[:, 0] - t0) / 100.0), ("rows", us(0, 1)), ("operands", us(1, 2)), ("gemm", us(2, 3)),
                  ("act", us(3, 4)), ("epilogue", us(4, 5)), ("g.idx", us(8, 9)), ("g.loop", us(9, 11)),
                  ("g.sync", us(11, 12)), ("g.finish", us(12, 13))]
            print("%s: %d tiles, launch %.1f us, span %.1f us | " % (name, n_wg, ms * 1e3,
                                                                    float((t[:, 5].max() - t0) / 100.0))
                  + " ".join("%s %.2f/%.2f" % (k, float(v.median()), float(v.max())) for k, v in ph), flush=True)


def trace_gru(V=7128, R=230, per_snap=246, d=200):
    """Phase stamps of the relation GRU kernel (regcn_set_trace): staging (relation means),
    MFMA k-split, cross-wave reduction, gate epilogue."""
    from regcn_amd import _lib
    snaps = snapshot_series(0, V, R, 1, per_snap)
    g = G.build_sub_graph(V, R, snaps[0], True, dev)
    torch.manual_seed(0)
    rel = torch.randn(2 * R, d, device=dev) * 0.1
    x = torch.randn(V, d, device=dev) * 0.1
    gru = torch.nn.GRUCell(2 * d, d).to(dev)
    n_wg = ((2 * R + 15) // 16) * ((d + 15) // 16)
    with torch.no_grad():
        for _ in range(3):
            relation_gru_step(gru, rel, x, g, rel)
        buf = torch.zeros(n_wg * 16, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        _lib.call("regcn_set_trace", _lib.addr(buf, torch.int64))
        relation_gru_step(gru, rel, x, g, rel)
        torch.cuda.synchronize()
        _lib.call("regcn_set_trace", None)
    t = buf.view(n_wg, 16).cpu().double()
    t0 = t[:, 0].min()
    us = lambda a, b: (t[:, b] - t[:, a]) / 100.0
    print("rel GRU R2=%d workgroups=%d total %.1f us" % (2 * R, n_wg, float((t[:, 4].max() - t0) / 100.0)))
    ph = [("start", (t[:, 0] - t0) / 100.0), ("stage", us(0, 1)), ("mfma", us(1, 2)), ("sync", us(2, 3)),
          ("gates", us(3, 4))]
    print("  " + " ".join("%s %.2f/%.2f" % (k, float(v.median()), float(v.max())) for k, v in ph))


def trace_score(B=492, N=7128, d=200):
    """Phase stamps of the all-entity scorer (k_score_f32): operand staging, then the MFMA
    loop (Q E^T) with the score epilogue."""
    from regcn_amd import _lib
    from regcn_amd.hyperbolic_decoder import _chunked_hyperbolic_dist_score as sc
    torch.manual_seed(0)
    q = H.exp_map_zero(torch.randn(B, d, device=dev) * 0.3, C)
    e = H.exp_map_zero(torch.randn(N, d, device=dev) * 0.3, C)
    bias = torch.randn(N, device=dev) * 0.1
    n_wg = ((B + 127) // 128) * ((N + 63) // 64)  # k_score_f32: 128 queries x 64 candidates
    with torch.no_grad():
        for _ in range(3):
            sc(q, e, bias, C, 128, 256)
        buf = torch.zeros(n_wg * 16, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        _lib.call("regcn_set_trace", _lib.addr(buf, torch.int64))
        sc(q, e, bias, C, 128, 256)
        torch.cuda.synchronize()
        _lib.call("regcn_set_trace", None)
    t = buf.view(n_wg, 16).cpu().double()
    t0 = t[:, 0].min()
    us = lambda a, b: (t[:, b] - t[:, a]) / 100.0
    print("score B=%d N=%d workgroups=%d total %.1f us" % (B, N, n_wg, float((t[:, 2].max() - t0) / 100.0)))
    start = (t[:, 0] - t0) / 100.0
    ph = [("start", start), ("stage", us(0, 1)), ("mfma+epilogue", us(1, 2))]
    print("  " + " ".join("%s %.2f/%.2f" % (k, float(v.median()), float(v.max())) for k, v in ph))
    print("  start quartiles %s" % [round(float(x), 2) for x in torch.quantile(start, torch.tensor([0.25, 0.5, 0.75, 1.0], dtype=torch.float64))])


if __name__ == "__main__":
    if "--pos" in sys.argv:
        trace_pos()
        sys.exit(0)
    if "--trace" in sys.argv:
        trace()
        trace_gru()
        trace_score()
        sys.exit(0)
    print("peaks: %.1f TF fp32 MFMA, %.0f GB/s HBM" % (FP32_MFMA_PEAK_TFLOPS, HBM_PEAK_GBS))
    for V, R, ps in [(7128, 230, 246), (23033, 256, 1540), (100000, 256, 250000), (1000000, 256, 2500000)]:
        run(V, R, ps)
