"""Per-workgroup stage timing of the fused layer kernel (csrc/layer.hip k_layer) on a
config-5 snapshot (|V| = 1M, |E| = 50M, d = 200): each workgroup stamps its stages
(s_memrealtime, 100 MHz, layer_parts.h trace_mark); printed per tile kind (in-edge tiles,
rows without in-edges): median stage durations, the launch span and the mean number of
workgroups resident (sum of workgroup durations / span).  Profiling only.

  python tools/layertrace.py [--triples 25000000] [--step]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
sys.path.insert(0, REPO)
from regcn_amd import graph as G  # noqa: E402
from regcn_amd import hyperbolic_layers as HL  # noqa: E402
from regcn_amd.hyperbolic_ops import HyperbolicOps as H  # noqa: E402
from regcn_amd.synthetic import snapshot_series  # noqa: E402

STAGES = [(0, 1, "rows"), (1, 8, "stage"), (8, 9, "idx"), (9, 11, "gather"), (11, 12, "flush"),
          (12, 13, "finish"), (13, 2, "operands"), (1, 2, "operands"), (2, 3, "gemm"), (3, 4, "epilogue"),
          (4, 5, "store")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--V", type=int, default=1_000_000)
    ap.add_argument("--triples", type=int, default=25_000_000)
    ap.add_argument("--uniform-src", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    V, R, d, C = a.V, 256, 200, 0.01
    snap = snapshot_series(0, V, R, 1, a.triples, uniform_s=a.uniform_src)[0]
    g = G.build_sub_graph(V, R, snap, True, dev)
    del snap
    torch.manual_seed(0)
    h = H.apply_radius(H.exp_map_zero(torch.randn(V, d, device=dev), C), torch.rand(V, 1, device=dev) * 2.5 + 0.5, C)
    rel = (torch.randn(2 * R, d, device=dev) * 0.1).contiguous()
    uni = HL.HyperbolicUnionRGCNLayer(d, d, 2 * R, c=C, activation=F.rrelu, self_loop=True,
                                      radius_msg_gamma=0.15).to(dev).eval()
    n_tiles = g.n_pos_tiles + (V - g.n_pos + 15) // 16
    with torch.no_grad():
        for _ in range(3):
            uni(g, h, rel)
        torch.cuda.synchronize()
        buf = torch.zeros(n_tiles * 16, dtype=torch.int64, device=dev)
        HL.TRACE = buf
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        uni(g, h, rel)
        e.record()
        torch.cuda.synchronize()
        HL.TRACE = None
    st = buf.view(-1, 16).cpu().double()
    t0 = st[:, 0].min()
    span = float((st[:, 5].max() - t0) / 100.0)
    print("tiles %d (in-edge %d) heavy rows %d: launch %.1f us (events, incl. heavy pre-aggregation), "
          "workgroup span %.1f us" % (n_tiles, g.n_pos_tiles, g.n_heavy, s.elapsed_time(e) * 1e3, span))
    for name, sl in (("in-edge tiles", slice(0, g.n_pos_tiles)), ("zero tiles", slice(g.n_pos_tiles, n_tiles))):
        x = st[sl]
        if len(x) == 0:
            continue
        dur = (x[:, 5] - x[:, 0]) / 100.0
        line = "%-14s x%d dur med %.2f p90 %.2f max %.2f us, resident %.0f |" % (
            name, len(x), float(dur.median()), float(dur.quantile(0.9)), float(dur.max()),
            float(dur.sum()) / span)
        for a0, a1, nm in STAGES:
            ok = (x[:, a0] > 0) & (x[:, a1] > 0)
            if not bool(ok.all()):
                continue
            seg = (x[ok, a1] - x[ok, a0]) / 100.0
            line += " %s %.2f" % (nm, float(seg.median()))
        print(line, flush=True)


if __name__ == "__main__":
    main()
