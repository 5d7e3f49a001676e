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


if __name__ == "__main__":
    print("peaks: %.1f TF fp32 MFMA, %.0f GB/s HBM" % (FP32_MFMA_PEAK_TFLOPS, HBM_PEAK_GBS))
    for V, R, ps in [(7128, 230, 246), (23033, 256, 1540), (100000, 256, 250000), (1000000, 256, 2500000)]:
        run(V, R, ps)
