"""Per-workgroup timing of the timestep phase launches (csrc/timestep.hip) on the bench
workload: each workgroup stamps its start and end (s_memrealtime, 100 MHz); per launch and
block kind (in-edge tiles, rows without in-edges, relation GRU blocks) the start offsets,
durations and the last end are printed.  Profiling only (regcn_set_trace)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from regcn_amd import hyperbolic_model as HM  # noqa: E402
from regcn_amd.synthetic import CONFIGS  # noqa: E402


def main(config="icews14s_lgcn_roth", empty="", memo="1"):
    dev = torch.device("cuda", 0)
    cfg = CONFIGS[config]
    model = bench.build_model(cfg, 200, dev, seed=1234)
    model.memo_pristine = memo != "0"  # "0": every row runs at every timestep
    sample = bench.make_samples(cfg, 1, dev, seed=100)[0]
    _, glist, _, _ = sample
    if empty:  # edgeless snapshots: every row on the in-degree-0 path (throughput of that path alone)
        import numpy as np
        from regcn_amd import graph as G
        glist = [G.build_sub_graph(cfg["V"], cfg["R"], np.zeros((0, 3), np.int64), True, dev) for _ in glist]
    with torch.no_grad():
        for _ in range(3):
            model.forward(glist, None, True)
        torch.cuda.synchronize()
        HM.PHASE_TRACE = []
        model.forward(glist, None, True)
        torch.cuda.synchronize()
        rec, HM.PHASE_TRACE = HM.PHASE_TRACE, None
    K = HM.TRACE_SLOTS
    seen = {}
    for phase, kinds, buf in rec:
        t = seen[phase] = seen.get(phase, -1) + 1  # timestep of this launch
        st = buf.view(-1, K).cpu().double()
        t0 = st[st[:, 0] > 0, 0].min()
        line = "%s%d span %6.2f us |" % (phase, t, float((st[:, K - 1].max() - t0) / 100.0))
        off = 0
        for name, n in kinds:
            if n == 0:
                continue
            s = st[off:off + n]
            off += n
            s = s[s[:, K - 1] > 0]  # workgroups past a device-counted list exit unstamped
            if len(s) == 0:
                continue
            n = len(s)
            start = (s[:, 0] - t0) / 100.0
            dur = (s[:, K - 1] - s[:, 0]) / 100.0
            end = (s[:, K - 1] - t0) / 100.0
            line += " %s x%d start %.2f/%.2f dur %.2f/%.2f end %.2f" % (
                name, n, float(start.median()), float(start.max()), float(dur.median()), float(dur.max()),
                float(end.max()))
            # segments between consecutive stamps present in every workgroup of the kind
            cols = [0] + [k for k in range(1, K - 1) if bool((s[:, k] > 0).all())] + [K - 1]
            if len(cols) > 2:
                seg = [(s[:, b] - s[:, a]) / 100.0 for a, b in zip(cols[:-1], cols[1:])]
                line += " [%s]" % " ".join("%d:%.2f" % (b, float(x.median())) for b, x in zip(cols[1:], seg))
            line += " |"
        print(line, flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
