"""Launch attribution of one eager training sample: which torch ops
issue the ~3,000 device launches of a get_loss_batches + backward + clip + Adam step.

torch.profiler records the sample; every device kernel is charged to the innermost CPU op
that launched it, and ops are grouped by (op, enclosing autograd node / module op).

  python tools/trainlaunches.py [--encoder lgcn] [--top 40]
"""
import argparse
import collections
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--encoder", default="lgcn", choices=["lgcn", "hyperbolic_uvrgcn"])
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    from regcn_amd import graph as G
    from regcn_amd.hyperbolic_model import HyperbolicRecurrentRGCN
    from regcn_amd.synthetic import CONFIGS, snapshot_series
    from regcn_amd.weights import bump_versions
    cfg = CONFIGS["icews14s_lgcn_roth"]
    V, R, T, per = cfg["V"], cfg["R"], cfg["T"], cfg["per_snap"]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    rt = np.random.default_rng(0).uniform(0.5, 3.0, V).astype(np.float32)
    m = HyperbolicRecurrentRGCN("roth", a.encoder, V, R, 0, 0, 200, "sub", T, num_bases=100, num_hidden_layers=2,
                                dropout=0.2, c=0.01, self_loop=True, layer_norm=False, input_dropout=0.2,
                                hidden_dropout=0.2, feat_dropout=0.2, entity_prediction=True, relation_prediction=True,
                                use_cuda=True, gpu=0, radius_target=rt, radius_msg_gamma=0.15).to(dev).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-5, capturable=True, fused=True)
    snaps = snapshot_series(1, V, R, T + 1, per)
    glist = [G.build_sub_graph(V, R, s, True, dev) for s in snaps[:T]]
    tr = torch.from_numpy(snaps[T]).to(dev)

    def step():
        opt.zero_grad()
        m.get_loss_batches(glist, tr, None, True, 64, combine=lambda le, lr, ls, lrad: 0.7 * le + 0.3 * lr + ls.sum() + lrad)
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
        bump_versions(m.parameters())  # as the CLI: the fused step leaves the version counters

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        step()
        torch.cuda.synchronize()
    events = prof.events()
    by_kernel = collections.Counter()
    by_op = collections.Counter()
    by_ctx = collections.Counter()
    total = 0
    for ev in events:
        if ev.device_type != torch.autograd.DeviceType.CPU:
            continue
        kids = [k for k in ev.kernels] if hasattr(ev, "kernels") else []
        if not kids:
            continue
        # innermost CPU op that owns kernels: skip if a child op also owns them
        if any(getattr(c, "kernels", None) for c in ev.cpu_children):
            continue
        n = len(kids)
        total += n
        by_op[ev.name] += n
        anc, p = [], ev.cpu_parent
        while p is not None and len(anc) < 3:
            anc.append(p.name)
            p = p.cpu_parent
        top = next((x for x in anc if "Backward" in x or x.startswith("autograd::") or "AccumulateGrad" in x
                    or x.startswith("Optimizer") or "clip" in x), anc[-1] if anc else "-")
        by_ctx[(ev.name, top)] += n
        for k in kids:
            by_kernel[k.name[:90]] += 1
    print("device launches in one sample: %d" % total)
    print("\n-- by launching op")
    for k, v in by_op.most_common(a.top):
        print("%6d  %s" % (v, k))
    print("\n-- by (op, enclosing autograd node)")
    for (k, c), v in by_ctx.most_common(a.top):
        print("%6d  %-40s %s" % (v, k, c))
    print("\n-- by kernel")
    for k, v in by_kernel.most_common(25):
        print("%6d  %s" % (v, k))


if __name__ == "__main__":
    main()
