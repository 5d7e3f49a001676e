"""Debug: which captured training step state does a host-side perturbation between replays
change?  Trains 2 epochs under --hip-graph (epoch 0 eager + capture, epoch 1 replays), then
replays one sample's graph from a saved state before and after a perturbation and lists the
gradients / parameters / optimizer-state tensors that differ.

  python tools/graphdbg2.py
"""
import os
import random
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))


def main():
    from regcn_amd import cli, ranking, training
    common = ["-d", "synthetic:icews14s_lgcn_roth", "--gpu", "0", "--encoder", "lgcn", "--decoder", "roth",
              "--n-hidden", "64", "--n-bases", "32", "--synthetic-snapshots", "10", "--train-history-len", "3",
              "--test-history-len", "3", "--relation-prediction", "--entity-prediction",
              "--checkpoint", "/tmp/graphdbg2.pth", "--seed", "0", "--lr", "0.01", "--triple-batch-size", "64",
              "--dropout", "0", "--input-dropout", "0", "--hidden-dropout", "0", "--feat-dropout", "0",
              "--n-epochs", "2", "--evaluate-every", "100", "--hip-graph"]
    dev = torch.device("cuda", 0)
    adam = torch.optim.Adam
    opts, gss = [], []

    class CapturableAdam(adam):
        def __init__(self, *a, **k):
            k["capturable"] = True
            super().__init__(*a, **k)
            opts.append(self)

    class RecGS(training.GraphedSteps):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            gss.append(self)

    torch.optim.Adam = CapturableAdam
    cli.GraphedSteps = RecGS
    args = cli.build_parser().parse_args(common)
    V, R, train, valid, _ = cli.load_dataset(args)
    tl = ranking.split_by_time(train)
    vl = ranking.split_by_time(valid)
    torch.manual_seed(0)
    model = cli.build_model(args, V, R, tl, dev)
    random.seed(0)
    cli.train_model(args, model, tl, valid, V, R, dev, "/tmp/graphdbg2.pth")
    torch.cuda.synchronize()
    gs, opt = gss[-1], opts[-1]
    names = {id(p): n for n, p in model.named_parameters()}
    tensors = {}
    for p in model.parameters():
        tensors[names[id(p)]] = p
        if p.grad is not None:
            tensors[names[id(p)] + ".grad"] = p.grad
        for key, v in opt.state.get(p, {}).items():
            if torch.is_tensor(v) and v.is_cuda:
                tensors["%s.%s" % (names[id(p)], key)] = v
    saved = {k: v.detach().clone() for k, v in tensors.items()}

    def restore():
        with torch.no_grad():
            for k, v in tensors.items():
                v.copy_(saved[k])
        torch.cuda.synchronize()

    def replay(key):
        restore()
        with torch.cuda.stream(gs.stream):
            gs.graphs[key][0].replay()
        torch.cuda.synchronize()
        return {k: v.detach().clone() for k, v in tensors.items()}, gs.graphs[key][1].detach().clone()

    def diff(a, b):
        out = []
        for k in a[0]:
            if not torch.equal(a[0][k], b[0][k]):
                d = float((a[0][k].double() - b[0][k].double()).abs().max())
                out.append("%s(%.2e)" % (k, d))
        return ("losses %s vs %s; " % (a[1].tolist(), b[1].tolist()) if not torch.equal(a[1], b[1]) else "") + \
            ("%d tensors differ: %s" % (len(out), " ".join(out[:40])) if out else "all equal")

    def h2d():
        t = torch.from_numpy(np.asarray(vl[0], dtype=np.int64)).to(dev)
        del t

    def snap():
        torch.cuda.memory_snapshot()

    def device_build():
        from regcn_amd.graph import build_sub_graph
        gl = [build_sub_graph(V, R, s, True, dev) for s in tl[-3:]]
        del gl

    def junk():
        j = [torch.full((1 << 26,), 3.0, device=dev) for _ in range(16)]
        del j

    def eager_alloc_small():
        j = [torch.full((1000 + 37 * i,), 3.0, device=dev) for i in range(64)]
        del j

    keys = sorted(gs.graphs)
    print("graphs:", len(keys), "keys", keys[:5], flush=True)
    for key in keys[:2]:
        base = replay(key)
        print("key %s: replay twice        -> %s" % (key, diff(base, replay(key))), flush=True)
        for name, fn in (("h2d", h2d), ("memory_snapshot", snap), ("device_build", device_build), ("junk", junk),
                         ("small allocs", eager_alloc_small)):
            fn()
            torch.cuda.synchronize()
            print("key %s: after %-16s -> %s" % (key, name, diff(base, replay(key))), flush=True)
    torch.optim.Adam = adam


if __name__ == "__main__":
    main()
