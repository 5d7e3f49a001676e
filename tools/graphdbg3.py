"""Debug (graphdbg3): which backward of a captured training step is the first to change when
eager work runs between replays?  Every custom autograd Function's backward is wrapped to
clone its incoming and outgoing gradients into per-graph debug buffers while the graph is
captured (the clones are graph nodes, refreshed by every replay); two replays from the same
saved state, with a perturbation between them, are then compared node by node in backward
order.  Based on graphdbg2:
which captured training step state does a host-side perturbation between replays
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


def install_recorders(rec, cur_key):
    """Wrap the backward of every torch.autograd.Function subclass of regcn_amd.{autograd,training}."""
    import inspect
    from regcn_amd import autograd as AG
    from regcn_amd import training as TR
    for mod in (AG, TR):
        for name, cls in list(vars(mod).items()):
            if not (inspect.isclass(cls) and issubclass(cls, torch.autograd.Function) and "backward" in cls.__dict__):
                continue
            orig = cls.__dict__["backward"]
            fn = orig.__func__ if isinstance(orig, staticmethod) else orig

            def make(fn, name):
                def bwd(ctx, *grads):
                    out = fn(ctx, *grads)
                    if torch.cuda.is_current_stream_capturing() and cur_key:
                        outs = out if isinstance(out, tuple) else (out,)
                        lst = rec.setdefault(cur_key[0], [])
                        for i, gi in enumerate(grads):
                            if torch.is_tensor(gi):
                                lst.append(("%s#%d in%d" % (name, len(lst), i), gi.detach().clone()))
                        for i, go in enumerate(outs):
                            if torch.is_tensor(go):
                                lst.append(("%s#%d out%d" % (name, len(lst), i), go.detach().clone()))
                    return out
                return staticmethod(bwd)
            setattr(cls, "backward", make(fn, name))


def main():
    from regcn_amd import cli, ranking, training
    common = ["-d", "synthetic:icews14s_lgcn_roth", "--gpu", "0", "--encoder", "lgcn", "--decoder", "roth",
              "--n-hidden", "64", "--n-bases", "32", "--synthetic-snapshots", "10", "--train-history-len", "3",
              "--test-history-len", "3", "--relation-prediction", "--entity-prediction",
              "--checkpoint", "/tmp/graphdbg2.pth", "--seed", "0", "--lr", "0.01", "--triple-batch-size", "64",
              "--dropout", "0", "--input-dropout", "0", "--hidden-dropout", "0", "--feat-dropout", "0",
              "--n-epochs", "3", "--evaluate-every", "1", "--hip-graph"]
    dev = torch.device("cuda", 0)
    adam = torch.optim.Adam
    opts, gss = [], []

    class CapturableAdam(adam):
        def __init__(self, *a, **k):
            k["capturable"] = True
            super().__init__(*a, **k)
            opts.append(self)

    steps = {}
    rec, cur_key = {}, []
    install_recorders(rec, cur_key)

    class RecGS(training.GraphedSteps):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            gss.append(self)

        def run(self, key, step):
            steps.setdefault(key, step)
            cur_key[:] = [key]
            try:
                return super().run(key, step)
            finally:
                cur_key[:] = []

    torch.optim.Adam = CapturableAdam
    cli.GraphedSteps = RecGS
    real_test = cli.test
    args = cli.build_parser().parse_args(common)
    V, R, train, valid, _ = cli.load_dataset(args)
    tl = ranking.split_by_time(train)
    vl = ranking.split_by_time(valid)
    torch.manual_seed(0)
    model = cli.build_model(args, V, R, tl, dev)
    done = []

    def experiment(*a, **k):
        """Runs as the first validation, inside train_model (the graphs' inputs are alive)."""
        if done:
            return (0.0, 0.0, 0.0, 0.0)
        done.append(1)
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
        saved = {kk: v.detach().clone() for kk, v in tensors.items()}

        def restore():
            with torch.no_grad():
                for kk, v in tensors.items():
                    v.copy_(saved[kk])
            torch.cuda.synchronize()

        def replay(key):
            restore()
            with torch.cuda.stream(gs.stream):
                gs.graphs[key][0].replay()
            torch.cuda.synchronize()
            out = ({kk: v.detach().clone() for kk, v in tensors.items()}, gs.graphs[key][1].detach().clone())
            restore()
            return out

        def eager(key):
            restore()
            with torch.cuda.stream(gs.stream):
                o = steps[key]()
            torch.cuda.synchronize()
            out = ({kk: v.detach().clone() for kk, v in tensors.items()}, o.detach().clone())
            restore()
            return out

        def diff(x, y):
            out = []
            for kk in x[0]:
                if not torch.equal(x[0][kk], y[0][kk]):
                    dd = float((x[0][kk].double() - y[0][kk].double()).abs().max())
                    rr = dd / max(float(x[0][kk].double().abs().max()), 1e-30)
                    out.append("%s(%.2e rel %.1e)" % (kk, dd, rr))
            head = "losses %s vs %s; " % (x[1].tolist(), y[1].tolist()) if not torch.equal(x[1], y[1]) else ""
            return head + ("%d tensors differ: %s" % (len(out), " ".join(out[:40])) if out else "all equal")

        def h2d():
            t = torch.from_numpy(np.asarray(vl[0], dtype=np.int64)).to(dev)
            del t

        def snap():
            torch.cuda.memory_snapshot()

        def device_build():
            from regcn_amd.graph import build_sub_graph
            gl = [build_sub_graph(V, R, s_, True, dev) for s_ in tl[-3:]]
            del gl

        def junk():
            j = [torch.full((1 << 26,), 3.0, device=dev) for _ in range(16)]
            del j

        def small_allocs():
            j = [torch.full((1000 + 37 * i,), 3.0, device=dev) for i in range(64)]
            del j

        keys = sorted(gs.graphs)
        print("graphs:", len(keys), "keys", keys[:5], "recorded:", {k: len(v) for k, v in rec.items()}, flush=True)

        def rec_snap(key):
            return [(n, t.clone()) for n, t in rec.get(key, [])]

        def rec_diff(a, b):
            out = []
            for (n, x), (_, y) in zip(a, b):
                if not torch.equal(x, y):
                    dd = float((x.double() - y.double()).abs().max())
                    out.append("%s(%.2e)" % (n, dd))
            return out

        for key in keys:
            replay(key)
            r0 = rec_snap(key)
            replay(key)
            r1 = rec_snap(key)
            junk()
            replay(key)
            r2 = rec_snap(key)
            for k2 in keys:
                if k2 != key:
                    replay(k2)
            replay(key)
            r3 = rec_snap(key)
            print("key %s: %d recorded; twice: %s | after junk: %s | after other graphs: %s" % (
                key, len(r0), rec_diff(r0, r1)[:4], rec_diff(r0, r2)[:6], rec_diff(r0, r3)[:6]), flush=True)
        for key in keys[:2]:
            e0 = eager(key)
            print("key %s: eager twice         -> %s" % (key, diff(e0, eager(key))), flush=True)
            junk()
            print("key %s: eager after junk    -> %s" % (key, diff(e0, eager(key))), flush=True)
            print("key %s: replay vs eager     -> %s" % (key, diff(e0, replay(key))), flush=True)
        import warnings
        torch.use_deterministic_algorithms(True, warn_only=True)
        with warnings.catch_warnings(record=True) as wl:
            warnings.simplefilter("always")
            eager(keys[0])
        torch.use_deterministic_algorithms(False)
        print("nondeterministic ops:", sorted({str(w.message)[:160] for w in wl}), flush=True)
        for key in keys[:2]:
            base = replay(key)
            print("key %s: replay twice        -> %s" % (key, diff(base, replay(key))), flush=True)
            for name, fn in (("h2d", h2d), ("memory_snapshot", snap), ("device_build", device_build),
                             ("junk", junk), ("small allocs", small_allocs)):
                fn()
                torch.cuda.synchronize()
                print("key %s: after %-16s -> %s" % (key, name, diff(base, replay(key))), flush=True)
        return (0.0, 0.0, 0.0, 0.0)

    cli.test = experiment
    random.seed(0)
    try:
        cli.train_model(args, model, tl, valid, V, R, dev, "/tmp/graphdbg2.pth")
    finally:
        cli.test = real_test
        torch.optim.Adam = adam
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
