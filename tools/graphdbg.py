"""Debug: does validation between graphed training epochs perturb the replays?  Runs the
CLI training loop (lgcn + RoTH, synthetic ICEWS14s, dropout 0) eagerly and with --hip-graph
under variants of what happens at validation time, printing the epoch losses.

  python tools/graphdbg.py
"""
import os
import random
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))


def main():
    if os.environ.get("DETERMINISTIC"):
        torch.use_deterministic_algorithms(True, warn_only=True)
    from regcn_amd import cli, ranking, weights
    common = ["-d", "synthetic:icews14s_lgcn_roth", "--gpu", "0", "--encoder", "lgcn", "--decoder", "roth",
              "--n-hidden", "64", "--n-bases", "32", "--synthetic-snapshots", "10", "--train-history-len", "3",
              "--test-history-len", "3", "--relation-prediction", "--entity-prediction",
              "--checkpoint", "/tmp/graphdbg.pth", "--seed", "0", "--lr", "0.01", "--triple-batch-size", "64",
              "--dropout", "0", "--input-dropout", "0", "--hidden-dropout", "0", "--feat-dropout", "0",
              "--n-epochs", "4", "--evaluate-every", "1"]
    dev = torch.device("cuda", 0)
    adam = torch.optim.Adam

    opts = []

    class CapturableAdam(adam):
        def __init__(self, *a, **k):
            k["capturable"] = True
            super().__init__(*a, **k)
            opts.append(self)

    torch.optim.Adam = CapturableAdam
    real_test, real_inv = cli.test, cli.invalidate

    def run(name, extra, test=None, inv=None):
        cli.test = test or real_test
        cli.invalidate = inv or real_inv
        args = cli.build_parser().parse_args(common + extra)
        V, R, train, valid, _ = cli.load_dataset(args)
        tl = ranking.split_by_time(train)
        torch.manual_seed(0)
        model = cli.build_model(args, V, R, tl, dev)
        random.seed(0)
        out = cli.train_model(args, model, tl, valid, V, R, dev, "/tmp/graphdbg.pth")
        torch.cuda.synchronize()
        print("%-28s loss %s valid %s" % (name, np.array2string(np.array(out["epoch_loss"]), precision=7),
                                           [round(v[2], 6) for v in out["valid"]]), flush=True)
        cli.test, cli.invalidate = real_test, real_inv

    def dummy_test(*a, **k):
        return (0.0, 0.0, 0.0, 0.0)

    def param_guard_test(model, *a, **k):
        torch.cuda.synchronize()
        names = {id(p): n for n, p in model.named_parameters()}
        state = {}
        for p in model.parameters():
            for key, v in opts[-1].state.get(p, {}).items():
                if torch.is_tensor(v):
                    state[(names[id(p)], key)] = (v, v.detach().clone())
            if p.grad is not None:
                state[(names[id(p)], "grad")] = (p.grad, p.grad.detach().clone())
        before = {n: p.detach().clone() for n, p in model.named_parameters()}
        res = real_test(model, *a, **k)
        torch.cuda.synchronize()
        changed = [n for n, p in model.named_parameters() if not torch.equal(p.detach(), before[n])]
        st_changed = [k for k, (v, c) in state.items() if not torch.equal(v, c)]
        print("   validation changed parameters:", changed, "state/grads:", st_changed[:12], len(st_changed),
              "of", len(state), flush=True)
        return res

    def variant(kind):
        def t(model, history_list, test_list, num_rels, num_nodes, device, *a, **k):
            from regcn_amd.graph import build_sub_graph
            model.eval()
            T = 3
            if kind == "junk_only":
                junk = [torch.full((1 << 26,), 3.0, device=device) for _ in range(16)]
                del junk
                torch.cuda.synchronize()
                return (0.0, 0.0, 0.0, 0.0)
            if kind in ("host_build", "device_build"):
                gl = [build_sub_graph(num_nodes, num_rels, s, kind == "device_build", device)
                      for s in history_list[-T:]]
                if kind == "host_build":
                    gl = [g.to(device) for g in gl]
                del gl
                torch.cuda.synchronize()
                return (0.0, 0.0, 0.0, 0.0)
            if kind == "h2d":
                tt = torch.from_numpy(np.asarray(test_list[0], dtype=np.int64)).to(device)
                del tt
                torch.cuda.synchronize()
                return (0.0, 0.0, 0.0, 0.0)
            glist = [build_sub_graph(num_nodes, num_rels, s, True, device) for s in history_list[-T:]]
            tt = torch.from_numpy(np.asarray(test_list[0], dtype=np.int64)).to(device)
            with torch.no_grad():
                if kind == "scope":
                    with model.shared_parameter_states(T):
                        pass
                elif kind == "forward":
                    model.forward(glist, None, True)
                elif kind == "forward_nophase":
                    ph = model.use_phases
                    model.use_phases = False
                    model.forward(glist, None, True)
                    model.use_phases = ph
                elif kind == "predict":
                    model.predict(glist, num_rels, None, tt, True)
                elif kind.startswith("garbage"):  # overwrite every free block of the default pool
                    val = float(kind.split(":")[1]) if ":" in kind else 3.0
                    junk = [torch.full((1 << 26,), val, device=device) for _ in range(16)]
                    del junk
                elif kind == "scope_predict":
                    with model.shared_parameter_states(T):
                        model.predict(glist, num_rels, None, tt, True)
            torch.cuda.synchronize()
            return (0.0, 0.0, 0.0, 0.0)
        return t

    # which operands of captured work (library calls and torch ops) sit in default-pool blocks
    # that are free by validation time: the graphs then read memory the allocator hands out
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    from regcn_amd import _lib
    rec = {}
    real_addr = _lib.addr

    def note(ptr, nbytes, label):
        if ptr and (ptr, label) not in rec:
            rec[(ptr, label)] = nbytes

    def addr(t, dtype=torch.float32, what="tensor"):
        a = real_addr(t, dtype, what)
        if a is not None and torch.cuda.is_current_stream_capturing():
            st = [f"{os.path.basename(f.filename)}:{f.lineno}" for f in traceback.extract_stack(limit=6)[:-1]]
            note(a, t.numel() * t.element_size(), "lib %s %s %s | %s" % (what, tuple(t.shape), t.dtype, " < ".join(reversed(st[-4:]))))
        return a

    _lib.addr = addr

    class Rec(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            if torch.cuda.is_current_stream_capturing():
                for x in list(args) + list((kwargs or {}).values()):
                    xs = x if isinstance(x, (list, tuple)) else [x]
                    for t in xs:
                        if isinstance(t, torch.Tensor) and t.is_cuda and t.numel():
                            st = [f"{os.path.basename(f.filename)}:{f.lineno}" for f in traceback.extract_stack(limit=8)[:-1]
                                  if "torch/" not in f.filename and "graphdbg" not in f.filename]
                            note(t.data_ptr(), t.numel() * t.element_size(),
                                 "op %s %s %s | %s" % (func.__name__, tuple(t.shape), t.dtype, " < ".join(reversed(st[-3:]))))
            return func(*args, **(kwargs or {}))

    mode = Rec()

    def report(*a, **k):
        torch.cuda.synchronize()
        blocks = []
        for sg in torch.cuda.memory_snapshot():
            pool = tuple(sg.get("segment_pool_id", (0, 0)))
            ad = sg["address"]
            for b in sg["blocks"]:
                blocks.append((ad, ad + b["size"], b["state"], pool))
                ad += b["size"]
        blocks.sort()
        import bisect
        starts = [b[0] for b in blocks]
        bad = {}
        for (ptr, label), nb in rec.items():
            i = bisect.bisect_right(starts, ptr) - 1
            if i < 0 or not (blocks[i][0] <= ptr < blocks[i][1]):
                continue
            lo, hi, state, pool = blocks[i]
            if state != "active_allocated" and pool == (0, 0):
                bad[label] = bad.get(label, 0) + 1
        print("   captured operands in free default-pool blocks: %d" % len(bad), flush=True)
        for label, n in sorted(bad.items(), key=lambda x: -x[1])[:30]:
            print("     %3d x %s" % (n, label[:260]), flush=True)
        return (0.0, 0.0, 0.0, 0.0)

    which = os.environ.get("VARIANTS", "base")
    if which == "base":
        run("eager", [])
        run("eager, garbage 3", [], test=variant("garbage:3"))
        run("eager, predict", [], test=variant("predict"))
        run("graph, garbage 0", ["--hip-graph"], test=variant("garbage:0"))
        run("graph, garbage 3", ["--hip-graph"], test=variant("garbage:3"))
        run("graph, garbage nan", ["--hip-graph"], test=variant("garbage:nan"))
    else:  # bisect the trigger: what between the replays makes them drift
        from regcn_amd import weights as W
        noop = lambda m: None  # noqa: E731

        def inv_only(attrs):
            def f(module):
                for t in list(module.parameters()) + list(module.buffers()):
                    for a in attrs:
                        if hasattr(t, a):
                            delattr(t, a)
            return f

        def inv_model(keys):
            def f(module):
                for m in module.modules():
                    for a in keys:
                        m.__dict__.pop(a, None)
            return f
        run("eager", [])
        if which == "report":  # captured operands sitting in free default-pool blocks at validation
            with mode:
                run("graph, report", ["--hip-graph"], test=report, inv=noop)
        else:
            for kind in ("junk_only", "device_build", "host_build", "h2d"):
                run("graph, %s" % kind, ["--hip-graph"], test=variant(kind), inv=noop)
    torch.optim.Adam = adam


if __name__ == "__main__":
    main()
