"""Debug: list the torch ops of a captured training step that read HOST memory (a CPU tensor
argument of an op whose result lives on the GPU): inside a HIP graph such a copy is a memcpy
node from the host address the tensor had at capture time, which every replay reads again
-- whatever that memory holds by then.

  python tools/capture_h2d.py
"""
import os
import random
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))


class HostReads(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.hits = {}

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        if torch.cuda.is_current_stream_capturing():
            flat = list(args) + list((kwargs or {}).values())
            flat = [y for x in flat for y in (x if isinstance(x, (list, tuple)) else [x])]
            cpu = [t for t in flat if isinstance(t, torch.Tensor) and t.device.type == "cpu"]
            outs = out if isinstance(out, (list, tuple)) else [out]
            gpu_out = any(isinstance(t, torch.Tensor) and t.is_cuda for t in outs)
            if cpu and gpu_out:
                st = " < ".join("%s:%d" % (os.path.basename(f.filename), f.lineno)
                                for f in reversed(traceback.extract_stack(limit=14)[:-1])
                                if "torch/" not in f.filename and "capture_h2d" not in f.filename)
                key = "%s cpu%s | %s" % (func.__name__, [tuple(t.shape) for t in cpu], st)
                self.hits[key] = self.hits.get(key, 0) + 1
        return out


def main():
    from regcn_amd import cli, ranking
    args = cli.build_parser().parse_args(
        ["-d", "synthetic:icews14s_lgcn_roth", "--gpu", "0", "--encoder", "lgcn", "--decoder", "roth", "--n-hidden",
         "64", "--n-bases", "32", "--synthetic-snapshots", "10", "--train-history-len", "3", "--test-history-len", "3",
         "--relation-prediction", "--entity-prediction", "--checkpoint", "/tmp/capture_h2d.pth", "--seed", "0",
         "--lr", "0.01", "--triple-batch-size", "64", "--dropout", "0", "--input-dropout", "0", "--hidden-dropout",
         "0", "--feat-dropout", "0", "--n-epochs", "1", "--evaluate-every", "100", "--hip-graph"])
    dev = torch.device("cuda", 0)
    V, R, train, valid, _ = cli.load_dataset(args)
    tl = ranking.split_by_time(train)
    torch.manual_seed(0)
    model = cli.build_model(args, V, R, tl, dev)
    random.seed(0)
    mode = HostReads()
    with mode:
        cli.train_model(args, model, tl, valid, V, R, dev, "/tmp/capture_h2d.pth")
    torch.cuda.synchronize()
    print("host-memory reads inside captures: %d distinct" % len(mode.hits))
    for k, n in sorted(mode.hits.items(), key=lambda x: -x[1]):
        print("%4d x %s" % (n, k[:400]))


if __name__ == "__main__":
    main()
