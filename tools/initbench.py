"""Time the initial-state map (regcn_init_entities_f32 over V = 1M rows of d = 200, and
regcn_init_entity_rows_f32 over a rank's ~531k listed rows) with HIP events; run once with
REGCN_INIT_PLAIN=1 (k_rowmap) and once without (k_init_rows) for the A/B.  Prints one JSON line
with the mean us per call and the rate over the algorithmic bytes (2.4 KB per row)."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
from regcn_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    V, d, c = 1_000_000, 200, 0.01
    g = torch.Generator(device=dev).manual_seed(0)
    dyn = 0.1 * torch.randn(V, d, device=dev, generator=g)
    rs = 0.2 + torch.rand(V, device=dev, generator=g)
    h, x, r = torch.empty(V, d, device=dev), torch.empty(V, d, device=dev), torch.empty(V, device=dev)
    ids = torch.randperm(V, device=dev, generator=g)[:531_000].sort().values.to(torch.int32)
    f, i = _lib.fptr, _lib.iptr
    out = {"plain": os.environ.get("REGCN_INIT_PLAIN", "0")}

    def full():
        _lib.call("regcn_init_entities_f32", f(dyn), f(rs), V, d, c, 0, f(h), f(x), f(r), _lib.stream())

    def rows():
        _lib.call("regcn_init_entity_rows_f32", f(dyn), f(rs), i(ids), i(ids), ids.numel(), d, c, 0, f(h), f(x),
                  f(r), _lib.stream())
    for name, fn, n in (("full", full, V), ("rows", rows, ids.numel())):
        for _ in range(3):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / reps
        out[name] = {"us": round(us, 1), "TB_s": round(n * (3 * d * 4 + 8) / us / 1e6, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
