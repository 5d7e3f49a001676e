"""Debug: regcn_union_aggregate_f32 in CSR and row/type edge order against a float64 torch
segment sum, on Zipf snapshots of growing size; prints the worst rows."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
from regcn_amd import _lib  # noqa: E402
from regcn_amd import graph as G  # noqa: E402
from regcn_amd.synthetic import snapshot_series  # noqa: E402

dev = torch.device("cuda", 0)
for V, T, chunk in [(2000, 20000, None), (20000, 500000, None), (100000, 4000000, None), (100000, 4000000, 64)]:
    R, d = 256, 200
    snap = snapshot_series(1, V, R, 1, T)[0]
    g = G.build_sub_graph(V, R, snap, True, dev, chunk_edges=chunk)
    wk = g.work()
    torch.manual_seed(0)
    x = torch.randn(V, d, device=dev) * 0.2
    r = torch.rand(V, device=dev) * 2.5 + 0.5
    rel = torch.randn(2 * R, d, device=dev) * 0.3
    tri = torch.from_numpy(snap).to(dev)
    src = torch.cat([tri[:, 0], tri[:, 2]])
    dst = torch.cat([tri[:, 2], tri[:, 0]])
    et = torch.cat([tri[:, 1], tri[:, 1] + R])
    w = torch.exp(-0.15 * (r[src] - r[dst]).abs()).double()
    msg = (x[src].double() + rel[et].double()) * w[:, None]
    ref = torch.zeros(V, d, device=dev, dtype=torch.float64).index_add_(0, dst, msg) * wk["norm"].double()[:, None]
    ch, fx = wk["chunks"], wk["fixups"]
    cs, ct = g.row_type_cols()
    for name, (c1, c2) in (("csr", (wk["col_src"], wk["col_type"])), ("rowtype", (cs, ct))):
        part = torch.empty(max(g.n_slots, 1), d + 4, device=dev)
        out = torch.zeros(V, d, device=dev)
        f, i = _lib.fptr, _lib.iptr
        _lib.call("regcn_union_aggregate_f32", f(x), f(r), f(rel), i(c1), i(c2), f(wk["norm"]), i(ch), ch.shape[0],
                  i(fx), fx.shape[0], 0.15, d, f(part), d + 4, f(out), _lib.stream())
        err = ((out.double() - ref).abs() / ref.abs().clamp_min(1.0)).max(1).values
        deg = g.in_degrees()
        bad = torch.nonzero(err > 1e-4).flatten()
        print("V=%d E=%d chunk=%d %s: max err %.3g, bad rows %d, worst row deg %d; bad degs %s"
              % (V, 2 * T, g.chunk_edges, name, float(err.max()), bad.numel(), int(deg[err.argmax()]),
                 deg[bad[:10]].tolist()), flush=True)
