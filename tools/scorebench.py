"""All-entity scorer at config-5 scale (B = 1024 queries, N = 1M candidates,
d = 200): the MFMA-bound decoder kernels, timed with HIP events on the launch stream.

flops per launch = 2 B N d (the Q E^T contraction only; the ~25-flop Mobius epilogue per pair
is not counted); peak = 157.3 TFLOP/s dense fp32 MFMA (MI355X_MICROARCH.md).  Modes: score
(writes B x N), ce (fused cross entropy, no B x N output), ce_bwd (training coefficients).

  python tools/scorebench.py [--B 1024] [--N 1000000] [--reps 5]
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))

PEAK = 157.3


def measure(B=1024, N=1_000_000, d=200, reps=5, modes="score,ce,ce_bwd", verbose=True):
    """HIP-event time per launch of each scorer mode at (B, N, d); returns a dict."""
    from regcn_amd import _lib
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)

    def ball(n):
        x = torch.randn(n, d, device=dev, generator=g)
        return x / x.norm(dim=1, keepdim=True) * torch.rand(n, 1, device=dev, generator=g) * 5.0

    q, e = ball(B), ball(N)
    bias = torch.randn(N, device=dev, generator=g) * 0.1
    scale = torch.tensor([1.3], device=dev)
    margin = torch.tensor([0.7], device=dev)
    tgt = torch.randint(0, N, (B,), device=dev, dtype=torch.int32, generator=g)
    f = _lib.fptr
    flops = 2.0 * B * N * d
    out = {"B": B, "N": N, "d": d, "flops_per_launch": flops, "peak_tflops": PEAK}
    S = torch.empty(B, N, device=dev) if "score" in modes else None
    ws = torch.empty((_lib.lib().regcn_hyp_ce_workspace_bytes(B, N) + 3) // 4, device=dev)
    loss = torch.empty(B, device=dev)
    lse = torch.empty(B, device=dev)
    nblk, ng = (N + 63) // 64, 8 * ((B + 127) // 128)
    coef = rsum = csum = None
    if "ce_bwd" in modes:
        coef = torch.empty(B, N, device=dev)
        rsum = torch.empty(B, nblk, device=dev)
        csum = torch.zeros(ng, N, 3, device=dev)
    gl = torch.full((B,), 1.0 / B, device=dev)
    runs = {
        "score": lambda: _lib.call("regcn_hyp_score_f32", f(q), f(e), f(bias), None, f(scale), f(margin), B, N, d,
                                   0.01, 0, f(S), _lib.stream()),
        "ce": lambda: _lib.call("regcn_hyp_ce_lse_f32", f(q), f(e), f(bias), f(scale), f(margin), _lib.iptr(tgt), B,
                                N, d, 0.01, 0, f(ws), f(loss), f(lse), _lib.stream()),
        "ce_bwd": lambda: _lib.call("regcn_hyp_ce_bwd_f32", f(q), f(e), f(bias), f(scale), f(margin), _lib.iptr(tgt),
                                    f(lse), f(gl), B, N, d, 0.01, 0, f(coef), f(rsum), f(csum), _lib.stream()),
    }
    if "ce_bwd" in modes:
        runs["ce"]()
    for mode in modes.split(","):
        fn = runs[mode]
        fn()
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        tf = flops / (ms * 1e-3) / 1e12
        out[mode] = {"ms": round(ms, 3), "tflops": round(tf, 2), "frac": round(tf / PEAK, 4)}
        if verbose:
            print(json.dumps({mode: out[mode]}), file=sys.stderr, flush=True)
    return out


def stamps(B=1024, N=1_000_000, d=200):
    """Per-phase cycle sums of the proxy scorer's workgroups (a library built with
    -DREGCN_SCORE_STAMPS=1, passed as REGCN_HIP_LIB): wave 0's s_memtime cycles in the products,
    the epilogue, the next tile's staging and the barrier, summed over its tiles; printed as the
    mean over workgroups and as fractions of their sum."""
    from regcn_amd import _lib
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, d, device=dev, generator=g) * 0.05
    e = torch.randn(N, d, device=dev, generator=g) * 0.05
    bias = torch.randn(N, device=dev, generator=g) * 0.1
    scale = torch.tensor([1.3], device=dev)
    margin = torch.tensor([0.7], device=dev)
    S = torch.empty(B, N, device=dev)
    f = _lib.fptr
    buf = torch.zeros(65536 * 16, dtype=torch.int64, device=dev)
    run = lambda: _lib.call("regcn_hyp_score_f32", f(q), f(e), f(bias), None, f(scale), f(margin), B, N, d, 0.01, 0,
                            f(S), _lib.stream())
    run()
    torch.cuda.synchronize()
    _lib.call("regcn_set_trace", _lib.addr(buf, torch.int64))
    run()
    torch.cuda.synchronize()
    _lib.call("regcn_set_trace", None)
    t = buf.view(-1, 16).cpu()
    used = t[:, 0] != 0
    ph = t[used][:, 4:8].double()
    names = ["products", "epilogue", "staging", "barrier"]
    mean = ph.mean(0)
    res = {"workgroups": int(used.sum()), "cycles_mean": {n: round(float(v)) for n, v in zip(names, mean)},
           "frac": {n: round(float(v / mean.sum()), 4) for n, v in zip(names, mean)},
           "span_us_mean": round(float((t[used][:, 2] - t[used][:, 0]).double().mean()) / 100.0, 1)}
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1024)
    ap.add_argument("--N", type=int, default=1_000_000)
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="score,ce,ce_bwd")
    ap.add_argument("--stamps", action="store_true", help="phase cycle sums (REGCN_SCORE_STAMPS build)")
    a = ap.parse_args()
    if a.stamps:
        stamps(a.B, a.N, a.d)
        return
    print(json.dumps(measure(a.B, a.N, a.d, a.reps, a.modes)), flush=True)


if __name__ == "__main__":
    main()
