"""Backward kernels (csrc/backward.hip, score.hip MODE 2) vs torch
autograd through the oracle's restatement of the reference ops, in fp64 on the CPU.

Tolerance: |delta| <= 2e-4 * max(1, max|ref|) per gradient tensor (fp32 kernels vs an fp64
reference; the forward bar of 1e-4 doubled for the extra chain-rule arithmetic)."""
import numpy as np
import pytest
import torch

from oracle import ops as O
from regcn_amd import autograd as A
from regcn_amd import graph as G
from regcn_amd.synthetic import zipf_triples

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
C = 0.01
TOL = 2e-4


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def close(got, ref, what, tol=TOL):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    scale = max(1.0, float(ref.abs().max())) if ref.numel() else 1.0
    err = float((got - ref).abs().max()) / scale if ref.numel() else 0.0
    assert err <= tol, "%s: max err %.3g (scale %.3g)" % (what, err, scale)


def rows(n, d, seed, lo=0.05, hi=12.0):
    """Rows with norms log-uniform in [lo, hi] (ball radius 1/sqrt(c) = 10: both sides of
    the projection clamp)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, d, generator=g, dtype=torch.float64)
    nr = torch.exp(torch.empty(n, 1, dtype=torch.float64).uniform_(np.log(lo), np.log(hi), generator=g))
    return x / x.norm(dim=1, keepdim=True) * nr


def grads(fn, inputs, gout):
    ins = [t.detach().clone().requires_grad_(True) for t in inputs]
    out = fn(*ins)
    outs = out if isinstance(out, tuple) else (out,)
    gouts = gout if isinstance(gout, tuple) else (gout,)
    torch.autograd.backward(outs, gouts)
    return outs, [t.grad for t in ins]


def run_both(ref_fn, hip_fn, inputs, gout):
    ro, rg = grads(ref_fn, inputs, gout)
    ho, hg = grads(hip_fn, [t.float().to(DEV) for t in inputs],
                   tuple(t.float().to(DEV) for t in (gout if isinstance(gout, tuple) else (gout,))))
    return ro, rg, ho, hg


@pytest.mark.parametrize("op", ["log0", "exp0", "project"])
@pytest.mark.parametrize("d", [200, 64, 12])
def test_radial_row_map_grads(op, d):
    hi = 9.0 if op == "log0" else (4.0 if op == "exp0" else 12.0)  # log0: inside the ball
    x = rows(300, d, 1, hi=hi)
    gout = rows(300, d, 2, lo=0.5, hi=2.0)
    ref = {"log0": lambda t: O.log0(t, C), "exp0": lambda t: O.exp0(t, C), "project": lambda t: O.project(t, C)}[op]
    hip = {"log0": lambda t: A.log0(t, C), "exp0": lambda t: A.exp0(t, C), "project": lambda t: A.project(t, C)}[op]
    ro, rg, ho, hg = run_both(ref, hip, [x], gout)
    close(ho[0], ro[0], op + " forward", 1e-4)
    close(hg[0], rg[0], op + " grad")


def test_log0_near_boundary_grad():
    """Rows at 0.99 of the ball radius: atanh' ~ 50 amplifies fp32 rounding; the bound
    scales with it."""
    x = rows(200, 200, 3, lo=9.8, hi=9.9)
    gout = rows(200, 200, 4, lo=0.5, hi=2.0)
    ro, rg, ho, hg = run_both(lambda t: O.log0(t, C), lambda t: A.log0(t, C), [x], gout)
    close(hg[0], rg[0], "log0 grad near boundary", 5e-3)


def test_apply_radius_and_get_radius_grads():
    x = rows(300, 200, 5, lo=1e-3, hi=5.0)
    r = torch.empty(300, dtype=torch.float64).uniform_(-0.5, 11.0, generator=torch.Generator().manual_seed(6))
    gout = rows(300, 200, 7, lo=0.5, hi=2.0)
    ro, rg, ho, hg = run_both(lambda a, b: O.apply_radius(a, b, C), lambda a, b: A.apply_radius(a, b, C), [x, r],
                              gout)
    close(ho[0], ro[0], "apply_radius forward", 1e-4)
    close(hg[0], rg[0], "apply_radius dx")
    close(hg[1], rg[1], "apply_radius dr")
    gr = torch.randn(300, dtype=torch.float64, generator=torch.Generator().manual_seed(8))
    ro, rg, ho, hg = run_both(lambda a: O.get_radius(a), lambda a: A.get_radius(a), [x], gr)
    close(hg[0], rg[0], "get_radius dx")


@pytest.mark.parametrize("scale", [1.0, 8.0])
def test_mobius_add_grads(scale):
    """scale 8: sums leave the ball and hit the projection."""
    x = rows(300, 200, 9, hi=scale)
    y = rows(300, 200, 10, hi=scale)
    gout = rows(300, 200, 11, lo=0.5, hi=2.0)
    ro, rg, ho, hg = run_both(lambda a, b: O.mobius_add(a, b, C), lambda a, b: A.mobius_add(a, b, C), [x, y], gout)
    close(ho[0], ro[0], "mobius forward", 1e-4)
    close(hg[0], rg[0], "mobius dx", 5e-4)
    close(hg[1], rg[1], "mobius dy", 5e-4)


def _graph(V, R, T, seed, **kw):
    tr = zipf_triples(np.random.default_rng(seed), V, R, T)
    g = G.build_sub_graph(V, R, tr, True, DEV, **kw)
    src = np.concatenate((tr[:, 0], tr[:, 2]))
    dst = np.concatenate((tr[:, 2], tr[:, 0]))
    et = np.concatenate((tr[:, 1], tr[:, 1] + R))
    return g, torch.from_numpy(src), torch.from_numpy(dst), torch.from_numpy(et)


def _segsum(m, dst, n):
    return torch.zeros((n,) + tuple(m.shape[1:]), dtype=m.dtype).index_add_(0, dst, m)


@pytest.mark.parametrize("gamma", [0.0, 0.15, 1.0])
def test_union_aggregate_grads(gamma):
    V, R, T, d = 600, 12, 3000, 200
    g, src, dst, et = _graph(V, R, T, 1)
    deg = torch.bincount(dst, minlength=V).double()
    norm = 1.0 / torch.where(deg > 0, deg, torch.ones_like(deg))
    x = rows(V, d, 12, hi=3.0)
    r = torch.empty(V, dtype=torch.float64).uniform_(0.5, 3.0, generator=torch.Generator().manual_seed(13))
    rel = rows(2 * R, d, 14, hi=2.0)
    gout = rows(V, d, 15, lo=0.5, hi=2.0)

    def ref(x, r, rel):
        w = torch.exp(-gamma * torch.abs(r[src] - r[dst]))
        return _segsum((x[src] + rel[et]) * w.unsqueeze(-1), dst, V) * norm.unsqueeze(-1)

    ro, rg, ho, hg = run_both(ref, lambda a, b, c: A.union_aggregate(a, b, c, g, gamma), [x, r, rel], gout)
    close(ho[0], ro[0], "union agg forward", 1e-4)
    close(hg[0], rg[0], "union dx")
    close(hg[1], rg[1], "union dradius")
    close(hg[2], rg[2], "union drel")


def _lorentz_ref(x, rel, W, src, dst, et, V, d, nb):
    s = d // nb
    m = torch.bmm(x[src].view(-1, 1, s), W.index_select(0, et).view(-1, s, s)).view(-1, d) + rel[et]
    L = O.to_lorentz(O.exp0(m, C), C)
    S = _segsum(L, dst, V)
    return S[:, 0], S[:, 1:]


@pytest.mark.parametrize("nb", [100, 200, 50])
def test_lorentz_sum_grads(nb):
    V, R, T, d = 500, 10, 2500, 200
    g, src, dst, et = _graph(V, R, T, 2)
    s = d // nb
    x = rows(V, d, 16, hi=3.0)
    rel = rows(2 * R, d, 17, hi=1.0)
    W = torch.randn(2 * R, nb * s * s, dtype=torch.float64, generator=torch.Generator().manual_seed(18)) * 0.5
    g0 = torch.randn(V, dtype=torch.float64, generator=torch.Generator().manual_seed(19))
    gv = rows(V, d, 20, lo=0.5, hi=2.0)
    ro, rg, ho, hg = run_both(lambda a, b, c: _lorentz_ref(a, b, c, src, dst, et, V, d, nb),
                              lambda a, b, c: A.lorentz_sum(a, b, c, g, nb, C), [x, rel, W], (g0, gv))
    close(ho[0], ro[0], "S0", 1e-4)
    close(ho[1], ro[1], "Sv", 1e-4)
    close(hg[0], rg[0], "lorentz dx")
    close(hg[1], rg[1], "lorentz drel")
    close(hg[2], rg[2], "lorentz dW")


def test_lorentz_aggregate_grads_vs_centroid():
    """Centroid -> to_poincare -> log0 on the raw sums vs the oracle's mailbox centroid with the
    reference's 1/deg weights (zero in-degree rows -> 0)."""
    V, R, T, d, nb = 400, 8, 1500, 200, 100
    g, src, dst, et = _graph(V, R, T, 3)
    x = rows(V, d, 21, hi=3.0)
    rel = rows(2 * R, d, 22, hi=1.0)
    W = torch.randn(2 * R, nb * 4, dtype=torch.float64, generator=torch.Generator().manual_seed(23)) * 0.5
    gout = rows(V, d, 24, lo=0.5, hi=2.0)
    deg = torch.bincount(dst, minlength=V)

    def ref(x, rel, W):
        s = d // nb
        m = torch.bmm(x[src].view(-1, 1, s), W.index_select(0, et).view(-1, s, s)).view(-1, d) + rel[et]
        L = O.to_lorentz(O.exp0(m, C), C)
        w = torch.ones(len(src), dtype=x.dtype) / deg[dst].double()
        w = w / (_segsum(w, dst, V)[dst] + 1e-6)
        w = w / (_segsum(w, dst, V)[dst] + 1e-6)
        cen = _segsum(w.unsqueeze(-1) * L, dst, V)
        ip = (-cen[:, :1] ** 2 + (cen[:, 1:] ** 2).sum(-1, keepdim=True))
        cen = cen / torch.sqrt(torch.clamp(-ip * C, min=1e-6))
        out = O.log0(O.to_poincare(cen, C), C)
        return torch.where((deg > 0).unsqueeze(-1), out, torch.zeros_like(out))

    ro, rg, ho, hg = run_both(ref, lambda a, b, c: A.lorentz_aggregate(a, b, c, g, nb, C), [x, rel, W], gout)
    close(ho[0], ro[0], "lorentz aggregate forward", 1e-4)
    for got, want, what in zip(hg, rg, ("dx", "drel", "dW")):
        close(got, want, "lorentz aggregate " + what)


@pytest.mark.parametrize("B,N", [(130, 700), (256, 2000), (7, 64)])
@pytest.mark.parametrize("bias", [False, True])
def test_hyp_ce_grads(B, N, bias):
    from oracle.model import ce_loss
    d = 200
    q = rows(B, d, 30, hi=9.0)
    e = rows(N, d, 31, hi=9.9)
    tgt = torch.randint(0, N, (B,), generator=torch.Generator().manual_seed(32))
    b = torch.randn(N, dtype=torch.float64, generator=torch.Generator().manual_seed(33)) * 0.1
    scale = torch.tensor(1.3, dtype=torch.float64)
    margin = torch.tensor(0.7, dtype=torch.float64)
    inputs = [q, e, b, scale, margin] if bias else [q, e, scale, margin]

    def ref(*t):
        if bias:
            return ce_loss(t[0], t[1], tgt, C, bias=t[2], scale=t[3], margin=t[4])
        return ce_loss(t[0], t[1], tgt, C, scale=t[2], margin=t[3])

    def hip(*t):
        if bias:
            return A.hyp_ce_loss(t[0], t[1], tgt.to(DEV), C, bias=t[2], scale=t[3], margin=t[4])
        return A.hyp_ce_loss(t[0], t[1], tgt.to(DEV), C, scale=t[2], margin=t[3])

    ro, rg, ho, hg = run_both(ref, hip, inputs, torch.tensor(1.0, dtype=torch.float64))
    close(ho[0], ro[0], "CE loss", 1e-4)
    names = ["dq", "de", "dbias", "dscale", "dmargin"] if bias else ["dq", "de", "dscale", "dmargin"]
    for got, want, what in zip(hg, rg, names):
        close(got, want, "CE " + what, 5e-4)


def test_transposed_lists():
    V, R, T = 700, 9, 4000
    g, src, dst, et = _graph(V, R, T, 4)
    tr = g.transposed()
    wk = g.work()
    rowptr = wk["rowptr"].cpu().numpy()
    cs, ct = wk["col_src"].cpu().numpy(), wk["col_type"].cpu().numpy()
    csr_dst = np.repeat(np.arange(V), np.diff(rowptr))
    np.testing.assert_array_equal(tr["csr_dst"].cpu().numpy(), csr_dst)
    sp = np.argsort(cs, kind="stable")
    np.testing.assert_array_equal(tr["sp"].cpu().numpy(), sp)
    np.testing.assert_array_equal(tr["sptr"].cpu().numpy(), np.concatenate([[0], np.cumsum(np.bincount(cs, minlength=V))]))
    tp = np.argsort(ct, kind="stable")
    np.testing.assert_array_equal(tr["tp"].cpu().numpy(), tp)
    # row / type order of the Lorentz edge lists: (row, type, CSR position), rows unchanged
    order = np.lexsort((np.arange(len(ct)), ct, csr_dst))
    s2, t2 = g.row_type_cols()
    np.testing.assert_array_equal(s2.cpu().numpy(), cs[order])
    np.testing.assert_array_equal(t2.cpu().numpy(), ct[order])
    np.testing.assert_array_equal(tr["tptr"].cpu().numpy(),
                                  np.concatenate([[0], np.cumsum(np.bincount(ct, minlength=2 * R))]))


@pytest.mark.parametrize("K,M,N,ak,bk", [(7128, 200, 200, True, True), (7128, 64, 200, False, True),
                                          (7127, 64, 200, False, True), (64, 7128, 200, True, True),
                                          (200, 128, 200, False, False), (201, 108, 100, False, False),
                                          (10000, 128, 200, False, False), (7128, 1, 200, True, True),
                                          (1, 3, 5, True, True), (37, 65, 129, False, True), (0, 16, 16, True, True),
                                          (100000, 16, 48, True, False), (3001, 204, 100, True, True),
                                          (7128, 200, 400, True, True), (100, 36, 52, True, True)])
def test_kreduce_mm(K, M, N, ak, bk):
    """regcn_kreduce_gemm_f32 (split-K MFMA, deterministic partial sum) against fp64 torch:
    every A/B layout, the float4 R-major reads (K % 4 == 0) and their scalar fallback (K odd),
    both-K-major products with odd K and partial tiles,
    ragged M/N, K = 0, a K long enough for many splits; no c0, a full c0, a bias row."""
    g = torch.Generator(device="cpu").manual_seed(K * 7 + M + N)
    a = torch.randn((K, M) if ak else (M, K), generator=g)
    b = torch.randn((K, N) if bk else (N, K), generator=g)
    ref = (a.double().t() if ak else a.double()) @ (b.double() if bk else b.double().t())
    tol = 1e-5 * max(1.0, float(ref.abs().max())) * max(1.0, K ** 0.5 / 30)
    for cc in (None, torch.randn(M, N, generator=g), torch.randn(N, generator=g)):
        got = A.kreduce_mm(a.to(DEV), b.to(DEV), ak, None if cc is None else cc.to(DEV), b_kmajor=bk)
        want = ref if cc is None else ref + cc.double()
        assert float((got.double().cpu() - want).abs().max()) <= tol
    again = A.kreduce_mm(a.to(DEV), b.to(DEV), ak, b_kmajor=bk)
    torch.testing.assert_close(again, A.kreduce_mm(a.to(DEV), b.to(DEV), ak, b_kmajor=bk), rtol=0, atol=0)


def test_linear_grads():
    """A.linear (nn.Linear forward, dx, dW, dbias on the split-K kernel) against fp64 torch."""
    g = torch.Generator(device="cpu").manual_seed(5)
    lin = torch.nn.Linear(200, 100).to(DEV)
    x = torch.randn(128, 200, generator=g).to(DEV).requires_grad_(True)
    gy = torch.randn(128, 100, generator=g).to(DEV)
    A.linear(lin, x).backward(gy)
    x64 = x.detach().double().requires_grad_(True)
    w64 = lin.weight.detach().double().requires_grad_(True)
    b64 = lin.bias.detach().double().requires_grad_(True)
    torch.nn.functional.linear(x64, w64, b64).backward(gy.double())
    for got, ref in ((x.grad, x64.grad), (lin.weight.grad, w64.grad), (lin.bias.grad, b64.grad)):
        assert float((got.double() - ref).abs().max()) <= 1e-5 * max(1.0, float(ref.abs().max()))


def test_mm_weight_grads():
    """A.mm_weight: x @ W with the weight gradient x^T dy on the split-K kernel."""
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(7128, 200, generator=g).to(DEV).requires_grad_(True)
    w = (torch.randn(200, 200, generator=g) / 200 ** 0.5).to(DEV).requires_grad_(True)
    gy = torch.randn(7128, 200, generator=g).to(DEV)
    A.mm_weight(x, w).backward(gy)
    x64, w64 = x.detach().double().requires_grad_(True), w.detach().double().requires_grad_(True)
    (x64 @ w64).backward(gy.double())
    for got, ref in ((x.grad, x64.grad), (w.grad, w64.grad)):
        assert float((got.double() - ref).abs().max()) <= 1e-5 * max(1.0, float(ref.abs().max()))


@pytest.mark.parametrize("case", ["layer_skip", "layer", "time_gate", "euclid"])
def test_fused_tail(case):
    """A.tail (regcn_tail_f32) against the op-by-op torch composition it replaces: forward to
    2e-5 absolute (same fp32 op order without contraction; only sigmoid's expf may differ in
    the last ulp), gradients of every input to 1e-5 of their max; values straddle the +-10
    clamps and 0."""
    V, d = 1037, 200
    g = torch.Generator(device="cpu").manual_seed(11)
    mk = lambda s=1.0: (s * torch.randn(V, d, generator=g)).to(DEV).requires_grad_(True)
    agg, z, p = mk(8.0), mk(2.0), mk(6.0)
    loop = (4.0 * torch.randn(V, 2 * d, generator=g)).to(DEV).requires_grad_(True)
    bias = (0.3 * torch.randn(d, generator=g)).to(DEV).requires_grad_(True)
    pos = (torch.rand(V, generator=g) > 0.4).to(torch.uint8).to(DEV)
    slope = (1.0 / 8 + 1.0 / 3) / 2
    args = {"layer_skip": (agg, loop, pos, z, bias, p, 7, slope), "layer": (agg, loop, pos, None, None, None, 7, slope),
            "time_gate": (agg, None, None, z, bias, p, 1, 0.0), "euclid": (agg, loop, pos, None, None, None, 4, slope)}[case]
    gy = torch.randn(V, d, generator=g).to(DEV)
    ins = [t for t in args[:6] if t is not None and t.dtype == torch.float32]
    out = A.tail(*args)
    got = torch.autograd.grad(out, ins, gy)
    ref_out = A._tail_torch(*args)
    ref = torch.autograd.grad(ref_out, ins, gy)
    assert float((out - ref_out).abs().max()) <= 2e-6 * 10
    for a, b in zip(got, ref):
        assert float((a - b).abs().max()) <= 1e-5 * max(1.0, float(b.abs().max()))


def test_lorentz_centroid():
    """regcn_lorentz_centroid_f32 (A._Centroid) against the torch composition it replaces,
    forward and both gradients; raw sums shaped like a Lorentz layer's (S0 > |Sv|), plus rows
    hitting the eps clamps (S0 = |Sv| = 0)."""
    V, d, c = 513, 200, 0.01
    g = torch.Generator(device="cpu").manual_seed(13)
    Sv = torch.randn(V, d, generator=g)
    S0 = (Sv.norm(dim=1) ** 2 + 1.0 / c).sqrt() * (1 + torch.rand(V, generator=g))
    S0[:7], Sv[:7] = 0.0, 0.0
    S0, Sv = S0.to(DEV).requires_grad_(True), Sv.to(DEV).requires_grad_(True)
    gy = torch.randn(V, d, generator=g).to(DEV)
    y = A._Centroid.apply(S0, Sv, c)
    got = torch.autograd.grad(y, (S0, Sv), gy)
    yr = A._centroid_torch(S0, Sv, c)
    ref = torch.autograd.grad(yr, (S0, Sv), gy)
    assert float((y - yr).abs().max()) <= 1e-5 * max(1.0, float(yr.abs().max()))
    for a, b in zip(got, ref):
        assert float((a - b).abs().max()) <= 1e-4 * max(1.0, float(b.abs().max()))


@pytest.mark.parametrize("reflect", [False, True])
def test_givens_rotation(reflect):
    """regcn_givens_rotation_f32 (A.givens_rotation) against the torch compositions of
    hyperbolic_decoder.givens_rotation / givens_reflection: forward to 1e-6, both gradients
    to 1e-5."""
    g = torch.Generator(device="cpu").manual_seed(17)
    x = torch.randn(128, 200, generator=g).to(DEV).requires_grad_(True)
    a = (3 * torch.randn(128, 100, generator=g)).to(DEV).requires_grad_(True)
    gy = torch.randn(128, 200, generator=g).to(DEV)
    out = A.givens_rotation(x, a, reflect=reflect)
    got = torch.autograd.grad(out, (x, a), gy)
    x1, x2 = x[:, 0::2], x[:, 1::2]
    co, si = torch.cos(a), torch.sin(a)
    pair = [co * x1 + si * x2, si * x1 - co * x2] if reflect else [co * x1 - si * x2, si * x1 + co * x2]
    ref_t = torch.stack(pair, dim=2).reshape(128, 200)
    ref = torch.autograd.grad(ref_t, (x, a), gy)
    assert float((out - ref_t).abs().max()) <= 1e-6 * max(1.0, float(ref_t.abs().max()))
    for u, v in zip(got, ref):
        assert float((u - v).abs().max()) <= 1e-5 * max(1.0, float(v.abs().max()))
