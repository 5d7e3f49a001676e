"""Autograd functions of the training path.

Each function runs its forward AND its backward as hand-written gfx950 kernels
(csrc/rowwise.hip, aggregate.hip, score.hip forward; csrc/backward.hip, score.hip backward),
with the gradients torch autograd would compute through the reference's op sequence:

  * row maps of hyperbolic_src/hyperbolic_ops.py (log0, exp0, project, apply_radius,
    get_radius, mobius_add) -> regcn_rowmap_bwd_f32;
  * the union layer's message sum (hyperbolic_layers.py:222-240, :290) ->
    regcn_union_aggregate_bwd_f32 over the snapshot's transposed edge lists;
  * the Lorentz layer's message sums (hyperbolic_layers.py:589-611) -> regcn_lorentz_sum_raw_f32
    / regcn_lorentz_aggregate_bwd_f32 (the centroid, to_poincare, log0 follow as row ops);
  * the all-entity cross entropy (_chunked_hyperbolic_ce_loss, hyperbolic_decoder.py:182-307)
    -> regcn_hyp_ce_lse_f32 / regcn_hyp_ce_bwd_f32 (+ dq, de on regcn_kreduce_gemm_f32);
  * the weight gradients of the (V x d) @ (d x d) products -> regcn_kreduce_gemm_f32.

A learned curvature (--learn-curvature, hyperbolic_model.py:299-300, :673-679) arrives as a
0-dim tensor `c` with requires_grad.  The reference lets its gradient flow through exp0,
log0, mobius_add and the decoders' scores, not through the project / apply_radius bounds (they
read c.item(), hyperbolic_ops.py:72, :228).  The row maps are radial (y = s(|x|, c) x) or, for
mobius_add, y = alpha(c) x + beta(c) y per row, so the HIP kernels keep the x-gradients and
the c-gradient is added by a zero-valued term (s(c) - s(c).detach()) x.detach() built from
per-row scalars on the device; the cross entropy gets the same from the per-pair scalars
(<q, e>, |q|^2, |e|^2) of its score.  The arctanh-distance score with per-query curvatures
(--plus-relation-specific-curvature, hyperbolic_decoder.py:145-164, :257-283) trains through
the same per-pair scalars in float64 (hyp_dist_ce_loss).
"""
import ctypes
import functools

import torch

from . import _lib

EPS = 1e-6
BWD = dict(log0=0, exp0=1, project=2, apply_radius=3, radius=4, mobius=5)
FWD = dict(log0="regcn_log0_f32", exp0="regcn_exp0_f32", project="regcn_project_f32")


def needs_grad(*ts):
    return torch.is_grad_enabled() and any(torch.is_tensor(t) and t.requires_grad for t in ts)


def _cf(c):
    return float(c.detach().item()) if torch.is_tensor(c) else float(c)


def _c_grad(c):
    """A learned curvature whose gradient this call must produce."""
    return torch.is_tensor(c) and c.requires_grad and torch.is_grad_enabled()


def _mx(c):
    """The project / clamp_norm bound 1/sqrt(c) - 2 eps as a constant (the reference reads
    c.item() there, hyperbolic_ops.py:72-74, :52)."""
    return 1.0 / (_cf(c) ** 0.5) - 2 * EPS


def _c_term(y, x, factor):
    """y + (factor - factor.detach()) x.detach(): the value of y, plus d/dc of the radial factor."""
    f = factor - factor.detach()
    return y + (f.to(y.dtype).unsqueeze(-1) * x.detach().reshape(y.shape))


def _rows(x):
    return x.reshape(-1, x.shape[-1]).contiguous().float()


def _bwd(op, x, y, g, c, dx, dy):
    f = _lib.fptr
    _lib.call("regcn_rowmap_bwd_f32", BWD[op], f(x, "x"), f(y), f(g.contiguous(), "grad"), x.shape[0], x.shape[-1],
              float(c), f(dx), f(dy), _lib.stream())


class _Radial(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, op, c):
        xr = _rows(x)
        out = torch.empty_like(xr)
        _lib.call(FWD[op], _lib.fptr(xr, "x"), xr.shape[0], xr.shape[1], float(c), _lib.fptr(out), _lib.stream())
        ctx.save_for_backward(xr)
        ctx.op, ctx.c, ctx.shape = op, c, x.shape
        return out.view(x.shape)

    @staticmethod
    def backward(ctx, g):
        (xr,) = ctx.saved_tensors
        dx = torch.empty_like(xr)
        _bwd(ctx.op, xr, None, _rows(g), ctx.c, dx, None)
        return dx.view(ctx.shape), None, None


class _ApplyRadius(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, radius, c):
        xr = _rows(x)
        rr = radius.reshape(-1).contiguous().float()
        out = torch.empty_like(xr)
        _lib.call("regcn_apply_radius_f32", _lib.fptr(xr, "x"), _lib.fptr(rr, "radius"), xr.shape[0], xr.shape[1],
                  float(c), _lib.fptr(out), _lib.stream())
        ctx.save_for_backward(xr, rr)
        ctx.c, ctx.shape, ctx.rshape = c, x.shape, radius.shape
        return out.view(x.shape)

    @staticmethod
    def backward(ctx, g):
        xr, rr = ctx.saved_tensors
        dx = torch.empty_like(xr)
        dr = torch.empty_like(rr)
        _bwd("apply_radius", xr, rr, _rows(g), ctx.c, dx, dr)
        return dx.view(ctx.shape), dr.view(ctx.rshape), None


class _Radius(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        xr = _rows(x)
        out = torch.empty(xr.shape[0], device=x.device, dtype=torch.float32)
        _lib.call("regcn_radius_f32", _lib.fptr(xr, "x"), xr.shape[0], xr.shape[1], _lib.fptr(out), _lib.stream())
        ctx.save_for_backward(xr)
        ctx.shape = x.shape
        return out.view(x.shape[:-1])

    @staticmethod
    def backward(ctx, g):
        (xr,) = ctx.saved_tensors
        dx = torch.empty_like(xr)
        _bwd("radius", xr, None, g.reshape(-1).contiguous().float(), 0.01, dx, None)
        return dx.view(ctx.shape)


class _Mobius(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, c):
        xr, yr = _rows(x), _rows(y)
        out = torch.empty_like(xr)
        _lib.call("regcn_mobius_add_f32", _lib.fptr(xr, "x"), _lib.fptr(yr, "y"), xr.shape[0], xr.shape[1], float(c),
                  _lib.fptr(out), _lib.stream())
        ctx.save_for_backward(xr, yr)
        ctx.c, ctx.shape = c, x.shape
        return out.view(x.shape)

    @staticmethod
    def backward(ctx, g):
        xr, yr = ctx.saved_tensors
        dx, dy = torch.empty_like(xr), torch.empty_like(yr)
        _bwd("mobius", xr, yr, _rows(g), ctx.c, dx, dy)
        return dx.view(ctx.shape), dy.view(ctx.shape), None


def log0(x, c):
    y = _Radial.apply(x, "log0", _cf(c))
    if _c_grad(c):  # atanh(min(sqrt(c) n, 1 - eps)) / (sqrt(c) n), n = max(|x|, eps)  (:97-116)
        sc = torch.sqrt(c)
        n = x.detach().norm(dim=-1).clamp(min=EPS)
        y = _c_term(y, x, torch.atanh((sc * n).clamp(max=1.0 - EPS)) / (sc * n))
    return y


def exp0(x, c):
    y = _Radial.apply(x, "exp0", _cf(c))
    if _c_grad(c):  # tanh(sqrt(c) n) / (sqrt(c) n), then project with a constant bound  (:76-95)
        sc = torch.sqrt(c)
        vn = x.detach().norm(dim=-1)
        n = vn.clamp(min=EPS)
        s = torch.tanh(sc * n) / (sc * n)
        pn = (s * vn).clamp(min=EPS)
        y = _c_term(y, x, s * pn.clamp(max=_mx(c)) / pn)
    return y


def project(x, c):
    return _Radial.apply(x, "project", _cf(c))


def apply_radius(x, radius, c):
    return _ApplyRadius.apply(x, radius, _cf(c))


def get_radius(x):
    return _Radius.apply(x)


def mobius_add(x, y, c):
    y = y.expand_as(x)
    out = _Mobius.apply(x, y, _cf(c))
    if _c_grad(c):  # out = p (a x + b y) / den, p the project factor of that row  (:118-143)
        xd, yd = x.detach(), y.detach()
        x2, y2, xy = (xd * xd).sum(-1), (yd * yd).sum(-1), (xd * yd).sum(-1)
        a = 1 + 2 * c * xy + c * y2
        b = 1 - c * x2
        den = 1 + 2 * c * xy + c * c * x2 * y2 + EPS
        rn = ((a * a * x2 + 2 * a * b * xy + b * b * y2).clamp(min=1e-30)).sqrt() / den.abs()
        pn = rn.clamp(min=EPS)
        pf = pn.clamp(max=_mx(c)) / pn
        out = _c_term(out, x, pf * a / den)
        out = _c_term(out, y, pf * b / den)
    return out


# ------------------------------------------------------------------------ edge aggregation
def _edge_desc(g, V, d, R2):
    wk = g.work()
    tr = g.transposed()
    a = _lib.EdgeBwdDesc()
    a.V, a.E, a.R2, a.d = V, int(wk["col_src"].shape[0]), R2, d
    for k in ("rowptr", "col_src", "col_type"):
        setattr(a, k, _lib.dptr(wk[k], torch.int32, k))
    for k in ("csr_dst", "sptr", "sp", "tptr", "tp"):
        setattr(a, k, _lib.dptr(tr[k], torch.int32, k))
    return a


class _UnionAggregate(torch.autograd.Function):
    """agg[v] = norm[v] sum_e w_e (x[src] + rel[type]), w_e = exp(-gamma |r_src - r_v|);
    rows without in-edges are 0 (DGL fn.sum zero fill)."""

    @staticmethod
    def forward(ctx, x, radius, rel, g, gamma):
        V, d = x.shape
        wk = g.work()
        x, radius, rel = x.contiguous(), radius.contiguous(), rel.contiguous()
        agg = torch.zeros_like(x)
        part = torch.empty(max(g.n_slots, 1), d, device=x.device, dtype=torch.float32)
        f, i = _lib.fptr, _lib.iptr
        _lib.call("regcn_union_aggregate_f32", f(x, "x"), f(radius, "radius"), f(rel, "rel"), i(wk["col_src"]),
                  i(wk["col_type"]), f(wk["norm"]), i(wk["chunks"]), wk["chunks"].shape[0], i(wk["fixups"]),
                  wk["fixups"].shape[0], float(gamma), d, f(part), d, f(agg), _lib.stream())
        ctx.save_for_backward(x, radius, rel)
        ctx.g, ctx.gamma = g, float(gamma)
        return agg

    @staticmethod
    def backward(ctx, G):
        x, radius, rel = ctx.saved_tensors
        V, d = x.shape
        R2 = rel.shape[0]
        a = _edge_desc(ctx.g, V, d, R2)
        E = a.E
        dx, drel = torch.empty_like(x), torch.empty_like(rel)
        dr = torch.empty_like(radius)
        scratch = torch.empty(2 * E + V, device=x.device, dtype=torch.float32)
        G = G.contiguous()
        a.x, a.radius, a.rel, a.norm, a.G = (_lib.fptr(t) for t in (x, radius, rel, ctx.g.work()["norm"], G))
        a.dx, a.drel, a.dradius, a.edge_scratch = (_lib.fptr(t) for t in (dx, drel, dr, scratch))
        _lib.check(_lib.lib().regcn_union_aggregate_bwd_f32(ctypes.byref(a), ctx.gamma, _lib.stream()),
                   "regcn_union_aggregate_bwd_f32")
        return dx, dr, drel, None, None


def union_aggregate(x, radius, rel, g, gamma):
    return _UnionAggregate.apply(x, radius, rel, g, gamma)


class _LorentzSum(torch.autograd.Function):
    """(S0[v], Sv[v]) = sum over v's in-edges of to_lorentz(exp0(blockdiag(W_t) x_src + rel_t))."""

    @staticmethod
    def forward(ctx, x, rel, W, g, nb, c):
        V, d = x.shape
        wk = g.work()
        x, rel, W = x.contiguous(), rel.contiguous(), W.contiguous()
        S0 = torch.empty(V, device=x.device, dtype=torch.float32)
        Sv = torch.empty_like(x)
        f, i = _lib.fptr, _lib.iptr
        _lib.call("regcn_lorentz_sum_raw_f32", f(x, "x"), f(rel, "rel"), f(W, "weight"), i(wk["rowptr"]),
                  i(wk["col_src"]), i(wk["col_type"]), V, d, int(nb), float(c), f(S0), f(Sv), _lib.stream())
        ctx.save_for_backward(x, rel, W)
        ctx.g, ctx.nb, ctx.c = g, int(nb), float(c)
        return S0, Sv

    @staticmethod
    def backward(ctx, g0, gv):
        x, rel, W = ctx.saved_tensors
        V, d = x.shape
        a = _edge_desc(ctx.g, V, d, rel.shape[0])
        g0 = torch.zeros(V, device=x.device) if g0 is None else g0.contiguous()
        gv = torch.zeros_like(x) if gv is None else gv.contiguous()
        dx, drel, dW = torch.empty_like(x), torch.empty_like(rel), torch.empty_like(W)
        a.x, a.rel, a.W, a.G, a.G0 = (_lib.fptr(t) for t in (x, rel, W, gv, g0))
        a.dx, a.drel, a.dW = (_lib.fptr(t) for t in (dx, drel, dW))
        _lib.check(_lib.lib().regcn_lorentz_aggregate_bwd_f32(ctypes.byref(a), ctx.nb, ctx.c, _lib.stream()),
                   "regcn_lorentz_aggregate_bwd_f32")
        return dx, drel, dW, None, None, None


def lorentz_sum(x, rel, W, g, nb, c):
    return _LorentzSum.apply(x, rel, W, g, nb, _cf(c))


def lorentz_aggregate(x, rel, W, g, nb, c):
    """LorentzRGCNLayer reduce + to_poincare + log0 (hyperbolic_layers.py:613-625, :669-670):
    the uniformly weighted Lorentz centroid is the normalised sum (scale-invariant: the
    reference's 1/deg weights cancel), rows without in-edges give 0."""
    cf = _cf(c)
    S0, Sv = lorentz_sum(x, rel, W, g, nb, cf)
    if Sv.shape[1] % 4 == 0 and Sv.shape[1] <= 256:
        y = _Centroid.apply(S0, Sv, cf)
    else:
        y = _centroid_torch(S0, Sv, cf)
    return log0(y, cf)


def _centroid_torch(S0, Sv, cf):
    ip = -S0 * S0 + (Sv * Sv).sum(-1)
    sc = torch.sqrt(torch.clamp(-ip * cf, min=EPS))
    c0 = S0 / sc
    return (Sv / sc.unsqueeze(-1)) / torch.clamp(1.0 + c0 * cf ** 0.5, min=EPS).unsqueeze(-1)


class _Centroid(torch.autograd.Function):
    """_centroid_torch in one row kernel forward and one backward (regcn_lorentz_centroid_f32)."""

    @staticmethod
    def forward(ctx, S0, Sv, cf):
        S0, Sv = S0.contiguous(), Sv.contiguous()
        y = torch.empty_like(Sv)
        f = _lib.fptr
        _lib.call("regcn_lorentz_centroid_f32", f(S0, "S0"), f(Sv, "Sv"), Sv.shape[0], Sv.shape[1], float(cf),
                  float(cf ** 0.5), None, f(y), None, None, _lib.stream())
        ctx.save_for_backward(S0, Sv)
        ctx.cf = cf
        return y

    @staticmethod
    def backward(ctx, gy):
        S0, Sv = ctx.saved_tensors
        dS0, dSv = torch.empty_like(S0), torch.empty_like(Sv)
        f = _lib.fptr
        _lib.call("regcn_lorentz_centroid_f32", f(S0), f(Sv), Sv.shape[0], Sv.shape[1], float(ctx.cf),
                  float(ctx.cf ** 0.5), f(gy.contiguous()), None, f(dS0), f(dSv), _lib.stream())
        return dS0, dSv, None


# ------------------------------------------------------------------------- cross entropy
class _HypCE(torch.autograd.Function):
    """Per-query CE loss of the proxy score S = scale (margin - |(-q) (+) e|^2) + bias."""

    @staticmethod
    def forward(ctx, q, cand, bias, scale, margin, target, c):
        B, d = q.shape
        N = cand.shape[0]
        q, cand = q.contiguous().float(), cand.contiguous().float()
        b = bias.contiguous().float() if bias is not None else None
        sc = scale.detach().reshape(1).float().contiguous()
        mg = margin.detach().reshape(1).float().contiguous()
        tgt = target.to(device=q.device, dtype=torch.int32).contiguous()
        ws = torch.empty((_lib.lib().regcn_hyp_ce_workspace_bytes(B, N) + 3) // 4, device=q.device)
        loss = torch.empty(B, device=q.device, dtype=torch.float32)
        lse = torch.empty(B, device=q.device, dtype=torch.float32)
        f = _lib.fptr
        _lib.call("regcn_hyp_ce_lse_f32", f(q, "query"), f(cand, "candidates"), f(b), f(sc), f(mg),
                  _lib.iptr(tgt, "target"), B, N, d, float(c), 0, f(ws), f(loss), f(lse), _lib.stream())
        ctx.save_for_backward(q, cand, b if b is not None else q.new_empty(0), sc, mg, tgt, lse)
        ctx.has_bias, ctx.c = b is not None, float(c)
        ctx.scale_shape, ctx.margin_shape = scale.shape, margin.shape
        return loss

    @staticmethod
    def backward(ctx, gl):
        q, cand, b, sc, mg, tgt, lse = ctx.saved_tensors
        B, d = q.shape
        N = cand.shape[0]
        nblk, ng = (N + 63) // 64, 8 * ((B + 127) // 128)
        coef = torch.empty(B, N, device=q.device, dtype=torch.float32)
        rsum = torch.empty(B, nblk, device=q.device, dtype=torch.float32)
        csum = torch.zeros(ng, N, 3, device=q.device, dtype=torch.float32)
        gl = gl.contiguous().float()
        f = _lib.fptr
        _lib.call("regcn_hyp_ce_bwd_f32", f(q), f(cand), f(b) if ctx.has_bias else None, f(sc), f(mg),
                  _lib.iptr(tgt), f(lse), f(gl), B, N, d, ctx.c, 0, f(coef), f(rsum), f(csum), _lib.stream())
        rs = rsum.sum(1, keepdim=True)
        cs = colsum(csum.reshape(ng, -1)).reshape(N, 3)
        dq = kreduce_mm(coef, cand, False, 2.0 * rs * q)            # coef E + 2 q sum_n G dS/d|q|^2
        de = kreduce_mm(coef, q, True, 2.0 * cs[:, :1] * cand)      # coef^T Q + 2 e sum_b G dS/d|e|^2
        dbias = cs[:, 1].clone() if ctx.has_bias else None
        dscale = cs[:, 2].sum().reshape(ctx.scale_shape)
        dmargin = (sc.reshape(()) * cs[:, 1].sum()).reshape(ctx.margin_shape)
        return dq, de, dbias, dscale, dmargin, None, None


def _const(v, like):
    """A device scalar from a python number by a fill kernel (no host-to-device copy, so a
    training step holding it stays capturable in a HIP graph)."""
    return torch.full((), float(v), device=like.device, dtype=torch.float32)


def _pair_terms(q, e, c):
    """Per pair (b, n): |project((-q_b) (+)_c e_n)|^2 from the per-pair scalars <q, e>, |q|^2,
    |e|^2 (float64; the bound of project a constant), with c a tensor."""
    xy = -(q @ e.t())
    x2 = (q * q).sum(1, keepdim=True)
    y2 = (e * e).sum(1).unsqueeze(0)
    a = 1 + 2 * c * xy + c * y2
    b = 1 - c * x2
    den = 1 + 2 * c * xy + c * c * x2 * y2 + EPS
    n2 = (a * a * x2 + 2 * a * b * xy + b * b * y2) / (den * den)
    pn = n2.clamp(min=1e-30).sqrt().clamp(min=EPS)
    pf = pn.clamp(max=_mx(c)) / pn
    return n2 * pf * pf


def _ce_c_term(q, cand, target, c, bias, scale, margin, chunk=65536, per_query=False):
    """Zero-valued term whose gradient is d(mean CE)/dc of the proxy score: sum_bn G_bn
    (S_bn(c) - S_bn(c).detach()) / B with G = softmax - one-hot from the same scores
    (per_query: the B per-query terms, without the 1 / B)."""
    qd, ed = q.detach().double(), cand.detach().double()
    cd = c.double()
    sc = scale.detach().double()
    mg = margin.detach().double()
    B, N = qd.shape[0], ed.shape[0]
    S = torch.empty(B, N, device=q.device, dtype=torch.float64)
    parts = []
    for n0 in range(0, N, chunk):
        n1 = min(N, n0 + chunk)
        Sc = sc * (mg - _pair_terms(qd, ed[n0:n1], cd))
        if bias is not None:
            Sc = Sc + bias.detach().double()[n0:n1]
        S[:, n0:n1] = Sc.detach()
        parts.append((n0, n1, Sc))
    G = torch.softmax(S, dim=1)
    G[torch.arange(B, device=q.device), target.long()] -= 1.0
    if per_query:
        return sum((G[:, n0:n1] * (Sc - Sc.detach())).sum(1) for n0, n1, Sc in parts).float()
    G /= B
    return sum((G[:, n0:n1] * (Sc - Sc.detach())).sum() for n0, n1, Sc in parts).float()


def hyp_ce_loss(q, cand, target, c, bias=None, scale=None, margin=None, reduction="mean"):
    """mean over queries of the CE loss (hyperbolic_decoder.py:182-307, proxy score);
    reduction="none": the per-query losses."""
    scale = scale if torch.is_tensor(scale) else _const(1.0 if scale is None else scale, q)
    margin = margin if torch.is_tensor(margin) else _const(0.0 if margin is None else margin, q)
    loss = _HypCE.apply(q, cand, bias, scale, margin, target, _cf(c))
    per_query = reduction == "none"
    if not per_query:
        loss = loss.mean()
    if _c_grad(c):
        loss = loss + _ce_c_term(q, cand, target, c, bias, scale, margin, per_query=per_query)
    return loss


def hyp_dist_ce_loss(q, cand, target, c_r, bias=None, scale=None, margin=None, reduction="mean"):
    """mean CE of the arctanh-distance score with per-query curvatures c_r
    (hyperbolic_decoder.py:257-283): logits = scale (margin - d_{c_r}(q, e)) + bias,
    d = 2 / (sqrt(c_r + eps) + eps) atanh(min(sqrt(c_r + eps) min(|n| / (den + eps), bound),
    1 - eps)).  Per-pair scalars in float64, autograd through q, e, c_r, bias, scale, margin."""
    qd, ed = q.double(), cand.double()
    c = c_r.double().reshape(-1, 1)
    sqrt_c = torch.sqrt(c + EPS)
    x2 = (qd * qd).sum(1, keepdim=True)
    y2 = (ed * ed).sum(1).unsqueeze(0)
    xy = qd @ ed.t()
    A = 1 - 2 * c * xy + c * y2  # num = A (-q) + B e
    Bc = 1 - c * x2
    num2 = A * A * x2 - 2 * A * Bc * xy + Bc * Bc * y2
    den = 1 - 2 * c * xy + c * c * x2 * y2
    n = (num2.clamp(min=1e-30).sqrt() / (den + EPS).abs()).clamp(min=EPS)
    n = torch.min(n, 1.0 / (sqrt_c + EPS) - EPS)
    dist = (2.0 / (sqrt_c + EPS)) * torch.atanh((sqrt_c * n).clamp(max=1.0 - EPS))
    logits = margin.double() - dist if torch.is_tensor(margin) else (0.0 if margin is None else margin) - dist
    if scale is not None:
        logits = scale.double() * logits
    if bias is not None:
        logits = logits + bias.double()
    return torch.nn.functional.cross_entropy(logits, target.long(), reduction=reduction).float()


# ------------------------------------------------------------------ long-K products
@functools.lru_cache(maxsize=4096)
def _kreduce_ws(K, M, N):
    return max(1, _lib.lib().regcn_kreduce_workspace_floats(K, M, N))


def kreduce_mm(a, b, a_kmajor, c0=None, b_kmajor=True):
    """(a^T if a_kmajor else a) @ (b if b_kmajor else b^T) (+ c0: M x N, or a length-N bias
    row) on regcn_kreduce_gemm_f32: K split over workgroups, partials summed in a fixed order.
    a: K x M (a_kmajor) or M x K; b: K x N (b_kmajor) or N x K; fp32."""
    a, b = a.contiguous().float(), b.contiguous().float()
    K = a.shape[0] if a_kmajor else a.shape[1]
    M = a.shape[1] if a_kmajor else a.shape[0]
    N = b.shape[1] if b_kmajor else b.shape[0]
    if (b.shape[0] if b_kmajor else b.shape[1]) != K:
        raise ValueError(f"kreduce_mm: a {tuple(a.shape)} does not match b {tuple(b.shape)}")
    out = torch.empty(M, N, device=b.device, dtype=torch.float32)
    c0_ld = 0
    if c0 is not None:
        c0 = c0.contiguous().float()
        if c0.dim() == 1 and c0.shape[0] == N:
            c0_ld = 0
        elif tuple(c0.shape) == (M, N):
            c0_ld = N
        else:
            c0, c0_ld = c0.expand(M, N).contiguous(), N
    ws = torch.empty(_kreduce_ws(K, M, N), device=b.device, dtype=torch.float32)
    f = _lib.fptr
    _lib.call("regcn_kreduce_gemm_f32", f(a, "a"), 1 if a_kmajor else 0, f(b, "b"), 1 if b_kmajor else 0, K, M, N,
              f(c0), c0_ld, f(out), f(ws), _lib.stream())
    return out


def colsum(x):
    """x.sum(0) of a 2-D fp32 device tensor on regcn_kreduce_gemm_f32 (ones^T x: K = rows split
    over workgroups, partials summed by a second launch in a fixed order).  torch's column sum
    of a tall matrix finishes in the kernel's last workgroup after an atomic ticket, reading
    the other workgroups' partials through the XCDs' separate L2s; in replayed HIP graphs it
    returned different sums for the same input (tools/graphdbg3.py: the time-gate bias
    gradient), so the training backward sums columns here."""
    x = x.contiguous().float()
    ones = torch.ones(x.shape[0], 1, device=x.device, dtype=torch.float32)
    return kreduce_mm(ones, x, True).reshape(x.shape[1])


class _Linear(torch.autograd.Function):
    """F.linear(x, W, bias) for a mini-batch of query rows: y = x W^T + bias, dx = dy W,
    dW = dy^T x, dbias = sum dy, all three products on regcn_kreduce_gemm_f32."""

    @staticmethod
    def forward(ctx, x, w, bias):
        x = x.contiguous()
        ctx.save_for_backward(x, w)
        ctx.has_bias = bias is not None
        return kreduce_mm(x, w, False, bias, b_kmajor=False)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = kreduce_mm(gy, w, False) if ctx.needs_input_grad[0] else None
        gw = kreduce_mm(gy, x, True) if ctx.needs_input_grad[1] else None
        gb = colsum(gy) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return gx, gw, gb


def linear(layer, x):
    """layer(x) for an nn.Linear on 2-D fp32 CUDA rows (the decoders' projections,
    hyperbolic_decoder.py:212-321), on the split-K kernel; anything else goes to the layer."""
    if (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and layer.weight.dtype == torch.float32
            and torch.is_grad_enabled()):
        return _Linear.apply(x, layer.weight, layer.bias)
    return layer(x)


class _RowsByWeight(torch.autograd.Function):
    """x (V x d_in) @ W (d_in x d_out): forward and the input gradient dy W^T are library GEMMs
    (large M, short K); the weight gradient x^T dy (K = V) runs on regcn_kreduce_gemm_f32."""

    @staticmethod
    def forward(ctx, x, w):
        x = x.contiguous()
        ctx.save_for_backward(x, w)
        return torch.mm(x, w)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = torch.mm(gy, w.t()) if ctx.needs_input_grad[0] else None
        gw = kreduce_mm(x, gy, True) if ctx.needs_input_grad[1] else None
        return gx, gw


def mm_weight(x, w):
    """torch.mm(x, w) for the training path's (V x d) @ (d x d) products (hyperbolic_layers.py
    self/evolve loop :273-280, neighbour weight :290, skip gate :315-318; hyperbolic_model.py
    time gate :852-858), with the weight gradient on the split-K kernel."""
    if x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() == 2 and w.dim() == 2:
        return _RowsByWeight.apply(x, w)
    return torch.mm(x, w)


# ------------------------------------------------------------------ fused layer tail / gate
TAIL_CLAMP_IN, TAIL_CLAMP_OUT, TAIL_LEAKY = 1, 2, 4


def _tail_torch(agg, loop, pos, z, bias, p, flags, slope):
    """The op-by-op composition regcn_tail_f32 fuses (used where the kernel does not apply)."""
    a = torch.clamp(agg, -10.0, 10.0) if flags & TAIL_CLAMP_IN else agg
    if loop is not None:
        d = agg.shape[1]
        a = a + torch.where(pos.bool().unsqueeze(-1), loop[:, :d], loop[:, d:])
    if z is not None:
        g = torch.sigmoid(z + bias if bias is not None else z)
        a = g * a + (1 - g) * p
    if flags & TAIL_CLAMP_OUT:
        a = torch.clamp(a, -10.0, 10.0)
    if flags & TAIL_LEAKY:
        a = torch.nn.functional.leaky_relu(a, slope)
    return a


def _halves(t, d):
    """(first, second) half-row pointers of a V x 2d tensor (None -> None, None)."""
    if t is None:
        return None, None
    base = _lib.addr(t)
    return ctypes.c_void_p(base), ctypes.c_void_p(base + 4 * d)


class _Tail(torch.autograd.Function):
    @staticmethod
    def forward(ctx, agg, loop, z, bias, p, pos, flags, slope):
        agg = agg.contiguous()
        d = agg.shape[1]
        loop = loop.contiguous() if loop is not None else None
        z, p = (z.contiguous(), p.contiguous()) if z is not None else (None, None)
        bias = bias.contiguous() if bias is not None else None
        out = torch.empty_like(agg)
        f = _lib.fptr
        lx, ex = _halves(loop, d)
        _lib.call("regcn_tail_f32", f(agg, "agg"), lx, ex, 2 * d, _lib.dptr(pos, torch.uint8, "pos"), f(z), f(bias),
                  f(p), agg.shape[0], d, flags, float(slope), None, f(out), None, None, None, None, None, _lib.stream())
        ctx.save_for_backward(agg, loop, z, bias, p, pos)
        ctx.flags, ctx.slope = flags, slope
        return out

    @staticmethod
    def backward(ctx, gy):
        agg, loop, z, bias, p, pos = ctx.saved_tensors
        d = agg.shape[1]
        gy = gy.contiguous()
        need = ctx.needs_input_grad
        dagg = torch.empty_like(agg) if need[0] else None
        dloop = torch.empty_like(loop) if loop is not None and need[1] else None
        dz = torch.empty_like(z) if z is not None and (need[2] or need[3]) else None
        dp = torch.empty_like(p) if p is not None and need[4] else None
        f = _lib.fptr
        lx, ex = _halves(loop, d)
        dlx, dex = _halves(dloop, d)
        _lib.call("regcn_tail_f32", f(agg), lx, ex, 2 * d, _lib.dptr(pos, torch.uint8), f(z), f(bias), f(p),
                  agg.shape[0], d, ctx.flags, float(ctx.slope), f(gy), None, f(dagg), dlx, dex, f(dz), f(dp),
                  _lib.stream())
        dbias = colsum(dz) if bias is not None and need[3] else None
        return dagg, dloop, dz if need[2] else None, dbias, dp, None, None, None


def tail(agg, loop=None, pos=None, z=None, bias=None, p=None, flags=0, slope=0.0):
    """clamp_in -> + (pos ? loop[:, :d] : loop[:, d:]) -> sigmoid(z + bias) gate with p ->
    clamp_out -> leaky, one HIP launch forward and one backward (regcn_tail_f32).
    loop: V x 2d, the product x [W_loop | W_evolve]; pos: uint8 per row."""
    ts = [t for t in (agg, loop, z, bias, p) if t is not None]
    if (agg.is_cuda and agg.dim() == 2 and agg.shape[1] % 4 == 0
            and all(t.dtype == torch.float32 for t in ts)):
        return _Tail.apply(agg, loop, z, bias, p, pos, flags, slope)
    return _tail_torch(agg, loop, pos, z, bias, p, flags, slope)


# ------------------------------------------------------------------ Givens rotation
class _Givens(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, angles, reflect):
        x, angles = x.contiguous(), angles.contiguous()
        out = torch.empty_like(x)
        f = _lib.fptr
        _lib.call("regcn_givens_rotation_f32", f(x, "x"), f(angles, "angles"), angles.numel(), int(reflect), None,
                  f(out), None, None, _lib.stream())
        ctx.save_for_backward(x, angles)
        ctx.reflect = int(reflect)
        return out

    @staticmethod
    def backward(ctx, gy):
        x, angles = ctx.saved_tensors
        dx, da = torch.empty_like(x), torch.empty_like(angles)
        f = _lib.fptr
        _lib.call("regcn_givens_rotation_f32", f(x), f(angles), angles.numel(), ctx.reflect, f(gy.contiguous()), None,
                  f(dx), f(da), _lib.stream())
        return dx, da, None


def givens_rotation(x, angles, reflect=False):
    """hyperbolic_decoder.py:1032-1051 (rotation) / :1392-1401 (reflection, reflect=True) of
    interleaved pairs as one launch each way (regcn_givens_rotation_f32) for B x d rows with
    B x d/2 angles; None otherwise."""
    if (x.is_cuda and x.dim() == 2 and angles.dim() == 2 and x.dtype == torch.float32
            and angles.dtype == torch.float32 and tuple(angles.shape) == (x.shape[0], x.shape[1] // 2)
            and x.shape[1] % 2 == 0):
        return _Givens.apply(x, angles, reflect)
    return None


def batch_norm(bn, x):
    """bn(x) (src/decoder.py's BatchNorm1d).  In eval mode through torch's native batch-norm
    kernel instead of MIOpen's: MIOpenBatchNormFwdInferSpatialEst took ~140 us per call at the
    ConvTransE / ConvTransR shapes, a third of the RE-GCN leg's kernel time
    (profiles/r6_regcn_leg_kernel_stats.csv); the native kernel computes the same
    (x - mean) / sqrt(var + eps) * weight + bias."""
    if bn.training or torch.is_grad_enabled() or not x.is_cuda:
        return bn(x)
    return torch.native_batch_norm(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, False, 0.0, bn.eps)[0]
