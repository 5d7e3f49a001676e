"""Poincaré-ball / Lorentz operations on HIP (mirror of hyperbolic_src/hyperbolic_ops.py).

Same class names, method names, argument meaning and defaults as the reference; every
method runs a hand-written gfx950 kernel (csrc/rowwise.hip) through the C-ABI.  Inputs
must be fp32 HIP tensors; `c` may be a python float or a 0-dim tensor (read once, as the
reference's `c.item()` does at hyperbolic_ops.py:72).  With autograd on (or a learned
curvature tensor that requires grad), the row maps route to autograd.py (HIP backward
kernels, the curvature's gradient where the reference has one); these are the
inference/forward row maps of the hot path.
"""
import math

import torch
import torch.nn as nn

from . import _lib
from . import autograd as _ag

EPS = 1e-6


def _cf(c):
    return float(c.item()) if torch.is_tensor(c) else float(c)


def _rows(x):
    d = x.shape[-1]
    return x.reshape(-1, d).contiguous(), d


def _rowmap(name, x, c, *extra_before, out_shape=None):
    x2, d = _rows(x)
    out = torch.empty(out_shape if out_shape is not None else x2.shape, device=x.device, dtype=torch.float32)
    _lib.call(name, _lib.fptr(x2, "x"), *extra_before, x2.shape[0], d, _cf(c), _lib.fptr(out), _lib.stream())
    return out


class HyperbolicOps:
    """hyperbolic_ops.py:22-305."""

    EPS = EPS

    @staticmethod
    def _sqrt_curvature(c):
        return torch.sqrt(c) if torch.is_tensor(c) else math.sqrt(c)

    @staticmethod
    def project_to_ball(x, c=0.01, eps=1e-6):
        """hyperbolic_ops.py:55-74."""
        _check_eps(eps)
        if _ag.needs_grad(x, c):
            return _ag.project(x, c)
        return _rowmap("regcn_project_f32", x, c).view(x.shape)

    @staticmethod
    def exp_map_zero(v, c=0.01, eps=1e-6):
        """hyperbolic_ops.py:76-95."""
        _check_eps(eps)
        if _ag.needs_grad(v, c):
            return _ag.exp0(v, c)
        return _rowmap("regcn_exp0_f32", v, c).view(v.shape)

    @staticmethod
    def log_map_zero(x, c=0.01, eps=1e-6):
        """hyperbolic_ops.py:97-116."""
        _check_eps(eps)
        if _ag.needs_grad(x, c):
            return _ag.log0(x, c)
        return _rowmap("regcn_log0_f32", x, c).view(x.shape)

    @staticmethod
    def mobius_add(x, y, c=0.01, eps=1e-6):
        """hyperbolic_ops.py:118-143."""
        _check_eps(eps)
        if _ag.needs_grad(x, y, c):
            return _ag.mobius_add(x, y, c)
        x2, d = _rows(x)
        y2, _ = _rows(y.expand_as(x))
        out = torch.empty_like(x2)
        _lib.call("regcn_mobius_add_f32", _lib.fptr(x2, "x"), _lib.fptr(y2, "y"), x2.shape[0], d, _cf(c),
                  _lib.fptr(out), _lib.stream())
        return out.view(x.shape)

    @staticmethod
    def get_radius(x, eps=1e-6):
        """hyperbolic_ops.py:193-206."""
        _check_eps(eps)
        if _ag.needs_grad(x):
            return _ag.get_radius(x)
        x2, d = _rows(x)
        out = torch.empty(x2.shape[0], device=x.device, dtype=torch.float32)
        _lib.call("regcn_radius_f32", _lib.fptr(x2, "x"), x2.shape[0], d, _lib.fptr(out), _lib.stream())
        return out.view(x.shape[:-1])

    @staticmethod
    def apply_radius(x, radius, c=0.01, eps=1e-6):
        """hyperbolic_ops.py:208-233."""
        if radius is None:
            return x
        _check_eps(eps)
        if _ag.needs_grad(x, radius, c):
            r = radius.reshape(-1)
            n = x.reshape(-1, x.shape[-1]).shape[0]
            return _ag.apply_radius(x, r.expand(n) if r.numel() == 1 else r, c)
        x2, d = _rows(x)
        r = radius.reshape(-1).expand(x2.shape[0]).contiguous().float() if radius.numel() in (1, x2.shape[0]) \
            else radius.reshape(-1).contiguous()
        out = torch.empty_like(x2)
        _lib.call("regcn_apply_radius_f32", _lib.fptr(x2, "x"), _lib.fptr(r, "radius"), x2.shape[0], d, _cf(c),
                  _lib.fptr(out), _lib.stream())
        return out.view(x.shape)

    @staticmethod
    def hyperbolic_distance(x, y, c=0.01, eps=1e-6):
        """hyperbolic_ops.py:168-191: 2/sqrt(c) atanh(sqrt(c) |(-x) (+) y|) with the reference clamps."""
        sc = math.sqrt(_cf(c))
        diff = HyperbolicOps.mobius_add(-x, y, c, eps)
        n = HyperbolicOps.get_radius(diff).clamp(max=1.0 / (sc + eps) - eps)
        return (2 / sc) * torch.atanh(sc * n)

    @staticmethod
    def mobius_matvec(M, x, c=0.01, eps=1e-6):
        """hyperbolic_ops.py:145-166."""
        return HyperbolicOps.exp_map_zero(torch.nn.functional.linear(HyperbolicOps.log_map_zero(x, c, eps), M), c, eps)

    @staticmethod
    def layer_norm_roundtrip(x, c=0.01):
        """exp0(normalize(log0(x))) in one pass (hyperbolic_model.py:832-835, :926-929)."""
        if _ag.needs_grad(x, c):
            return _ag.exp0(torch.nn.functional.normalize(_ag.log0(x, c)), c)
        return _rowmap("regcn_ln_roundtrip_f32", x, c).view(x.shape)

    @staticmethod
    def log_embedding_stats(x, name="embeddings", c=0.01):
        """hyperbolic_ops.py:235-269: norm statistics of `x` as a host dict (the reference's own
        return value; one device read).  The model keeps them on the device instead
        (analysis.log_embedding)."""
        from .analysis import embedding_dict, embedding_stats
        with torch.no_grad():
            return embedding_dict(embedding_stats(HyperbolicOps.get_radius(x), _cf(c)), name, _cf(c))

    @staticmethod
    def sumsq(x):
        x2, d = _rows(x)
        out = torch.empty(x2.shape[0], device=x.device, dtype=torch.float32)
        _lib.call("regcn_sumsq_f32", _lib.fptr(x2, "x"), x2.shape[0], d, _lib.fptr(out), _lib.stream())
        return out.view(x.shape[:-1])


def _check_eps(eps):
    if eps != EPS:
        raise ValueError("the HIP kernels implement eps=1e-6 (the reference default); got %r" % (eps,))


class LorentzOps:
    """hyperbolic_ops.py:442-598 (the maps used on the lgcn path)."""

    EPS = EPS

    @staticmethod
    def to_lorentz(x, c=0.01, eps=1e-6):
        """hyperbolic_ops.py:476-499."""
        _check_eps(eps)
        x2, d = _rows(x)
        out = torch.empty(x2.shape[0], d + 1, device=x.device, dtype=torch.float32)
        _lib.call("regcn_to_lorentz_f32", _lib.fptr(x2, "x"), x2.shape[0], d, _cf(c), _lib.fptr(out), _lib.stream())
        return out.view(*x.shape[:-1], d + 1)

    @staticmethod
    def to_poincare(y, c=0.01, eps=1e-6):
        """hyperbolic_ops.py:501-518."""
        _check_eps(eps)
        y2 = y.reshape(-1, y.shape[-1]).contiguous()
        d = y2.shape[1] - 1
        out = torch.empty(y2.shape[0], d, device=y.device, dtype=torch.float32)
        _lib.call("regcn_to_poincare_f32", _lib.fptr(y2, "y"), y2.shape[0], d, _cf(c), _lib.fptr(out), _lib.stream())
        return out.view(*y.shape[:-1], d)

    @staticmethod
    def inner_product(x, y, keepdim=False):
        """hyperbolic_ops.py:459-474."""
        return (-torch.sum(x[..., :1] * y[..., :1], dim=-1, keepdim=keepdim)
                + torch.sum(x[..., 1:] * y[..., 1:], dim=-1, keepdim=keepdim))

    @staticmethod
    def lorentz_centroid(embeddings, weights, c=0.01, eps=1e-6):
        """hyperbolic_ops.py:562-581 (single-set form; the per-destination centroid of the
        hot path is fused into regcn_lorentz_aggregate_f32)."""
        w = weights / (weights.sum() + eps)
        cen = torch.sum(w.unsqueeze(-1) * embeddings, dim=0)
        ip = LorentzOps.inner_product(cen, cen, keepdim=True)
        return cen / torch.sqrt(torch.clamp(-ip * _cf(c), min=eps))


class TemporalRadiusEvolution(nn.Module):
    """hyperbolic_ops.py:364-439.  Parameters and state_dict keys match the reference
    (`radius_mlp.weight` (1, d), `radius_mlp.bias` (1,)).  In the model the whole
    evolution is fused into regcn_timestep_f32; this standalone forward composes the
    row kernels."""

    def __init__(self, dim, c=0.01, epsilon=0.1, anchor_beta=1.0):
        super().__init__()
        if anchor_beta < 0.0 or anchor_beta > 1.0:
            raise ValueError("anchor_beta must be in [0, 1]")
        self.dim, self.c, self.epsilon, self.anchor_beta = dim, c, epsilon, float(anchor_beta)
        self.radius_mlp = nn.Linear(dim, 1)
        nn.init.xavier_uniform_(self.radius_mlp.weight, gain=0.1)
        nn.init.zeros_(self.radius_mlp.bias)
        self.last_evolution_stats = None

    # The statistics of the last evolution (hyperbolic_ops.py:426-434) are kept as one device
    # vector (analysis.evolution_terms) and read on the host when looked at.
    @property
    def last_evolution_stats(self):
        from .analysis import evolution_dict
        return evolution_dict(self.__dict__.get("_ev"))

    @last_evolution_stats.setter
    def last_evolution_stats(self, ev):
        self.__dict__["_ev"] = ev

    def forward(self, x, static_radius):
        from .analysis import evolution_terms
        t = HyperbolicOps.log_map_zero(x, self.c)
        delta = torch.clamp(self.radius_mlp(t).squeeze(-1), -self.epsilon, self.epsilon)
        dyn = HyperbolicOps.get_radius(x)
        st = dyn if static_radius is None else static_radius
        base = self.anchor_beta * st + (1.0 - self.anchor_beta) * dyn
        self.last_evolution_stats = evolution_terms(delta, dyn, base, st, self.anchor_beta, self.epsilon)
        return HyperbolicOps.apply_radius(x, base + delta, self.c)

    def get_evolution_stats(self):
        """hyperbolic_ops.py:437-439 (a host dict; one device read)."""
        return self.last_evolution_stats
