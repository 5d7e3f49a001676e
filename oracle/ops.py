"""Poincaré / Lorentz row operations restated (oracle; test infrastructure only).

Follows hyperbolic_src/hyperbolic_ops.py.  `c` is a python float.
All functions operate row-wise over the last dimension in fp32 torch (CPU).
"""
import math

import torch

EPS = 1e-6


def clamp_norm(x, max_norm, eps=EPS):
    """hyperbolic_ops.py:37-53 (norm clamp min eps, max max_norm - eps)."""
    norm = torch.norm(x, p=2, dim=-1, keepdim=True).clamp(min=eps)
    return x * (torch.clamp(norm, max=max_norm - eps) / norm)


def project(x, c, eps=EPS):
    """hyperbolic_ops.py:55-74: max_norm = 1/sqrt(c) - eps, then clamp_norm."""
    return clamp_norm(x, 1.0 / math.sqrt(c) - eps, eps)


def exp0(v, c, eps=EPS):
    """hyperbolic_ops.py:76-95: tanh(sqrt(c)|v|) v/(sqrt(c)|v|), then project."""
    sc = math.sqrt(c)
    n = torch.norm(v, p=2, dim=-1, keepdim=True).clamp(min=eps)
    return project(torch.tanh(sc * n) * (v / n) / sc, c, eps)


def log0(x, c, eps=EPS):
    """hyperbolic_ops.py:97-116: atanh(min(sqrt(c)|x|, 1-eps)) x/(sqrt(c)|x|)."""
    sc = math.sqrt(c)
    n = torch.norm(x, p=2, dim=-1, keepdim=True).clamp(min=eps)
    return torch.atanh((sc * n).clamp(max=1.0 - eps)) * x / (sc * n)


def mobius_add(x, y, c, eps=EPS):
    """hyperbolic_ops.py:118-143 (denominator + eps, then project)."""
    x2 = torch.sum(x * x, dim=-1, keepdim=True)
    y2 = torch.sum(y * y, dim=-1, keepdim=True)
    xy = torch.sum(x * y, dim=-1, keepdim=True)
    num = (1 + 2 * c * xy + c * y2) * x + (1 - c * x2) * y
    den = 1 + 2 * c * xy + c * c * x2 * y2
    return project(num / (den + eps), c, eps)


def hyperbolic_distance(x, y, c, eps=EPS):
    """hyperbolic_ops.py:168-191."""
    sc = math.sqrt(c)
    diff = mobius_add(-x, y, c, eps)
    n = torch.norm(diff, p=2, dim=-1).clamp(min=eps, max=1.0 / (sc + eps) - eps)
    return (2 / sc) * torch.atanh(sc * n)


def get_radius(x, eps=EPS):
    """hyperbolic_ops.py:193-206."""
    return torch.norm(x, p=2, dim=-1).clamp(min=eps)


def apply_radius(x, radius, c, eps=EPS):
    """hyperbolic_ops.py:208-233: direction * clamp(r, eps, 1/sqrt(c) - eps)."""
    r = radius if radius.dim() == x.dim() else radius.unsqueeze(-1)
    r = r.clamp(min=eps, max=1.0 / math.sqrt(c) - eps)
    n = torch.norm(x, p=2, dim=-1, keepdim=True).clamp(min=eps)
    return (x / n) * r


def to_lorentz(x, c, eps=EPS):
    """hyperbolic_ops.py:476-499."""
    sc = math.sqrt(c)
    x2 = torch.sum(x ** 2, dim=-1, keepdim=True)
    den = (1.0 - c * x2).clamp(min=eps)
    return torch.cat([(1.0 + c * x2) / (sc * den), 2.0 * x / den], dim=-1)


def to_poincare(y, c, eps=EPS):
    """hyperbolic_ops.py:501-518."""
    return y[..., 1:] / (1.0 + y[..., :1] * math.sqrt(c)).clamp(min=eps)


def lorentz_inner(x, y, keepdim=False):
    """hyperbolic_ops.py:459-474."""
    return (-torch.sum(x[..., :1] * y[..., :1], dim=-1, keepdim=keepdim)
            + torch.sum(x[..., 1:] * y[..., 1:], dim=-1, keepdim=keepdim))


def lorentz_centroid(emb, w, c, eps=EPS):
    """hyperbolic_ops.py:562-581 (weights renormalised, then projected so <x,x>_L=-1/c)."""
    w = w / (w.sum() + eps)
    cen = torch.sum(w.unsqueeze(-1) * emb, dim=0)
    ip = lorentz_inner(cen, cen, keepdim=True)
    return cen / torch.sqrt(torch.clamp(-ip * c, min=eps))


def leaky(x):
    """F.rrelu called as activation(x) (training=False): slope (1/8 + 1/3)/2 = 11/48
    (hyperbolic_model.py:120, hyperbolic_layers.py:715, src/rrgcn.py:16)."""
    return torch.where(x >= 0, x, x * ((1.0 / 8 + 1.0 / 3) / 2))
