"""Hyperbolic message-passing layers on HIP (mirror of hyperbolic_src/hyperbolic_layers.py).

Constructor arguments, parameter names/shapes (hence state_dict keys) and forward
signatures follow the reference; forward runs three gfx950 kernels per layer:
  1. row prologue x = log0(h), r = |h| (skipped when the producer already emitted them);
  2. CSR gather + segment reduce (csrc/aggregate.hip);
  3. MFMA layer tail: neighbour/self-loop/skip GEMMs + clamp/rrelu/dropout/exp0 and the
     next layer's prologue, fused (csrc/rowgemm.hip).
Forward only (no autograd); FHNN/HGAT encoders are outside this build's scope.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .tangent import attach, tangent_of
from .weights import packed

EPS = 1e-6


def _drop_mask(layer, like):
    if layer.dropout is None or not layer.training:
        return None
    p = layer.dropout.p
    return torch.empty_like(like).bernoulli_(1.0 - p).div_(1.0 - p)


def layer_tail(agg, w_n, x, w_loop, w_evolve, prev_t, w_skip, b_skip, drop_mask, g, c, euclid):
    """regcn_layer_tail_f32 wrapper (weights as (d, d) tensors, packed on first use);
    returns (h, x_next, r_next)."""
    wk = g.work()
    V, d = x.shape
    h = torch.empty_like(x)
    xn = torch.empty_like(x)
    rn = torch.empty(V, device=x.device, dtype=torch.float32)
    f = _lib.fptr
    w_n, w_loop, w_evolve, w_skip = packed(w_n), packed(w_loop), packed(w_evolve), packed(w_skip)
    _lib.call("regcn_layer_tail_f32", f(agg), f(w_n), f(x, "x"), f(w_loop), f(w_evolve), f(prev_t), f(w_skip),
              f(b_skip), f(drop_mask), _lib.iptr(wk["rows"]), g.n_pos, V, d, int(euclid), float(c), f(h), f(xn),
              f(rn), _lib.stream())
    return h, xn, rn


def _partial(g, d, device, lorentz=False):
    if g.n_slots == 0:
        return None, 0
    stride = (d + 4) if lorentz else d
    return torch.empty(g.n_slots, stride, device=device, dtype=torch.float32), stride


class HyperbolicUnionRGCNLayer(nn.Module):
    """hyperbolic_layers.py:164-323 (encoder `hyperbolic_uvrgcn`)."""

    def __init__(self, in_feat, out_feat, num_rels, num_bases=-1, c=0.01, activation=None, self_loop=False,
                 dropout=0.0, skip_connect=False, radius_msg_gamma=1.0):
        super().__init__()
        if in_feat != out_feat:
            raise ValueError("HyperbolicUnionRGCNLayer needs in_feat == out_feat")
        if activation not in (None, F.rrelu):
            raise ValueError("only the reference activation (F.rrelu, deterministic slope 11/48) is fused")
        self.in_feat, self.out_feat, self.num_rels, self.c = in_feat, out_feat, num_rels, c
        self.activation, self.self_loop, self.skip_connect = activation, self_loop, skip_connect
        self.rel_emb = None
        self.radius_msg_gamma = radius_msg_gamma
        self.weight_neighbor = nn.Parameter(torch.Tensor(in_feat, out_feat))
        nn.init.xavier_uniform_(self.weight_neighbor, gain=nn.init.calculate_gain("relu"))
        if self_loop:
            self.loop_weight = nn.Parameter(torch.Tensor(in_feat, out_feat))
            nn.init.xavier_uniform_(self.loop_weight, gain=nn.init.calculate_gain("relu"))
            self.evolve_loop_weight = nn.Parameter(torch.Tensor(in_feat, out_feat))
            nn.init.xavier_uniform_(self.evolve_loop_weight, gain=nn.init.calculate_gain("relu"))
        if skip_connect:
            self.skip_weight = nn.Parameter(torch.Tensor(out_feat, out_feat))
            nn.init.xavier_uniform_(self.skip_weight, gain=nn.init.calculate_gain("relu"))
            self.skip_bias = nn.Parameter(torch.zeros(out_feat))
        self.dropout = nn.Dropout(dropout) if dropout > 0 else None

    def forward(self, g, h_hyper, rel_emb, prev_h=None):
        """hyperbolic_layers.py:242-323."""
        if self.activation is None:
            raise NotImplementedError("the fused tail applies rrelu; activation=None is not supported")
        self.rel_emb = rel_emb
        c = float(self.c)
        x, r = tangent_of(h_hyper, c)
        wk = g.work()
        V, d = x.shape
        agg = torch.empty_like(x)
        part, stride = _partial(g, d, x.device)
        ch, fx = wk["chunks"], wk["fixups"]
        _lib.call("regcn_union_aggregate_f32", _lib.fptr(x), _lib.fptr(r), _lib.fptr(rel_emb.contiguous(), "rel_emb"),
                  _lib.iptr(wk["col_src"]), _lib.iptr(wk["col_type"]), _lib.fptr(wk["norm"]), _lib.iptr(ch),
                  ch.shape[0], _lib.iptr(fx), fx.shape[0], float(self.radius_msg_gamma), d, _lib.fptr(part), stride,
                  _lib.fptr(agg), _lib.stream())
        prev_t = None
        if self.skip_connect and prev_h is not None:
            prev_t = tangent_of(prev_h, c)[0]
        wl = self.loop_weight if self.self_loop else None
        we = self.evolve_loop_weight if self.self_loop else None
        h, xn, rn = layer_tail(agg, self.weight_neighbor, x, wl, we, prev_t,
                               self.skip_weight if prev_t is not None else None,
                               self.skip_bias if prev_t is not None else None,
                               _drop_mask(self, x), g, c, euclid=False)
        return attach(h, xn, rn, c)


class LorentzRGCNLayer(nn.Module):
    """hyperbolic_layers.py:524-694 (encoder `lgcn`)."""

    def __init__(self, in_feat, out_feat, num_rels, num_bases=-1, c=0.01, activation=None, self_loop=False,
                 dropout=0.0, skip_connect=False):
        super().__init__()
        if in_feat != out_feat:
            raise ValueError("LorentzRGCNLayer needs in_feat == out_feat")
        if activation not in (None, F.rrelu):
            raise ValueError("only the reference activation (F.rrelu) is fused")
        self.in_feat, self.out_feat, self.num_rels = in_feat, out_feat, num_rels
        self.num_bases = num_bases if num_bases > 0 else num_rels
        if self.num_bases > self.num_rels:
            self.num_bases = self.num_rels
        self.c, self.activation, self.self_loop, self.skip_connect = c, activation, self_loop, skip_connect
        self.submat_in = in_feat // self.num_bases
        self.submat_out = out_feat // self.num_bases
        self.weight = nn.Parameter(torch.Tensor(self.num_rels, self.num_bases * self.submat_in * self.submat_out))
        nn.init.xavier_uniform_(self.weight, gain=nn.init.calculate_gain("relu"))
        if self_loop:
            self.loop_weight = nn.Parameter(torch.Tensor(in_feat, out_feat))
            nn.init.xavier_uniform_(self.loop_weight, gain=nn.init.calculate_gain("relu"))
            self.evolve_loop_weight = nn.Parameter(torch.Tensor(in_feat, out_feat))
            nn.init.xavier_uniform_(self.evolve_loop_weight, gain=nn.init.calculate_gain("relu"))
        if skip_connect:
            self.skip_weight = nn.Parameter(torch.Tensor(out_feat, out_feat))
            nn.init.xavier_uniform_(self.skip_weight, gain=nn.init.calculate_gain("relu"))
            self.skip_bias = nn.Parameter(torch.zeros(out_feat))
        self.dropout = nn.Dropout(dropout) if dropout > 0 else None
        self.rel_emb = None

    def forward(self, g, h_hyper, rel_emb=None, prev_h=None):
        """hyperbolic_layers.py:627-694."""
        if self.activation is None:
            raise NotImplementedError("the fused tail applies rrelu; activation=None is not supported")
        if self.submat_in * self.num_bases != self.in_feat:
            # the reference's view(-1, 1, submat_in) fails on this shape too
            raise RuntimeError("in_feat=%d is not divisible by num_bases=%d" % (self.in_feat, self.num_bases))
        self.rel_emb = rel_emb
        c = float(self.c)
        x, _ = tangent_of(h_hyper, c)
        wk = g.work()
        V, d = x.shape
        rel = rel_emb[:, :d].contiguous() if rel_emb is not None else \
            torch.zeros(self.num_rels, d, device=x.device, dtype=torch.float32)
        agg = torch.empty_like(x)
        part, stride = _partial(g, d, x.device, lorentz=True)
        ch, fx = wk["chunks"], wk["fixups"]
        _lib.call("regcn_lorentz_aggregate_f32", _lib.fptr(x), _lib.fptr(rel, "rel_emb"),
                  _lib.fptr(self.weight.contiguous(), "weight"), _lib.iptr(wk["col_src"]), _lib.iptr(wk["col_type"]),
                  _lib.iptr(ch), ch.shape[0], _lib.iptr(fx), fx.shape[0], self.num_bases, c, d, _lib.fptr(part),
                  stride, _lib.fptr(agg), _lib.stream())
        prev_t = None
        if self.skip_connect and prev_h is not None:
            prev_t = tangent_of(prev_h, c)[0]
        wl = self.loop_weight if self.self_loop else None
        we = self.evolve_loop_weight if self.self_loop else None
        h, xn, rn = layer_tail(agg, None, x, wl, we, prev_t,
                               self.skip_weight if prev_t is not None else None,
                               self.skip_bias if prev_t is not None else None,
                               _drop_mask(self, x), g, c, euclid=False)
        return attach(h, xn, rn, c)


class LorentzRGCNCell(nn.Module):
    """hyperbolic_layers.py:697-743."""

    def __init__(self, num_nodes, h_dim, out_dim, num_rels, num_bases=-1, num_hidden_layers=1, dropout=0.0, c=0.01,
                 self_loop=False, skip_connect=False, encoder_name="lgcn", rel_emb=None, use_cuda=False,
                 analysis=False):
        super().__init__()
        self.h_dim, self.c = h_dim, c
        self.layers = nn.ModuleList()
        for idx in range(num_hidden_layers):
            sc = False if idx == 0 or not skip_connect else True
            self.layers.append(LorentzRGCNLayer(h_dim, h_dim, num_rels, num_bases, c=c, activation=F.rrelu,
                                                self_loop=self_loop, dropout=dropout, skip_connect=sc))

    def forward(self, g, init_ent_emb, init_rel_emb):
        h = init_ent_emb  # node ids are arange(V) (rgcn/utils.py:122): the gather is the identity
        rel_embs = init_rel_emb if isinstance(init_rel_emb, list) else [init_rel_emb] * len(self.layers)
        prev_h = None
        for i, layer in enumerate(self.layers):
            h_new = layer(g, h, rel_embs[i], prev_h=prev_h)
            prev_h = h
            h = h_new
        return h
