"""Euclidean RE-GCN aggregation layer on HIP (mirror of rgcn/layers.py:182-279).

`UnionRGCNLayer.forward(g, prev_h, emb_rel)` reads g.ndata['h'], writes the new node
representation back to g.ndata['h'] and returns it, as the reference does (:222-255).
One fused launch (regcn_layer_f32, AGG_EUCLID): the CSR gather-sum of (h_src + rel[type])
and the MFMA tail leaky(agg @ W_n + h @ W_loop|W_evolve).
Unlike the reference, it runs without CUDA (`.cuda()` at :230 is not needed).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .hyperbolic_layers import _drop_mask, run_layer


class UnionRGCNLayer(nn.Module):
    def __init__(self, in_feat, out_feat, num_rels, num_bases=-1, bias=None, activation=None, self_loop=False,
                 dropout=0.0, skip_connect=False, rel_emb=None):
        super().__init__()
        if in_feat != out_feat:
            raise ValueError("UnionRGCNLayer needs in_feat == out_feat")
        if activation not in (None, F.rrelu):
            raise ValueError("only the reference activation (F.rrelu) is fused")
        self.in_feat, self.out_feat, self.bias, self.activation = in_feat, out_feat, bias, activation
        self.self_loop, self.num_rels, self.rel_emb, self.skip_connect = self_loop, num_rels, None, skip_connect
        self.ob = self.sub = None
        self.weight_neighbor = nn.Parameter(torch.Tensor(in_feat, out_feat))
        nn.init.xavier_uniform_(self.weight_neighbor, gain=nn.init.calculate_gain("relu"))
        if self_loop:
            self.loop_weight = nn.Parameter(torch.Tensor(in_feat, out_feat))
            nn.init.xavier_uniform_(self.loop_weight, gain=nn.init.calculate_gain("relu"))
            self.evolve_loop_weight = nn.Parameter(torch.Tensor(in_feat, out_feat))
            nn.init.xavier_uniform_(self.evolve_loop_weight, gain=nn.init.calculate_gain("relu"))
        if skip_connect:
            self.skip_connect_weight = nn.Parameter(torch.Tensor(out_feat, out_feat))
            nn.init.xavier_uniform_(self.skip_connect_weight, gain=nn.init.calculate_gain("relu"))
            self.skip_connect_bias = nn.Parameter(torch.Tensor(out_feat))
            nn.init.zeros_(self.skip_connect_bias)
        self.dropout = nn.Dropout(dropout) if dropout else None

    def forward(self, g, prev_h, emb_rel):
        if self.activation is None:
            raise NotImplementedError("the fused tail applies rrelu; activation=None is not supported")
        self.rel_emb = emb_rel
        h = g.ndata["h"].contiguous()
        skip = len(prev_h) != 0 and self.skip_connect
        out, _, _ = run_layer(_lib.AGG_EUCLID, g, h, None, emb_rel.contiguous(), None, 0, 0.0, self.weight_neighbor,
                              self.loop_weight if self.self_loop else None,
                              self.evolve_loop_weight if self.self_loop else None,
                              prev_h.contiguous() if skip else None,
                              self.skip_connect_weight if skip else None,
                              self.skip_connect_bias.detach() if skip else None, _drop_mask(self, h), 0.01,
                              euclid=True)
        g.ndata["h"] = out
        return out
