"""HyperbolicRecurrentRGCN on HIP (mirror of hyperbolic_src/hyperbolic_model.py).

Same constructor arguments, state_dict keys and the drop-in
signatures `forward(g_list, static_graph, use_cuda)` -> (history_embs, static_emb, h_0,
gate_list, degree_list), `predict(...)` and `get_loss(...)`.

Per timestep (hyperbolic_model.py:797-884) the path is:
  relation context mean + GRU  regcn_relation_gru_f32     (one launch, MFMA)
  encoder cell (L layers)      regcn_layer_f32            (one launch per layer: gather + MFMA tail)
  project/LN/time gate/radius  fused into the last layer's launch (regcn_layer_f32 fuse_step)
The initial entity state is one fused row kernel (regcn_init_entities_f32).

Scope: eval/forward.  Static graph (--add-static-graph), EST components, FHNN/HGAT
encoders and geoopt manifold parameters are out of scope and raise.
"""
import contextlib
import ctypes
import os
import logging
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import analysis as _ana
from .hyperbolic_decoder import (HyperbolicAttH, HyperbolicAttHRel, HyperbolicConvTransE, HyperbolicConvTransR,
                                 HyperbolicMuRP, HyperbolicMuRPRel, HyperbolicRotH, HyperbolicRotHRel,
                                 roth_pair_fusable, roth_pair_predict)
from .graph import SnapshotGraph, rel_block_work
from .hyperbolic_layers import HyperbolicUnionRGCNLayer, LorentzRGCNCell, LorentzRGCNLayer, StepSpec, \
    _heavy_aggregate
from .hyperbolic_ops import HyperbolicOps, TemporalRadiusEvolution
from .parallel import FULL_EXCHANGE, ShardedGraph, complete
from .tangent import attach, tangent_of
from .weights import invalidate, packed

logger = logging.getLogger("hyperbolic_model")
TRACE_SLOTS = 8  # timestep.hip: stamps per workgroup
PHASE_TRACE = None  # profiling: a list to collect per-workgroup stamps of the phase launches
PHASE_CAPTURE = None  # profiling: a dict to receive replayable launches of the last timestep's phases
GEOOPT_AVAILABLE = False


class HyperbolicBaseRGCN(nn.Module):
    """hyperbolic_model.py:74-111."""

    def __init__(self, num_nodes, h_dim, out_dim, num_rels, num_bases=-1, num_hidden_layers=1, dropout=0, c=0.01,
                 self_loop=False, skip_connect=False, encoder_name="hyperbolic_uvrgcn", rel_emb=None, use_cuda=False,
                 analysis=False, radius_msg_gamma=1.0):
        super().__init__()
        self.num_nodes, self.h_dim, self.out_dim, self.num_rels = num_nodes, h_dim, out_dim, num_rels
        self.num_bases, self.num_hidden_layers, self.dropout, self.c = num_bases, num_hidden_layers, dropout, c
        self.self_loop, self.skip_connect, self.encoder_name = self_loop, skip_connect, encoder_name
        self.rel_emb = rel_emb
        self.use_cuda, self.run_analysis, self.radius_msg_gamma = use_cuda, analysis, radius_msg_gamma
        self.layers = nn.ModuleList([self.build_hidden_layer(i) for i in range(num_hidden_layers)])

    def build_hidden_layer(self, idx):
        raise NotImplementedError


class HyperbolicRGCNCell(HyperbolicBaseRGCN):
    """hyperbolic_model.py:114-154."""

    def build_hidden_layer(self, idx):
        sc = False if idx == 0 or not self.skip_connect else True
        return HyperbolicUnionRGCNLayer(self.h_dim, self.h_dim, self.num_rels, self.num_bases, c=self.c,
                                        activation=F.rrelu, self_loop=self.self_loop, dropout=self.dropout,
                                        skip_connect=sc, radius_msg_gamma=self.radius_msg_gamma)

    def forward(self, g, init_ent_emb, init_rel_emb, step=None, pos_only=False, out=None):
        """`step` (StepSpec): the timestep runs fused into the last layer's launch;
        pos_only/out: the launches cover the rows with in-edges only (run_layer)."""
        h = init_ent_emb  # node ids are arange(V): the reference gather is the identity
        rel_embs = init_rel_emb if isinstance(init_rel_emb, list) else [init_rel_emb] * len(self.layers)
        n = len(self.layers)
        for i, layer in enumerate(self.layers):
            # prev_h is never passed (hyperbolic_model.py:152)
            last = i == n - 1
            h = layer(g, h, rel_embs[i], step=step if last else None, pos_only=pos_only, out=out if last else None,
                      gate=step if (i == 0 and not last) else None,
                      need_h=last or step is None)  # a fused-step cell's inner h: read as x, |h| only
        return h


def relation_context(x, g, num_rels2):
    """x_input[r] = mean_{e in r_to_e span} x[e] (hyperbolic_model.py:802-812), HIP.  The
    work lists chunk the forward relations' spans only: r2e gives an inverse id r + R the
    same entity list as r, in the same order (rgcn/utils.py:88-89), so its mean is the
    same sum of the same rows, copied instead of recomputed (half the row gathers)."""
    if getattr(g, "partition", None) == "owner" and g.world > 1:  # partitioned pairs (parallel.py)
        return g.relation_means(x, num_rels2)
    wk = g.work()
    V, d = x.shape
    R = num_rels2 // 2
    out = torch.zeros(num_rels2, d, device=x.device, dtype=torch.float32)
    blocks = rel_block_work(g, R)
    if blocks is not None:  # large snapshot: entity-block chunks, XCD-dealt (graph.rel_block_lists)
        ch, fx, n_slots = blocks
    else:
        ch, fx, n_slots = wk["rel_chunks"], wk["rel_fixups"], g.rel_slots
    part = torch.empty(n_slots, d, device=x.device, dtype=torch.float32) if n_slots else None
    _lib.call("regcn_segment_mean_f32", _lib.fptr(x, "x"), _lib.iptr(wk["rel_idx"]), _lib.fptr(wk["rel_count"]),
              _lib.iptr(ch), ch.shape[0], _lib.iptr(fx), fx.shape[0], d, _lib.fptr(part), d, _lib.fptr(out),
              _lib.stream())
    out[R:].copy_(out[:R])
    return out


# the owner partition's exchange: the rows the next layer reads (parallel.ExchangePlan); 0: every
# row after every layer (in-place all-gathers)
SPARSE_EXCHANGE = os.environ.get("REGCN_SPARSE_EXCHANGE", "1") != "0"
# ... and each rank maps only the initial rows it reads (ShardedGraph.initial_state); 0: all V
OWNER_INIT = os.environ.get("REGCN_OWNER_INIT", "1") != "0"

INIT_SKIP_H = os.environ.get("REGCN_INIT_SKIP_H", "1") != "0"  # see HyperbolicRecurrentRGCN._initial_state
# predict's last timestep on the 64-row tail writes h only (StepSpec.need_xr); 0: x and |h| too
LAST_SKIP_XR = os.environ.get("REGCN_LAST_SKIP_XR", "1") != "0"
REL_INLINE_MAX_SPAN = 64  # longer r_to_e spans are averaged by the chunked segment-mean kernel first


def _means_first(g):
    """The relation means as their own launch: long r_to_e spans, or an owner-partitioned
    snapshot (a rank holds only the rows the exchange sent it: the partitioned sums, never the
    GRU's inline means over every entity)."""
    return g.rel_max_span > REL_INLINE_MAX_SPAN or (getattr(g, "partition", None) == "owner" and g.world > 1)


def relation_gru_step(gru, emb_rel, x, g, h_prev):
    """h_0' = GRUCell([emb_rel | mean_{r_to_e} x], h_prev) in one launch
    (regcn_relation_gru_f32; hyperbolic_model.py:797-818, src/rrgcn.py:161-174)."""
    from .weights import packed_linear
    wk = g.work()
    R2, d = emb_rel.shape
    x_mean = relation_context(x, g, R2) if _means_first(g) else None
    zeros = None
    if gru.bias_ih is None:
        zeros = torch.zeros(3 * d, device=emb_rel.device, dtype=torch.float32)
    b_ih = gru.bias_ih.detach() if gru.bias_ih is not None else zeros
    b_hh = gru.bias_hh.detach() if gru.bias_hh is not None else zeros
    out = torch.empty(R2, d, device=emb_rel.device, dtype=torch.float32)
    f = _lib.fptr
    _lib.call("regcn_relation_gru_f32", f(x, "x"), _lib.iptr(wk["rel_idx"]) if wk["rel_idx"].numel() else None,
              _lib.iptr(wk["rel_start"]), f(wk["rel_count"]), f(x_mean), f(emb_rel.detach(), "emb_rel"),
              f(h_prev.detach().contiguous(), "h_0"), f(packed_linear(gru.weight_ih, 3)),
              f(packed_linear(gru.weight_hh, 3)), f(b_ih), f(b_hh), R2, d, f(out), _lib.stream())
    return out


def _gru_biases(gru, d, device):
    zeros = None
    if gru.bias_ih is None or gru.bias_hh is None:
        zeros = torch.zeros(3 * d, device=device, dtype=torch.float32)
    b_ih = gru.bias_ih.detach() if gru.bias_ih is not None else zeros
    b_hh = gru.bias_hh.detach() if gru.bias_hh is not None else zeros
    return b_ih, b_hh


def relation_gru_pre(gru, emb_rel, h_prev):
    """The gate pre-activations of GRUCell([emb_rel | x_mean], h_prev) that do not depend on
    x_mean (regcn_relation_gru_pre_f32): R2 x 4 x d."""
    from .weights import packed_linear, packed_linear_cols
    R2, d = emb_rel.shape
    b_ih, b_hh = _gru_biases(gru, d, emb_rel.device)
    pre = torch.empty(R2, 4, d, device=emb_rel.device, dtype=torch.float32)
    f = _lib.fptr
    _lib.call("regcn_relation_gru_pre_f32", f(emb_rel.detach(), "emb_rel"), f(h_prev.detach().contiguous(), "h_0"),
              f(packed_linear_cols(gru.weight_ih, 3, 0, d)), f(packed_linear(gru.weight_hh, 3)), f(b_ih), f(b_hh),
              R2, d, f(pre), _lib.stream())
    return pre


def relation_gru_x(gru, x, g, h_prev, pre):
    """h_0' from the relation means of x over the snapshot's r_to_e spans and `pre`
    (regcn_relation_gru_x_f32; hyperbolic_model.py:797-818)."""
    from .weights import packed_linear_cols
    wk = g.work()
    R2, d = h_prev.shape
    x_mean = relation_context(x, g, R2) if _means_first(g) else None
    out = torch.empty(R2, d, device=h_prev.device, dtype=torch.float32)
    f = _lib.fptr
    _lib.call("regcn_relation_gru_x_f32", f(x, "x"), _lib.iptr(wk["rel_idx"]) if wk["rel_idx"].numel() else None,
              _lib.iptr(wk["rel_start"]), f(wk["rel_count"]), f(x_mean), f(h_prev.detach().contiguous(), "h_0"),
              f(packed_linear_cols(gru.weight_ih, 3, d, 2 * d)), f(pre), R2, d, f(out), _lib.stream())
    return out


class HyperbolicRecurrentRGCN(nn.Module):
    """hyperbolic_model.py:157-1128."""

    # inference of a 2-layer cell: each timestep in three phase launches (_forward_phases,
    # csrc/timestep.hip); False keeps the per-layer launches (same values bit for bit)
    use_phases = True
    # with the phases: a row without an in-edge so far in the window holds a state that is a
    # function of the parameters only (F^t of the initial state, F = the cell and timestep of
    # a row without messages); those states are memoised per parameter version
    # (regcn_cold_chain_f32 over all rows, _pristine_states) and copied, so a timestep runs
    # only its in-edge rows and the rows that had in-edges earlier.  Same values bit for bit.
    memo_pristine = True
    # parameter-only states (static radius, initial entity state, timestep 0's GRU pre-half,
    # the pristine-row memo) kept across calls per parameter version; False recomputes them in
    # every forward (bench.py's headline: a step computes everything from the parameters)
    param_caches = True
    # with the phases and no memo: a snapshot's rows without in-edges run their whole
    # timestep in one launch (regcn_zero_step_f32) on a side stream beside the phase launches,
    # which then carry only the in-edge tiles and the relation GRU.  Same values bit for bit.
    split_zero_rows = True
    zero_rows_side_stream = False  # True: the zero-row launch forks to a side stream
    # eval predict with RotH + RotHRel: the decoders as two launches on the calling stream
    # (hyperbolic_decoder.roth_pair_predict); False keeps the per-decoder path on two streams
    fused_decoders = True

    def __init__(self, decoder_name, encoder_name, num_ents, num_rels, num_static_rels, num_words, h_dim, opn,
                 sequence_len, num_bases=-1, num_hidden_layers=1, dropout=0, c=0.01, self_loop=False,
                 skip_connect=False, layer_norm=False, input_dropout=0, hidden_dropout=0, feat_dropout=0, weight=1,
                 discount=0, angle=0, use_static=False, entity_prediction=False, relation_prediction=False,
                 use_cuda=False, gpu=0, analysis=False, learn_curvature=False, use_residual_evolution=True,
                 radius_target=None, radius_lambda=0.02, radius_min=0.5, radius_max=3.0, radius_epsilon=0.1,
                 radius_anchor_beta=1.0, curvature_min=1e-4, curvature_max=1e-1, num_heads=4, query_chunk_size=128,
                 candidate_chunk_size=256, hyp_init_scale=1e-3, hyp_score_scale_init=1.0, hyp_score_margin_init=1.0,
                 use_entity_euclidean_bias=False, use_relation_specific_curvature=False, use_est=False,
                 est_state_alpha=0.2, est_encoder="gru", use_time_aware_negative=False, radius_msg_gamma=1.0):
        super().__init__()
        if use_static:
            raise NotImplementedError("--add-static-graph is outside this build's scope (SURVEY.md §2 row 1)")
        if use_est:
            raise NotImplementedError("EST components are outside this build's scope (SURVEY.md §2 row 8)")
        if encoder_name not in ("hyperbolic_uvrgcn", "lgcn"):
            raise NotImplementedError("encoder %r is outside this build's scope (hyperbolic_uvrgcn, lgcn)"
                                      % encoder_name)
        self.decoder_name, self.encoder_name = decoder_name, encoder_name
        self.num_rels, self.num_ents, self.opn, self.num_words = num_rels, num_ents, opn, num_words
        self.num_static_rels, self.sequence_len, self.h_dim = num_static_rels, sequence_len, h_dim
        self.layer_norm, self.h, self.run_analysis = layer_norm, None, analysis
        self.weight, self.discount, self.use_static, self.angle = weight, discount, use_static, angle
        self.relation_prediction, self.entity_prediction, self.gpu = relation_prediction, entity_prediction, gpu
        self.learn_curvature, self.use_residual_evolution = learn_curvature, use_residual_evolution
        self.radius_lambda, self.radius_min, self.radius_max = radius_lambda, radius_min, radius_max
        self.radius_anchor_beta, self.curvature_min, self.curvature_max = radius_anchor_beta, curvature_min, \
            curvature_max
        self.num_heads, self.query_chunk_size, self.candidate_chunk_size = num_heads, query_chunk_size, \
            candidate_chunk_size
        self.use_entity_euclidean_bias = use_entity_euclidean_bias
        self.use_relation_specific_curvature = use_relation_specific_curvature
        self.radius_msg_gamma, self.use_est = radius_msg_gamma, use_est
        self.est_state_alpha, self.use_time_aware_negative = est_state_alpha, use_time_aware_negative
        self.temporal_index, self.true_tails_by_hr = None, None
        if learn_curvature:
            self.log_c = nn.Parameter(torch.tensor(math.log(c)))
        else:
            self.register_buffer("c", torch.tensor(c))
        self.training_stats = _ana.TrainingStats()  # device values, read on access (analysis.py)
        self.dynamic_emb = nn.Parameter(torch.Tensor(num_ents, h_dim))
        nn.init.normal_(self.dynamic_emb, std=1.0)
        self.emb_rel = nn.Parameter(torch.Tensor(num_rels * 2, h_dim))
        nn.init.xavier_normal_(self.emb_rel)
        self.temporal_radius_evolution = TemporalRadiusEvolution(h_dim, c=c, epsilon=radius_epsilon,
                                                                 anchor_beta=radius_anchor_beta)
        self.w1 = nn.Parameter(torch.Tensor(h_dim, h_dim))
        nn.init.xavier_normal_(self.w1)
        self.w2 = nn.Parameter(torch.Tensor(h_dim, h_dim))
        nn.init.xavier_normal_(self.w2)
        self.loss_r = nn.CrossEntropyLoss()
        self.loss_e = nn.CrossEntropyLoss()
        if encoder_name == "hyperbolic_uvrgcn":
            self.rgcn = HyperbolicRGCNCell(num_ents, h_dim, h_dim, num_rels * 2, num_bases, num_hidden_layers,
                                           dropout, c=c, self_loop=self_loop, skip_connect=skip_connect,
                                           encoder_name=encoder_name, rel_emb=self.emb_rel, use_cuda=use_cuda,
                                           analysis=analysis, radius_msg_gamma=radius_msg_gamma)
        else:
            self.rgcn = LorentzRGCNCell(num_ents, h_dim, h_dim, num_rels * 2, num_bases, num_hidden_layers, dropout,
                                        c=c, self_loop=self_loop, skip_connect=skip_connect,
                                        encoder_name=encoder_name, rel_emb=self.emb_rel, use_cuda=use_cuda,
                                        analysis=analysis)
        self.time_gate_weight = nn.Parameter(torch.Tensor(h_dim, h_dim))
        nn.init.xavier_uniform_(self.time_gate_weight, gain=nn.init.calculate_gain("relu"))
        self.time_gate_bias = nn.Parameter(torch.zeros(h_dim))
        self.relation_gru = nn.GRUCell(h_dim * 2, h_dim)
        dk = dict(query_chunk_size=query_chunk_size, candidate_chunk_size=candidate_chunk_size)
        hk = dict(init_scale=hyp_init_scale, score_scale_init=hyp_score_scale_init,
                  score_margin_init=hyp_score_margin_init)
        ek = dict(use_entity_euclidean_bias=use_entity_euclidean_bias,
                  use_relation_specific_curvature=use_relation_specific_curvature)
        if decoder_name == "hyperbolic_convtranse":
            self.decoder_ob = HyperbolicConvTransE(num_ents, h_dim, c=c, input_dropout=input_dropout,
                                                   hidden_dropout=hidden_dropout, feature_map_dropout=feat_dropout)
            self.rdecoder = HyperbolicConvTransR(num_rels, h_dim, c=c, input_dropout=input_dropout,
                                                 hidden_dropout=hidden_dropout, feature_map_dropout=feat_dropout)
        elif decoder_name == "murp":
            self.decoder_ob = HyperbolicMuRP(num_ents, num_rels * 2, h_dim, c=c, dropout=input_dropout, **dk, **hk,
                                             **ek)
            self.rdecoder = HyperbolicMuRPRel(num_rels, h_dim, c=c, dropout=input_dropout, **dk)
        elif decoder_name == "roth":
            self.decoder_ob = HyperbolicRotH(num_ents, num_rels * 2, h_dim, c=c, dropout=input_dropout, **dk, **hk,
                                             **ek)
            self.rdecoder = HyperbolicRotHRel(num_rels, h_dim, c=c, dropout=input_dropout, **dk, **hk)
        elif decoder_name == "atth":
            self.decoder_ob = HyperbolicAttH(num_ents, num_rels * 2, h_dim, c=c, dropout=input_dropout, **dk, **hk,
                                             **ek)
            self.rdecoder = HyperbolicAttHRel(num_rels, h_dim, c=c, dropout=input_dropout, **dk, **hk)
        else:
            raise NotImplementedError("Decoder '%s' not implemented. Choose from: hyperbolic_convtranse, murp, "
                                      "roth, atth" % decoder_name)
        target = torch.full((num_ents,), 0.5 * (radius_min + radius_max)) if radius_target is None else \
            torch.as_tensor(radius_target, dtype=torch.float)
        self.register_buffer("radius_target", target)
        self.radius_static = nn.Parameter(self.radius_target.clone())
        # load_state_dict copies through no-grad in-place writes; drop the parameter-keyed
        # caches explicitly rather than rely on version counters alone
        self.register_load_state_dict_post_hook(lambda module, _keys: invalidate(module))

    # ---------------------------------------------------------------------------- helpers
    def get_curvature(self):
        """hyperbolic_model.py:673-679."""
        if self.learn_curvature:
            return torch.clamp(torch.exp(self.log_c), min=self.curvature_min, max=self.curvature_max)
        return self.c

    def set_curvature_bounds(self, curvature_min=None, curvature_max=None):
        if curvature_min is not None:
            self.curvature_min = curvature_min
        if curvature_max is not None:
            self.curvature_max = curvature_max

    def set_relation_curvature_bounds(self, curvature_max=None):
        dec = getattr(self, "decoder_ob", None)
        if dec is not None and hasattr(dec, "set_relation_curvature_bounds"):
            dec.set_relation_curvature_bounds(curvature_max=curvature_max)

    def _c_float(self):
        """The curvature as a python float.  A fixed curvature is a buffer that only
        changes through load_state_dict/in-place edits, so its value is cached against
        the buffer's version counter: no device->host sync per forward, which keeps the
        forward capturable into a HIP graph.  A learned curvature is read each call, as
        the reference does (hyperbolic_model.py:755)."""
        if self.learn_curvature:
            return float(self.get_curvature().detach().item())
        key = (self.c.data_ptr(), self.c._version)
        if getattr(self, "_c_cache", (None, None))[0] != key:
            self._c_cache = (key, float(self.c.item()))
        return self._c_cache[1]

    def _static_radius(self, c_val=None):
        """hyperbolic_model.py:715-720."""
        if c_val is None:
            c_val = self._c_float()
        p = self.radius_static
        key = (p.data_ptr(), p._version, float(c_val), self.radius_min, self.radius_max)
        hit = getattr(self, "_r_static_cache", None)
        if hit is not None and hit[0] == key and not torch.is_grad_enabled() and self.param_caches:
            return hit[1]  # parameter-only value: computed once per parameter version
        radius = torch.clamp(p, min=self.radius_min, max=self.radius_max)
        radius = torch.clamp(radius, max=1.0 / math.sqrt(c_val) - 1e-6)
        if not torch.is_grad_enabled() and self.param_caches:
            self._r_static_cache = (key, radius.detach().contiguous())
            _lib.publish()
        return radius

    def _wants_grad(self):
        return torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())

    # ---------------------------------------------------------------------------- forward
    def forward(self, g_list, static_graph, use_cuda):
        """hyperbolic_model.py:722-890.  With autograd on (training) the differentiable
        composition of training.py runs; otherwise the fused inference kernels."""
        if self._wants_grad():
            from .training import model_forward
            out = model_forward(self, g_list)
            self.h, self.h_0 = out[0][-1], out[2]
            return out
        c_val = self._c_float()
        dev = self.dynamic_emb.device
        V, d = self.dynamic_emb.shape
        fused_step = len(self.rgcn.layers) > 0 and not self.run_analysis
        g_list = list(g_list)
        if g_list:
            g_list[0] = g_list[0].to(dev)
        g0 = g_list[0] if g_list else None
        # owner partition with the sparse halo exchange: each rank maps only the initial rows it
        # reads (its own + the first snapshot's halo) instead of all V (ShardedGraph.initial_state)
        owner0 = (fused_step and SPARSE_EXCHANGE and OWNER_INIT and isinstance(g0, ShardedGraph) and g0.halo_initial_state())
        scope = self.__dict__.get("_scope")
        if scope is not None and scope["c"] == c_val:  # a batch's shared parameter-only states
            r_static = scope["r_static"]
            h, x, r = scope["init"]
        else:
            r_static = self._static_radius(c_val).contiguous()
            # the fused per-layer path (config 5) reads the initial state's x and |h| only; the
            # phase launches and the unfused timestep may read h itself
            need_h = not (fused_step and not self._phases_ok(g_list) and INIT_SKIP_H)
            h, x, r = self._initial_state(c_val, r_static, g0 if owner0 else None, need_h=need_h)
        attach(h, x, r, c_val)
        self.h = h
        R2 = self.num_rels * 2
        history_embs = []
        trev = self.temporal_radius_evolution
        wg, bg, w_r, b_r = self._step_tensors()
        if self._phases_ok(g_list):
            return self._forward_phases(g_list, c_val, r_static, wg, bg, w_r, b_r)
        ana = self.run_analysis
        if ana and self.training:  # hyperbolic_model.py:791-792
            _ana.log_embedding(self, h, "init_embeddings", c_val)
        gate_list, gate_means = [], []
        for i, g in enumerate(g_list):
            g = g.to(dev)
            if isinstance(g, ShardedGraph) and g.partition == "owner":
                # the owner partition sends each layer's new rows only to the ranks whose next
                # layer reads them: this snapshot's sources, then the next timestep's; after the
                # last timestep all rows, unless the caller reads only its own (predict_ranks)
                nxt = g_list[i + 1] if i + 1 < len(g_list) else \
                    (None if self.__dict__.get("_owner_rows_only") else FULL_EXCHANGE)
                g.consumers = (g, nxt) if fused_step and SPARSE_EXCHANGE else None
            x_prev, _ = tangent_of(self.h, c_val)
            h_prev = self.emb_rel if i == 0 else self.h_0  # the two-phase GRU, as _forward_phases runs it
            self.h_0 = relation_gru_x(self.relation_gru, x_prev, g, h_prev,
                                      relation_gru_pre(self.relation_gru, self.emb_rel, h_prev))
            self.h_0 = F.normalize(self.h_0) if self.layer_norm else self.h_0
            if len(self.rgcn.layers) and not self.run_analysis:
                # cell + timestep: the last layer's launch runs the timestep on its output
                step = StepSpec(x_prev, wg, bg, r_static, w_r, b_r, trev.epsilon, trev.anchor_beta,
                                self.layer_norm, self.use_residual_evolution, trev.c,
                                w_g_param=self.time_gate_weight)
                # predict reads the last state's h only; the next timestep reads x and |h|
                step.need_h = i == len(g_list) - 1 or not self.__dict__.get("_last_h_only")
                # ... and its x and |h| are dead (the decoders read h; nothing follows the last
                # timestep), unless ranks still exchange them (owner partition)
                step.need_xr = not (LAST_SKIP_XR and i == len(g_list) - 1 and self.__dict__.get("_last_h_only")
                                    and not isinstance(g, ShardedGraph))
                self.h = self.rgcn.forward(g, self.h, [self.h_0, self.h_0], step=step)
            else:
                # the timestep kernel reads every row of current_h (and recomputes x, |h| from
                # it): under the owner partition only this rank's rows are written, so gather
                # the rest first (the all-gather of h the fused step's sparse exchange avoids)
                current_h = complete(self.rgcn.forward(g, self.h, [self.h_0, self.h_0]))
                h_new = torch.empty_like(x_prev)
                x_new = torch.empty_like(x_prev)
                r_new = torch.empty(V, device=dev, dtype=torch.float32)
                args = (_lib.fptr(current_h.contiguous(), "current_h"), _lib.fptr(x_prev), _lib.fptr(wg),
                        _lib.fptr(bg), _lib.fptr(r_static), _lib.fptr(w_r), _lib.fptr(b_r), float(trev.epsilon),
                        float(trev.anchor_beta), int(bool(self.layer_norm)), int(bool(self.use_residual_evolution)),
                        V, d, c_val, float(trev.c), _lib.fptr(h_new), _lib.fptr(x_new), _lib.fptr(r_new))
                if ana:  # the time gate and the radius terms come out of the timestep launch
                    gate = torch.empty_like(x_prev)
                    stat = torch.empty(3, V, device=dev, dtype=torch.float32) \
                        if self.use_residual_evolution else None
                    _lib.call("regcn_timestep_analysis_f32", *args, _lib.fptr(gate), _lib.fptr(stat), _lib.stream())
                    gate_list.append(gate)                                      # :852-856
                    gate_means.append(gate.mean())
                    if stat is not None:                                        # hyperbolic_ops.py:426-434
                        trev.last_evolution_stats = _ana.evolution_terms(stat[0], stat[1], stat[2], r_static,
                                                                             trev.anchor_beta, trev.epsilon)
                    _ana.log_timestep(i, gate_means[-1], trev.__dict__.get("_ev"))
                else:
                    _lib.call("regcn_timestep_f32", *args, _lib.stream())
                self.h = attach(h_new, x_new, r_new, c_val)
            history_embs.append(self.h)
        if history_embs and not self.__dict__.get("_owner_rows_only"):
            # owner partition: the last state holds this rank's rows only until its h rows are
            # all-gathered (its x and |h| already were: the last exchange is FULL_EXCHANGE), so
            # every caller of forward (predict, get_loss, ...) sees complete rows; the earlier
            # history entries stay rank-local (parallel.complete fills one in when needed)
            last = history_embs[-1]
            xr = getattr(last, "_regcn_xr", None)
            if getattr(last, "_regcn_owner", None) is not None:
                complete(last)
                if xr is not None:  # the in-place gather bumped h's version: same x and |h|
                    attach(last, xr[0], xr[1], xr[2])
        if ana:  # hyperbolic_model.py:887-888
            dict.__setitem__(self.training_stats, "time_gate_values",
                             torch.stack(gate_means) if gate_means else [])
        return history_embs, None, self.h_0, gate_list, []

    def _initial_state(self, c_val, r_static, owner=None, need_h=True):
        """(h, x, r) of the initial entity state (hyperbolic_model.py:775-782): a function of
        parameters only, computed once per parameter version (param_caches) and reused by every
        predict (the kernels read it, none writes it), so a captured predict graph holds no init
        launch.  owner: the first snapshot of an owner partition -- only the rows this rank
        reads (ShardedGraph.initial_state).  need_h=False: the Poincare rows h are not written
        (the fused timestep path reads x = log0 h and |h| only: 800 MB less per predict at
        config 5); h is then an unwritten buffer carrying x and |h| (tangent.attach)."""
        pe = self.dynamic_emb
        V, d = pe.shape
        key = (pe.data_ptr(), pe._version, self.radius_static.data_ptr(), self.radius_static._version,
               float(c_val), bool(self.layer_norm), float(self.radius_min), float(self.radius_max), id(owner),
               bool(need_h))
        hit = self.__dict__.get("_init_cache")
        if hit is not None and hit[0] == key and hit[2] is owner and self.param_caches:
            return hit[1]
        dyn = pe.detach().contiguous()
        if owner is not None:
            h, x, r = owner.initial_state(dyn, r_static, c_val, self.layer_norm)
        else:
            h = torch.empty_like(dyn)
            x = torch.empty_like(dyn)
            r = torch.empty(V, device=pe.device, dtype=torch.float32)
            _lib.call("regcn_init_entities_f32", _lib.fptr(dyn, "dynamic_emb"), _lib.fptr(r_static), V, d, c_val,
                      int(bool(self.layer_norm)), _lib.fptr(h) if need_h else None, _lib.fptr(x), _lib.fptr(r),
                      _lib.stream())
        if self.param_caches and not torch.cuda.is_current_stream_capturing():
            _lib.publish()
            self.__dict__["_init_cache"] = (key, (h, x, r), owner)
        return h, x, r

    def _step_tensors(self):
        """Timestep operands: packed time-gate weight, its bias, the radius MLP row and bias."""
        trev = self.temporal_radius_evolution
        w_r = trev.radius_mlp.weight.detach().reshape(-1).contiguous()
        b_r = trev.radius_mlp.bias.detach().reshape(-1).contiguous()
        return packed(self.time_gate_weight), self.time_gate_bias.detach().contiguous(), w_r, b_r

    @contextlib.contextmanager
    def shared_parameter_states(self, T):
        """A batch of independent predicts (e.g. the test snapshots of one evaluation pass
        without --multi-step, hyperbolic_main.py:100-149) over windows of T snapshots shares its
        parameter-only states: the static radius, the initial entity state, timestep 0's GRU
        pre-half and, with the phase launches, the states F^t(initial state) of rows without an
        in-edge so far in the window (regcn_cold_chain_f32 over all rows: every predict inside
        copies them instead of running those rows).  Computed once on entry, on the current
        stream, and dropped on exit: nothing outlives the batch.  Same values bit for bit."""
        saved = self.__dict__.get("_scope")
        try:
            scope = self._shared_states(T)
        except BaseException:
            self.__dict__["_scope"] = saved
            raise
        self.__dict__["_scope"] = scope
        try:
            yield
        finally:
            self.__dict__["_scope"] = saved
            if torch.cuda.is_current_stream_capturing():  # a captured graph reads them at replay
                self.__dict__.setdefault("_capture_keep", []).append(scope)

    def _shared_states(self, T):
        """The dict shared_parameter_states installs (computed with no scope active)."""
        self.__dict__["_scope"] = None
        with torch.no_grad():
            c_val = self._c_float()
            r_static = self._static_radius(c_val).contiguous()
            init = self._initial_state(c_val, r_static)
            pre0 = relation_gru_pre(self.relation_gru, self.emb_rel, self.emb_rel)
            memo, keep = None, []
            layers = list(self.rgcn.layers)
            if (self.use_phases and self.dynamic_emb.device.type == "cuda" and len(layers) == 2
                    and not self.run_analysis and not any(l.training for l in layers) and T <= _lib.MAX_WINDOW):
                desc, keep = self._phase_desc(r_static, *self._step_tensors())
                memo = self._pristine_states(T, c_val, desc, cache=False, x_init=init[1])
                keep = keep + [self.__dict__.pop("_chain_operands")]
            return dict(T=T, c=c_val, r_static=r_static, init=init, pre0=pre0, memo=memo, keep=keep)

    def _phases_ok(self, g_list):
        """The phase pipeline serves eval forwards of a 2-layer cell over plain snapshots
        (no dropout masks, no analysis hooks, no multi-GPU partition)."""
        layers = list(self.rgcn.layers)
        return (self.use_phases and self.dynamic_emb.device.type == "cuda" and len(layers) == 2
                and not self.run_analysis and not any(l.training for l in layers)
                and all(isinstance(g, SnapshotGraph) for g in g_list))

    def _gru_pre_initial(self):
        """Timestep 0's GRU pre-half: a function of parameters only (h_prev = emb_rel),
        computed once per parameter version."""
        scope = self.__dict__.get("_scope")
        if scope is not None:
            return scope["pre0"]
        gru, emb = self.relation_gru, self.emb_rel
        key = tuple((t.data_ptr(), t._version) for t in (emb, gru.weight_ih, gru.weight_hh, gru.bias_ih, gru.bias_hh)
                    if t is not None)
        hit = self.__dict__.get("_gru_pre0")
        if hit is not None and hit[0] == key and self.param_caches:
            return hit[1]
        pre = relation_gru_pre(gru, emb, emb)
        if self.param_caches and not torch.cuda.is_current_stream_capturing():
            _lib.publish()
            self.__dict__["_gru_pre0"] = (key, pre)
        return pre

    def _phase_desc(self, r_static, wg, bg, w_r, b_r):
        """regcn_phase_desc fields that depend on the parameters only (packed weights, the
        timestep and relation-GRU operands); returns (desc, tensors it points into)."""
        from .weights import packed_linear, packed_linear_cols
        dev = self.dynamic_emb.device
        d = self.dynamic_emb.shape[1]
        R2 = self.emb_rel.shape[0]
        layers = list(self.rgcn.layers)
        lorentz = isinstance(layers[0], LorentzRGCNLayer)
        trev = self.temporal_radius_evolution
        gru, emb = self.relation_gru, self.emb_rel.detach()
        b_ih, b_hh = _gru_biases(gru, d, dev)
        a = _lib.addr
        desc = _lib.PhaseDesc()
        desc.agg_mode = _lib.AGG_LORENTZ if lorentz else _lib.AGG_UNION
        desc.c, desc.d = float(layers[0].c), d  # the layers' own curvature, as their launches use
        for i, l in enumerate(layers):
            if lorentz:
                desc.w_rel[i] = a(l.weight.detach().contiguous())
                desc.num_bases = int(l.num_bases)
            else:
                desc.w_n[i] = a(packed(l.weight_neighbor))
                desc.gamma = float(l.radius_msg_gamma)
            if l.self_loop:
                desc.w_loop[i] = a(packed(l.loop_weight))
                desc.w_evolve[i] = a(packed(l.evolve_loop_weight))
        if lorentz and layers[1].skip_connect:
            desc.w_skip1 = a(packed(layers[1].skip_weight))
            desc.b_skip1 = a(layers[1].skip_bias.detach())
        desc.step_w_g, desc.step_b_g, desc.step_r_static = a(wg), a(bg), a(r_static)
        desc.step_w_r, desc.step_b_r = a(w_r), a(b_r)
        desc.step_eps_r, desc.step_beta = float(trev.epsilon), float(trev.anchor_beta)
        desc.step_layer_norm, desc.step_residual = int(bool(self.layer_norm)), int(bool(self.use_residual_evolution))
        desc.step_c_radius = float(trev.c)
        desc.gru_emb_rel, desc.gru_R2 = a(emb), R2
        desc.gru_w_ih_e = a(packed_linear_cols(gru.weight_ih, 3, 0, d))
        desc.gru_w_ih_x = a(packed_linear_cols(gru.weight_ih, 3, d, 2 * d))
        desc.gru_w_hh = a(packed_linear(gru.weight_hh, 3))
        desc.gru_b_ih, desc.gru_b_hh = a(b_ih), a(b_hh)
        return desc, [b_ih, b_hh]

    def _forward_phases(self, g_list, c_val, r_static, wg, bg, w_r, b_r):
        """The timestep loop with a 2-layer cell as three launches per snapshot on one
        stream (regcn_timestep_phase_f32, csrc/timestep.hip):
          A  relation GRU x-half; in-edge rows' self-loop and time-gate GEMMs (need only the
             timestep input); rows without in-edges: layer 0;
          B  in-edge tiles: layer-0 gather -> finish -> epilogue -> layer 1's self-loop
             GEMM; other rows: layer 1; relation GRU pre-half of the next timestep;
          C  in-edge tiles: layer-1 gather -> timestep; other rows: timestep.
        Without the memo (split_zero_rows) the rows without in-edges leave A/B/C: one
        regcn_zero_step_f32 launch on a side stream runs their layer 0, layer 1 and timestep,
        forked after timestep t - 1 and joined after C.
        Same values as the per-layer launches bit for bit (tests/test_gpu_parity.py)."""
        dev = self.dynamic_emb.device
        V, d = self.dynamic_emb.shape
        R2 = self.emb_rel.shape[0]
        a = _lib.addr
        f32 = torch.float32
        layers = list(self.rgcn.layers)
        lorentz = isinstance(layers[0], LorentzRGCNLayer)
        emb = self.emb_rel.detach()
        s1, tw, x1, h2 = (torch.empty(V, d, device=dev, dtype=f32) for _ in range(4))
        r1, n2 = torch.empty(V, device=dev, dtype=f32), torch.empty(V, device=dev, dtype=f32)
        pre = self._gru_pre_initial()
        desc, keep = self._phase_desc(r_static, wg, bg, w_r, b_r)
        keep += [s1, tw, x1, h2, r1, n2]  # tensors the launches read (profiling replays them)
        desc.s1, desc.tw, desc.x1, desc.r1, desc.h2, desc.n2 = a(s1), a(tw), a(x1), a(r1), a(h2), a(n2)
        lib_call = _lib.lib().regcn_timestep_phase_f32

        def call(dp, phase, stream):
            if PHASE_CAPTURE is not None:  # profiling: a replayable launch of this phase (bench.py)
                snap = type(desc).from_buffer_copy(desc)
                PHASE_CAPTURE["ABC"[phase]] = (lambda: _lib.check(lib_call(ctypes.byref(snap), phase, _lib.stream()),
                                                                  "regcn_timestep_phase_f32"), keep + [snap])
            if PHASE_TRACE is None:
                return lib_call(dp, phase, stream)
            # profiling: per-workgroup {start, end} stamps of this launch (tools/phasetrace.py)
            n_gru = ((R2 + 15) // 16) * ((d + 15) // 16)
            n_zero = ((sum(desc.prev_n_pos[i] for i in range(desc.n_prev)) if desc.memo_h else
                       0 if desc.skip_zero_rows else V - desc.n_pos) + 15) // 16
            n_copy = min(128, (V * d // 4 + 2047) // 2048) if desc.memo_h else 0  # timestep.hip launcher
            pad8 = lambda n: (n + 7) // 8 * 8  # noqa: E731  (segments padded for the XCD grouping)
            kinds = ([("zero", pad8(n_zero)), ("gru_x", pad8(n_gru)), ("pos_rows", 2 * ((desc.n_pos + 15) // 16)),
                      ("copy", n_copy)]
                     if phase == 0 else
                     [("pos_tiles", desc.n_pos_tiles), ("zero", n_zero)]
                     + ([("gru_pre", n_gru)] if phase == 1 and desc.gru_pre else []))
            buf = torch.zeros(TRACE_SLOTS * max(1, sum(n for _, n in kinds)), dtype=torch.int64, device=dev)
            _lib.call("regcn_set_trace", _lib.addr(buf, torch.int64))
            rc = lib_call(dp, phase, stream)
            _lib.call("regcn_set_trace", None)
            PHASE_TRACE.append(("ABC"[phase], kinds, buf))
            return rc

        h_prev = emb
        history_embs = []
        g_list = [g.to(dev) for g in g_list]
        T = len(g_list)
        outs = [(torch.empty(V, d, device=dev, dtype=f32), torch.empty(V, d, device=dev, dtype=f32),
                 torch.empty(V, device=dev, dtype=f32)) for _ in g_list]
        scope = self.__dict__.get("_scope")
        if scope is not None and scope["memo"] is not None and scope["T"] == T:
            memo = scope["memo"]  # computed once for the batch (shared_parameter_states)
        else:
            memo = self._pristine_states(T, c_val, desc) if self.memo_pristine and T <= _lib.MAX_WINDOW else None
        if memo is not None:
            keep.append(memo)
        split = memo is None and self.split_zero_rows
        desc.skip_zero_rows = int(split)
        cur = torch.cuda.current_stream(dev)
        side = self._side(dev, 2) if split and self.zero_rows_side_stream else cur
        if split:
            zd = _lib.ChainDesc()
            zd.T, zd.d, zd.c = 1, d, desc.c
            zd.w_evolve0, zd.w_evolve1 = desc.w_evolve[0], desc.w_evolve[1]
            zd.w_skip1, zd.b_skip1 = desc.w_skip1, desc.b_skip1
            for f in ("w_g", "b_g", "r_static", "w_r", "b_r", "eps_r", "beta", "layer_norm", "residual", "c_radius"):
                setattr(zd, "step_" + f, getattr(desc, "step_" + f))
            zero_call = _lib.lib().regcn_zero_step_f32
        for t, g in enumerate(g_list):
            wk = g.work()
            x0, r0 = tangent_of(self.h, c_val)
            h0 = torch.empty(R2, d, device=dev, dtype=f32)
            out = outs[t]
            if memo is not None:  # pristine rows: memoised; rows without in-edges: the earlier in-edge rows
                desc.memo_h, desc.memo_x, desc.memo_r = (a(m) for m in memo[t])
                desc.n_prev = t
                for i, gp in enumerate(g_list[:t]):
                    wp = gp.work()
                    desc.prev_rows[i], desc.prev_rowptr[i] = a(wp["rows"], torch.int32), a(wp["rowptr"], torch.int32)
                    desc.prev_n_pos[i] = gp.n_pos
            desc.rowptr, desc.col_src, desc.col_type = (a(wk[k], torch.int32) for k in ("rowptr", "col_src", "col_type"))
            desc.norm, desc.budget = a(wk["norm"]), g.budget
            desc.tiles, desc.n_pos_tiles = a(wk["tiles"], torch.int32), g.n_pos_tiles
            desc.item_ptr = a(wk["item_ptr"], torch.int32)
            desc.item_src = a(wk["item_src"], torch.int32) if wk["item_src"].numel() else None
            desc.item_tl = a(wk["item_tl"], torch.int32) if wk["item_tl"].numel() else None
            desc.rows, desc.n_pos, desc.V = a(wk["rows"], torch.int32), g.n_pos, V
            desc.x0, desc.r0 = a(x0), a(r0)
            keep.extend([x0, r0, h0, out])
            desc.step_h_out, desc.step_x_out, desc.step_r_out = a(out[0]), a(out[1]), a(out[2])
            if split and V > g.n_pos:
                # Z: this snapshot's rows without in-edges through the timestep, on the side
                # stream: after timestep t - 1 (its input x0), joined before timestep t + 1
                zd.rows, zd.grid_bound = a(wk["rows"], torch.int32) + 4 * g.n_pos, V - g.n_pos
                zd.x0 = a(x0)
                zd.h_out[0], zd.x_out[0], zd.r_out[0] = a(out[0]), a(out[1]), a(out[2])
                if PHASE_CAPTURE is not None:  # profiling: a replayable launch (bench.py)
                    zsnap = type(zd).from_buffer_copy(zd)
                    PHASE_CAPTURE["Z"] = (lambda: _lib.check(zero_call(ctypes.byref(zsnap), _lib.stream()),
                                                             "regcn_zero_step_f32"), keep + [zsnap])
                if side is not cur:
                    side.wait_stream(cur)
                with torch.cuda.stream(side):
                    if PHASE_TRACE is not None:  # profiling: per-workgroup stamps (tools/phasetrace.py)
                        n_zt = (V - g.n_pos + 15) // 16
                        zbuf = torch.zeros(TRACE_SLOTS * n_zt, dtype=torch.int64, device=dev)
                        _lib.call("regcn_set_trace", _lib.addr(zbuf, torch.int64))
                    _lib.check(zero_call(ctypes.byref(zd), _lib.stream()), "regcn_zero_step_f32")
                    if PHASE_TRACE is not None:
                        _lib.call("regcn_set_trace", None)
                        PHASE_TRACE.append(("Z", [("zero_step", n_zt)], zbuf))
            # A: GRU x-half (relation means of x0 over this snapshot's r_to_e spans)
            x_mean = relation_context(x0, g, R2) if g.rel_max_span > REL_INLINE_MAX_SPAN else None
            desc.gru_rel_idx = a(wk["rel_idx"], torch.int32) if wk["rel_idx"].numel() else None
            desc.gru_rel_start, desc.gru_rel_count = a(wk["rel_start"], torch.int32), a(wk["rel_count"])
            desc.gru_x_mean = a(x_mean)
            keep.extend([x_mean, pre, h_prev])
            desc.gru_h_prev, desc.gru_pre, desc.gru_h_out = a(h_prev.detach().contiguous()), a(pre), a(h0)
            desc.rel = None
            _lib.check(call(ctypes.byref(desc), 0, _lib.stream()), "regcn_timestep_phase_f32(A)")
            if self.layer_norm:
                h0 = F.normalize(h0)
            # B: layer 0 of the in-edge rows (messages use h_0), layer 1 of the others, and the
            # next timestep's GRU pre-half (h_prev = h_0)
            desc.rel = a(h0)
            if g.n_heavy:
                agg0 = _heavy_aggregate(desc.agg_mode, g, x0, r0, h0, layers[0].weight.detach().contiguous()
                                        if lorentz else None, desc.num_bases, desc.gamma, c_val)
                desc.agg[0] = a(agg0)
                keep.append(agg0)
            pre_next = torch.empty(R2, 4, d, device=dev, dtype=f32) if t + 1 < len(g_list) else None
            keep.append(pre_next)
            desc.gru_h_prev, desc.gru_pre, desc.gru_h_out = a(h0), a(pre_next), None
            _lib.check(call(ctypes.byref(desc), 1, _lib.stream()), "regcn_timestep_phase_f32(B)")
            if g.n_heavy:
                agg1 = _heavy_aggregate(desc.agg_mode, g, x1, r1, h0, layers[1].weight.detach().contiguous()
                                        if lorentz else None, desc.num_bases, desc.gamma, c_val)
                desc.agg[1] = a(agg1)
                keep.append(agg1)
            _lib.check(call(ctypes.byref(desc), 2, _lib.stream()), "regcn_timestep_phase_f32(C)")
            if split and side is not cur:
                cur.wait_stream(side)  # the timestep's rows are complete
            desc.agg[0] = desc.agg[1] = None
            pre, h_prev = pre_next, h0
            self.h_0 = h0
            self.h = attach(out[0], out[1], out[2], c_val)
            history_embs.append(self.h)
        return history_embs, None, self.h_0, [], []

    def _pristine_states(self, T, c_val, desc, cache=True, x_init=None):
        """[(h, x, r) after timestep k for k < T] of a row that receives no message in
        timesteps 0..k: F^(k+1)(initial state) with F = layer 0 and layer 1 without messages
        (W_evolve, the skip gate) and the timestep (time gate, radius evolution), all rows in
        one regcn_cold_chain_f32 launch (the zero-tile op sequence: same bits).  A function of
        the parameters only: computed once per parameter version and per T."""
        pe = self.dynamic_emb
        key = (T, float(c_val), bool(self.layer_norm), bool(self.use_residual_evolution), float(self.radius_min),
               float(self.radius_max)) + tuple((p.data_ptr(), p._version) for p in self.parameters()) \
            + tuple((b.data_ptr(), b._version) for b in self.buffers())
        hit = self.__dict__.get("_pristine_cache")
        if cache and hit is not None and hit[0] == key and self.param_caches:
            return hit[1]
        V, d = pe.shape
        dev = pe.device
        f32 = torch.float32
        states = [(torch.empty(V, d, device=dev, dtype=f32), torch.empty(V, d, device=dev, dtype=f32),
                   torch.empty(V, device=dev, dtype=f32)) for _ in range(T)]
        rows = torch.arange(V, device=dev, dtype=torch.int32)
        n_rows = torch.full((1,), V, device=dev, dtype=torch.int32)
        if x_init is None:  # the initial state forward() just attached
            x_init, _ = tangent_of(self.h, c_val)
        a = _lib.addr
        ch = _lib.ChainDesc()
        ch.rows, ch.n_rows = a(rows, torch.int32), a(n_rows, torch.int32)
        ch.T, ch.d, ch.grid_bound, ch.c, ch.x0 = T, d, V, desc.c, a(x_init)
        ch.w_evolve0, ch.w_evolve1 = desc.w_evolve[0], desc.w_evolve[1]
        ch.w_skip1, ch.b_skip1 = desc.w_skip1, desc.b_skip1
        for f in ("w_g", "b_g", "r_static", "w_r", "b_r", "eps_r", "beta", "layer_norm", "residual", "c_radius"):
            setattr(ch, "step_" + f, getattr(desc, "step_" + f))
        for t, (ho, xo, ro) in enumerate(states):
            ch.h_out[t], ch.x_out[t], ch.r_out[t] = a(ho), a(xo), a(ro)
        if PHASE_CAPTURE is not None:  # profiling: a replayable launch (bench.py)
            chs = type(ch).from_buffer_copy(ch)
            PHASE_CAPTURE["chain"] = (lambda: _lib.call_desc("regcn_cold_chain_f32", chs), [chs, rows, n_rows, states])
        _lib.call_desc("regcn_cold_chain_f32", ch)
        if not cache:  # the caller keeps the launch's operands alive (shared_parameter_states)
            self.__dict__["_chain_operands"] = (rows, n_rows)
            return states
        if not torch.cuda.is_current_stream_capturing():
            _lib.publish()
            self.__dict__["_pristine_cache"] = (key, states)
        else:
            self.__dict__.setdefault("_capture_keep", []).append((rows, n_rows, states))
        return states

    def _final_embedding(self, emb, c_val):
        if self.layer_norm:
            return HyperbolicOps.layer_norm_roundtrip(emb, c_val)  # :926-929 / :992-995
        return emb

    def _forward_last_h(self, test_graph, static_graph, use_cuda):
        """forward for predict: only the last history state's Poincare rows are read, so the
        earlier timesteps' h need not be written (the fused per-layer path skips them; their x
        and |h| are written as always).  The history list's earlier entries are not valid h."""
        self.__dict__["_last_h_only"] = True
        try:
            return self.forward(test_graph, static_graph, use_cuda)
        finally:
            self.__dict__.pop("_last_h_only", None)

    def predict(self, test_graph, num_rels, static_graph, test_triplets, use_cuda):
        """hyperbolic_model.py:892-939."""
        with torch.no_grad():
            c_val = self._c_float()
            dev = self.dynamic_emb.device
            if self.fused_decoders and test_triplets.device == dev and \
                    roth_pair_fusable(self.decoder_ob, self.rdecoder, self.dynamic_emb):
                # one stream end to end: encoder, then the two-launch RotH/RotHRel front
                # (queries + candidates + all_triples, then both scores in one launch)
                evolve_embs, _, r_emb, _, _ = self._forward_last_h(test_graph, static_graph, use_cuda)
                last = evolve_embs[-1]
                if getattr(last, "_regcn_owner", None) is not None:  # owner partition: rank-local rows
                    last._regcn_owner[0].complete_rows(last)
                embedding = self._final_embedding(last, c_val)
                if self.run_analysis:  # hyperbolic_model.py:932-933
                    _ana.log_embedding(self, embedding, "predict_embeddings", c_val)
                return roth_pair_predict(self.decoder_ob, self.rdecoder, embedding, r_emb, test_triplets, num_rels)
            # the query triples do not depend on the encoder: on a HIP device they are built on
            # the side stream while the encoder runs (joined in _decode_both)
            side = self._side(dev) if dev.type == "cuda" and test_triplets.device == dev else None
            if side is not None:
                side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                # [o, r, s] (hyperbolic_model.py:917); flip() keeps the index on the device
                inverse_test_triplets = test_triplets.flip(1)
                inverse_test_triplets[:, 1] = inverse_test_triplets[:, 1] + num_rels
                all_triples = torch.cat((test_triplets, inverse_test_triplets))
            if side is not None:
                built = torch.cuda.Event()
                built.record(side)
            evolve_embs, _, r_emb, _, _ = self._forward_last_h(test_graph, static_graph, use_cuda)
            if side is not None:
                torch.cuda.current_stream(dev).wait_event(built)
                all_triples.record_stream(torch.cuda.current_stream(dev))
            last = evolve_embs[-1]
            if getattr(last, "_regcn_owner", None) is not None:  # owner partition: rank-local rows
                last._regcn_owner[0].complete_rows(last)
            embedding = self._final_embedding(last, c_val)
            if self.run_analysis:  # hyperbolic_model.py:932-933
                _ana.log_embedding(self, embedding, "predict_embeddings", c_val)
            at = all_triples.to(embedding.device)
            score, score_rel = self._decode_both(embedding, r_emb, at)
            return all_triples, score, score_rel

    def predict_ranks(self, test_graph, num_rels, static_graph, test_triplets, use_cuda, all_ans=None,
                      all_ans_r=None):
        """predict followed by the evaluation loop's two get_total_rank calls
        (hyperbolic_main.py:111-121, rgcn/utils.py:136-166).  Returns (all_triples,
        (rank, filtered rank) of the entity queries, (rank, filtered rank) of the relation
        queries), 1-based.  When the snapshots are partitioned over several ranks
        (parallel.ShardedGraph), each rank scores only its contiguous slice of the entity
        candidates (parallel.CandidateShard): the target score on every rank, the per-slice
        count of candidates above it (raw and with the slice's part of the time-aware filter),
        ONE all-reduce of 2B counts -- no rank scores all N entities (SURVEY.md §8(e) decoder).
        The relation decoder (2R candidates) runs replicated.  Ranks equal the unsharded ones."""
        from . import ranking
        from .parallel import CandidateShard, ShardedGraph
        sharded = [g for g in test_graph if isinstance(g, ShardedGraph) and g.world > 1]
        if not sharded:
            all_tr, score, score_rel = self.predict(test_graph, num_rels, static_graph, test_triplets, use_cuda)
            r_e, f_e = ranking.get_total_rank(all_tr, score, all_ans, 1000, 0)[2:]
            r_r, f_r = ranking.get_total_rank(all_tr, score_rel, all_ans_r, 1000, 1)[2:]
            return all_tr, (r_e, f_e), (r_r, f_r)
        dec = self.decoder_ob
        if not hasattr(dec, "_query") or dec.use_relation_specific_curvature:
            raise NotImplementedError("candidate-sharded ranking needs a MuRP / RotH / AttH decoder with the proxy "
                                      "distance score")
        sg = sharded[-1]
        with torch.no_grad():
            c_val = self._c_float()
            # every rank reads only its own rows of the last state (its candidates) plus the
            # queries' rows, fetched below: the last layer's exchange is skipped
            self.__dict__["_owner_rows_only"] = True
            try:
                embs, _, r_emb, _, _ = self.forward(test_graph, static_graph, use_cuda)
            finally:
                self.__dict__.pop("_owner_rows_only", None)
            inv = test_triplets.flip(1)
            inv[:, 1] = inv[:, 1] + num_rels
            at = torch.cat([test_triplets, inv])
            last = embs[-1]
            if getattr(last, "_regcn_owner", None) is not None:
                # owner partition: every rank holds its own rows of the last state; the queries'
                # subjects / objects come from their owners (one all_reduce of 2B x d rows)
                sg.fetch_rows(last, test_triplets[:, [0, 2]].reshape(-1))
            emb = self._final_embedding(last, c_val).contiguous()
            q = dec._query(emb, r_emb, at)
            N = emb.shape[0]
            shard = CandidateShard(N, sg.rank, sg.world, sg.group, ranges=sg.candidate_ranges(N))
            kw = dict(scale=dec.score_scale_raw, margin=dec.score_margin, raw_scale=True)
            # the candidates' entity_bias[n] as in the full scoring; the decoder's extra
            # entity_bias[s] shifts a whole query row alike, so the ranks do not see it
            bias = dec.entity_bias.detach() if dec.entity_bias is not None else None
            ts = shard.target_scores(q, emb, bias, at[:, 2], dec.c, **kw)
            # without answer lists (a benchmark step) no host round trip: raw ranks only
            fp, fi = ranking._filter_csr(at, all_ans, False) if all_ans is not None else (None, None)
            r_e, f_e = shard.range_ranks(q, emb, bias, dec.c, ts, fp, fi, **kw)
            score_rel = self.rdecoder.forward(emb, r_emb, at, mode="test")
            if all_ans_r is None:
                r_r = f_r = ranking.ranks(score_rel, at[:, 1])[0]
            else:
                r_r, f_r = ranking.get_total_rank(at, score_rel, all_ans_r, 1000, 1)[2:]
        return at, (r_e, f_e), (r_r, f_r)

    def _side(self, dev, k=1):
        """Side stream k of the calling stream (1: relation decoder / query triples / cold
        rows): keyed by the current stream, so predicts issued on different streams (e.g.
        independent samples in flight together) never share a side stream."""
        streams = self.__dict__.setdefault("_side_streams", {})
        key = (torch.cuda.current_stream(dev).cuda_stream, k)
        side = streams.get(key)
        if side is None or side.device != dev:
            side = streams[key] = torch.cuda.Stream(dev)
        return side

    def _decode_both(self, embedding, r_emb, at):
        """Entity and relation decoders are independent: on a HIP device the relation
        decoder runs on a side stream, so each uses the CUs the other's ~30-workgroup
        launches leave idle (also inside a captured HIP graph: a fork/join)."""
        if embedding.device.type != "cuda":
            return (self.decoder_ob.forward(embedding, r_emb, at, mode="test"),
                    self.rdecoder.forward(embedding, r_emb, at, mode="test"))
        main = torch.cuda.current_stream(embedding.device)
        side = self._side(embedding.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            score_rel = self.rdecoder.forward(embedding, r_emb, at, mode="test")
        score = self.decoder_ob.forward(embedding, r_emb, at, mode="test")
        main.wait_stream(side)
        score_rel.record_stream(main)
        return score, score_rel

    def _loss_curvature(self):
        """The curvature get_loss hands the decoders (hyperbolic_model.py:972-973): the learned
        tensor while training it (its gradient flows through the decoders), else the float."""
        c_val = self._c_float()
        if self.learn_curvature and self._wants_grad():
            return self.get_curvature()
        return c_val

    def get_loss(self, glist, triples, static_graph, use_cuda, query_time=None):
        """hyperbolic_model.py:941-1088 (forward value of the four losses)."""
        c_val = self._loss_curvature()
        self.decoder_ob.c = c_val
        self.rdecoder.c = c_val
        evolve_embs, static_emb, r_emb, _, _ = self.forward(glist, static_graph, use_cuda)
        pre_emb = self._final_embedding(evolve_embs[-1], c_val)
        losses = self._decode_losses(pre_emb, r_emb, triples, c_val)
        if self.run_analysis:  # hyperbolic_model.py:1076-1086
            _ana.record_losses(self, *losses)
        return losses

    def get_loss_batches(self, glist, triples, static_graph, use_cuda, batch_size, query_time=None,
                         combine=None, group_budget=1 << 28):
        """One snapshot's training losses and gradients with ONE encoder forward (SURVEY.md
        §8(f) f1).  hyperbolic_main.py:585-598 recomputes the encoder for every
        `batch_size` mini-batch, back-propagates each mini-batch loss and steps once per
        snapshot, so the gradient is the sum over mini-batches.  Here the final entity and
        relation embeddings are cut from the graph as leaf tensors; the decoders run once over
        a GROUP of consecutive mini-batches (every mini-batch while the group's B x |V|
        backward coefficient block stays under `group_budget` floats), each mini-batch's loss
        is the mean of its own queries' losses (the decoder losses are per query, the radius
        loss per mini-batch over its own distinct entities), the group back-propagates
        sum_b combine(losses_b) once, and one backward through the encoder follows with the
        accumulated embedding gradients.  Same gradients as the reference loop; the dropout
        masks are drawn once per group (decoders) and once per snapshot (encoder) instead of
        once per mini-batch.

        `combine(le, lr, ls, lrad)` -> the scalar each mini-batch back-propagates
        (default: the plain sum).  Returns the detached [(loss_ent, loss_rel, loss_static,
        loss_radius), ...] per mini-batch."""
        if combine is None:
            combine = lambda le, lr, ls, lrad: le + lr + ls.sum() + lrad  # noqa: E731
        c_val = self._loss_curvature()
        evolve_embs, static_emb, r_emb, _, _ = self.forward(glist, static_graph, use_cuda)
        pre_emb = self._final_embedding(evolve_embs[-1], c_val)
        grad_on = torch.is_grad_enabled()
        srcs = (pre_emb, r_emb) + ((c_val,) if torch.is_tensor(c_val) else ())
        # a learned curvature is cut too: the decoders accumulate its gradient into the leaf,
        # which the final encoder backward carries on to log_c
        cut = [t.detach().requires_grad_(grad_on and t.requires_grad) for t in srcs]
        c_dec = cut[2] if len(cut) > 2 else c_val
        self.decoder_ob.c = c_dec
        self.rdecoder.c = c_dec
        parts = []
        n = triples.shape[0]
        per_group = self._loss_group_size(batch_size, group_budget, torch.is_tensor(c_dec) and c_dec.requires_grad)
        for g0 in range(0, n, per_group * batch_size):
            g1 = min(n, g0 + per_group * batch_size)
            vecs = self._decode_losses(cut[0], cut[1], triples[g0:g1], c_dec, batch_size=batch_size)
            per_batch = list(zip(*(v.unbind(0) for v in vecs)))  # views; one stack in backward
            if grad_on:
                total = sum(combine(*losses) for losses in per_batch)
                if total.requires_grad:
                    total.backward()
            parts.extend(tuple(t.detach() for t in losses) for losses in per_batch)
            if self.run_analysis:  # one loss-components entry per mini-batch (hyperbolic_model.py:1076-1086)
                for losses in per_batch:
                    _ana.record_losses(self, *losses)
        roots = [(src, leaf.grad) for src, leaf in zip(srcs, cut)
                 if src.requires_grad and leaf.grad is not None]
        if roots:
            torch.autograd.backward([r[0] for r in roots], [r[1] for r in roots])
        return parts

    # per-element footprint (in fp32 words) of the B x N decoder blocks a group holds: the fused
    # fp32 CE keeps one backward coefficient per element; the dense fp64 paths (a learned
    # curvature's _ce_c_term S matrix and its retained pair terms, the relation-specific
    # curvature's arctanh-distance score) keep fp64 intermediates and their autograd state,
    # measured at ~150 B per element (tests/test_gpu_training.py::test_loss_batches_memory_dense_fp64)
    DENSE_FP64_WORDS = 40

    def _loss_group_size(self, batch_size, group_budget, learned_c):
        """Mini-batches decoded together by get_loss_batches: the group's B x max(|V|, 2R)
        blocks (queries and their inverses) stay under `group_budget` fp32 words."""
        words = 1
        if learned_c or self.use_relation_specific_curvature:
            words = self.DENSE_FP64_WORDS
        per_elem = 2 * batch_size * max(self.num_ents, 2 * self.num_rels) * words
        return max(1, int(group_budget) // max(1, per_elem))

    def _decode_losses(self, pre_emb, r_emb, triples, c_val, batch_size=None):
        """hyperbolic_model.py:996-1073: decoders on the final embedding + radius loss.
        batch_size: `triples` holds consecutive mini-batches of that size (the last may be
        short); returns each loss as a vector with one entry per mini-batch, each the value
        the mini-batch alone gives (the decoders' per-query losses averaged over the
        mini-batch's queries by one small product, the radius loss over its own entities)."""
        dev = pre_emb.device
        n = triples.shape[0]
        nb = 1 if batch_size is None else (n + batch_size - 1) // batch_size
        inverse_triples = triples.flip(1)
        inverse_triples[:, 1] = inverse_triples[:, 1] + self.num_rels
        all_triples = torch.cat([triples, inverse_triples]).to(dev)
        if batch_size is None:
            red, avg, seg = "mean", None, None
        else:
            # query i (and its inverse n + i) belongs to mini-batch i // batch_size
            seg = torch.arange(n, device=dev) // batch_size
            seg = torch.cat([seg, seg])
            onehot = (seg.unsqueeze(0) == torch.arange(nb, device=dev).unsqueeze(1)).float()
            avg = onehot / onehot.sum(1, keepdim=True)  # nb x 2n, rows average a mini-batch
            red = "none"
        zero = torch.zeros(nb, device=dev) if batch_size is not None else torch.zeros(1, device=dev)
        loss_ent, loss_rel = zero, zero
        loss_static = torch.zeros(nb, 1, device=dev) if batch_size is not None else torch.zeros(1, device=dev)
        if self.entity_prediction:
            if hasattr(self.decoder_ob, "loss"):
                loss_ent = self.decoder_ob.loss(pre_emb, r_emb, all_triples, reduction=red)
            else:
                scores_ob = self.decoder_ob.forward(pre_emb, r_emb, all_triples).view(-1, self.num_ents)
                loss_ent = F.cross_entropy(scores_ob, all_triples[:, 2], reduction=red)
            if avg is not None:
                loss_ent = avg @ loss_ent
        if self.relation_prediction:
            if hasattr(self.rdecoder, "loss"):
                loss_rel = self.rdecoder.loss(pre_emb, r_emb, all_triples, reduction=red)
            else:
                score_rel = self.rdecoder.forward(pre_emb, r_emb, all_triples, mode="train").view(-1, 2 * self.num_rels)
                loss_rel = F.cross_entropy(score_rel, all_triples[:, 1], reduction=red)
            if avg is not None:
                loss_rel = avg @ loss_rel
        # MSE over the batch's distinct entities (hyperbolic_model.py:1067-1073 takes
        # torch.unique of them): a membership mask over all entities instead, so the loss has
        # a static shape and no host synchronisation (unique's output size is data-dependent)
        diff = self._static_radius(float(c_val)) - self.radius_target.to(dev)
        ents = all_triples[:, 0::2]  # s and o (a view)
        if batch_size is None:
            seen = torch.zeros(self.num_ents, device=dev, dtype=torch.float32)
            seen.index_fill_(0, ents.reshape(-1), 1.0)
            loss_radius = self.radius_lambda * (seen * diff * diff).sum() / seen.sum()
        else:
            seen = torch.zeros(nb, self.num_ents, device=dev, dtype=torch.float32)
            seen.index_put_((seg.repeat_interleave(2), ents.reshape(-1)), torch.ones((), device=dev))
            loss_radius = self.radius_lambda * (seen @ (diff * diff)) / seen.sum(1)
        return loss_ent, loss_rel, loss_static, loss_radius

    def log_gradient_stats(self):
        """hyperbolic_model.py:1090-1108 (the total gradient norm, kept on the device)."""
        return _ana.gradient_stats(self)

    def get_training_summary(self):
        """hyperbolic_model.py:1110-1127."""
        return _ana.training_summary(self)
