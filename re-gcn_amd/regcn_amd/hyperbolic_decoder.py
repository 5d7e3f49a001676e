"""Hyperbolic decoders with HIP scoring (mirror of hyperbolic_src/hyperbolic_decoder.py).

The scoring half — `_chunked_hyperbolic_dist_score` and `_chunked_hyperbolic_ce_loss`,
same signatures — runs on the fp32-MFMA scorer (csrc/score.hip): one GEMM Q E^T plus a
per-pair epilogue that reproduces mobius_add(-q, e) / the arctanh distance without
expanding B x N x d.  The chunk sizes are accepted as tiling hints and do not change the
math (hyperbolic_decoder.py:104-106).  Query prologues (MuRP / RotH / AttH and their
relation variants) keep the reference's parameters and state_dict keys; their row maps
run on the HIP row kernels, their small projections on torch.  Forward only.
"""
import ctypes
import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.parameter import Parameter

from . import _lib
from . import autograd as _ag
from .hyperbolic_ops import HyperbolicOps
from .weights import packed_k4, packed_t

SCORE_SCALE_EPSILON = 1e-6
REL_CURVATURE_EPSILON = 1e-5
REL_CURVATURE_SAFETY_MARGIN = 0.999
REL_CURVATURE_INIT_RATIO = 0.95


def _softplus_inverse(x, eps=1e-12):
    return math.log(max(math.exp(float(x)) - 1.0, eps))


def _relation_curvature_theta_init(global_c):
    """hyperbolic_decoder.py:46-63."""
    if torch.is_tensor(global_c):
        global_c = global_c.detach().item()
    return _softplus_inverse(max(float(global_c) * REL_CURVATURE_INIT_RATIO, REL_CURVATURE_EPSILON))


def _clamp_relation_curvature(rel_c_raw, global_c, warmup_max=None):
    """hyperbolic_decoder.py:66-86."""
    # device scalars by fill kernels (new_full), not host copies: the step stays capturable
    g = global_c if torch.is_tensor(global_c) else rel_c_raw.new_full((), float(global_c))
    upper = REL_CURVATURE_SAFETY_MARGIN * g.to(rel_c_raw.device, rel_c_raw.dtype)
    if warmup_max is not None:
        upper = torch.min(upper, rel_c_raw.new_full((), float(warmup_max)))
    return torch.max(torch.min(rel_c_raw, upper), rel_c_raw.new_full((), REL_CURVATURE_EPSILON))


def _cf(c):
    return float(c.item()) if torch.is_tensor(c) else float(c)


def _scalar(v, like):
    """Device fp32 scalar tensor for the kernel (None -> None)."""
    if v is None:
        return None
    if torch.is_tensor(v):
        return v.detach().reshape(1).to(device=like.device, dtype=torch.float32).contiguous()
    return torch.full((1,), float(v), device=like.device, dtype=torch.float32)


def _score_operands(query, candidates, bias, score_scale, score_margin, query_curvature):
    q = query.detach().contiguous().float()
    e = candidates.detach().contiguous().float()
    b = bias.detach().contiguous().float() if bias is not None else None
    cr = query_curvature.detach().reshape(-1).contiguous().float() if query_curvature is not None else None
    return q, e, b, cr, _scalar(score_scale, q), _scalar(score_margin, q)


def _chunked_hyperbolic_dist_score(query, candidates, bias, c, q_chunk_size, c_chunk_size, score_scale=None,
                                   score_margin=0.0, query_curvature=None, use_hyperbolic_distance=False,
                                   _raw_scale=False):
    """hyperbolic_decoder.py:89-179 -> regcn_hyp_score_f32.  Returns (B, N).
    _raw_scale: score_scale is score_scale_raw; softplus + eps is applied on the device."""
    B, d = query.shape
    N = candidates.shape[0]
    q, e, b, cr, sc, mg = _score_operands(query, candidates, bias, score_scale, score_margin,
                                                    query_curvature if use_hyperbolic_distance else None)
    out = torch.empty(B, N, device=q.device, dtype=torch.float32)
    f = _lib.fptr
    flags = (_lib.SCORE_DIST if use_hyperbolic_distance else 0) | (_lib.SCORE_RAW_SCALE if _raw_scale else 0)
    _lib.call("regcn_hyp_score_f32", f(q, "query"), f(e, "candidates"), f(b), f(cr), f(sc), f(mg),
              B, N, d, _cf(c), flags, f(out), _lib.stream())
    return out


def _chunked_hyperbolic_ce_loss(query, candidates, target, c, c_chunk_size, candidate_bias=None, query_bias=None,
                                q_chunk_size=None, score_scale=None, score_margin=0.0, query_curvature=None,
                                use_hyperbolic_distance=False, reduction="mean"):
    """hyperbolic_decoder.py:182-307 -> regcn_hyp_ce_f32 (fused scores + log-sum-exp; the
    B x N logits are never materialised).  query_bias cancels in CE and is ignored (:204-205).
    reduction="none": the B per-query losses instead of their mean."""
    B, d = query.shape
    N = candidates.shape[0]
    if _ag.needs_grad(query, candidates, candidate_bias, score_scale, score_margin, query_curvature, c):
        if use_hyperbolic_distance and query_curvature is not None:  # --plus-relation-specific-curvature
            return _ag.hyp_dist_ce_loss(query, candidates, target, query_curvature, bias=candidate_bias,
                                        scale=score_scale, margin=score_margin, reduction=reduction)
        if use_hyperbolic_distance:
            raise NotImplementedError("the global-curvature arctanh-distance score has no caller in the reference "
                                      "(its decoders pass per-relation curvatures)")
        return _ag.hyp_ce_loss(query, candidates, target, c, bias=candidate_bias, scale=score_scale,
                               margin=score_margin, reduction=reduction)
    q, e, b, cr, sc, mg = _score_operands(query, candidates, candidate_bias, score_scale, score_margin,
                                                    query_curvature if use_hyperbolic_distance else None)
    tgt = target.to(device=q.device, dtype=torch.int32).contiguous()
    ws_bytes = _lib.lib().regcn_hyp_ce_workspace_bytes(B, N)
    ws = torch.empty((ws_bytes + 3) // 4, device=q.device, dtype=torch.float32)
    loss = torch.empty(B, device=q.device, dtype=torch.float32)
    f = _lib.fptr
    _lib.call("regcn_hyp_ce_f32", f(q, "query"), f(e, "candidates"), f(b), f(cr), f(sc), f(mg),
              _lib.iptr(tgt, "target"), B, N, d, _cf(c), int(bool(use_hyperbolic_distance)), f(ws), f(loss),
              _lib.stream())
    return loss if reduction == "none" else loss.mean()


def _grad_path(mod, *ts):
    """True when autograd must see the decoder (training): the fused eval-only query kernels
    are skipped for the differentiable op sequence."""
    return _ag.needs_grad(*ts) or (torch.is_grad_enabled() and any(p.requires_grad for p in mod.parameters()))


def givens_rotation(x, angles):
    """hyperbolic_decoder.py:1032-1051 (interleaved pairs)."""
    if torch.is_grad_enabled():
        fused = _ag.givens_rotation(x, angles)
        if fused is not None:
            return fused
    if angles.dim() == 1:
        angles = angles.unsqueeze(0).expand(x.shape[0], -1)
    x1, x2 = x[:, 0::2], x[:, 1::2]
    co, si = torch.cos(angles), torch.sin(angles)
    return torch.stack([co * x1 - si * x2, si * x1 + co * x2], dim=2).reshape(x.shape[0], x.shape[1])


def givens_reflection(x, angles):
    """hyperbolic_decoder.py:1392-1401."""
    if torch.is_grad_enabled():
        fused = _ag.givens_rotation(x, angles, reflect=True)
        if fused is not None:
            return fused
    if angles.dim() == 1:
        angles = angles.unsqueeze(0).expand(x.shape[0], -1)
    x1, x2 = x[:, 0::2], x[:, 1::2]
    co, si = torch.cos(angles), torch.sin(angles)
    return torch.stack([co * x1 + si * x2, si * x1 - co * x2], dim=2).reshape(x.shape[0], x.shape[1])


class _EntityDecoderBase(nn.Module):
    """Shared state of MuRP/RotH/AttH entity decoders (hyperbolic_decoder.py:662-731)."""

    def _init_common(self, num_entities, num_relations, embedding_dim, c, dropout, query_chunk_size,
                     candidate_chunk_size, score_scale_init, score_margin_init, use_entity_euclidean_bias,
                     use_relation_specific_curvature):
        self.num_entities, self.embedding_dim, self.c = num_entities, embedding_dim, c
        self.query_chunk_size, self.candidate_chunk_size = query_chunk_size, candidate_chunk_size
        self.num_relations = num_relations
        self.use_entity_euclidean_bias = use_entity_euclidean_bias
        self.use_relation_specific_curvature = use_relation_specific_curvature

    def _init_tail(self, num_entities, num_relations, c, score_scale_init, score_margin_init, dropout,
                   use_entity_euclidean_bias, use_relation_specific_curvature):
        if use_entity_euclidean_bias:
            self.entity_bias = nn.Parameter(torch.zeros(num_entities))
        else:
            self.register_parameter("entity_bias", None)
        if use_relation_specific_curvature:
            self.rel_curvature_raw = nn.Parameter(torch.full((num_relations,), _relation_curvature_theta_init(c)))
            self.rel_curvature_max = float(c)
        else:
            self.register_parameter("rel_curvature_raw", None)
            self.rel_curvature_max = None
        self.score_scale_raw = nn.Parameter(torch.tensor(float(score_scale_init)))
        self.score_margin = nn.Parameter(torch.tensor(float(score_margin_init)))
        self.dropout = nn.Dropout(dropout)

    def _score_scale(self):
        return F.softplus(self.score_scale_raw) + SCORE_SCALE_EPSILON

    def _relation_curvature(self, r_idx):
        if self.rel_curvature_raw is None:
            return None
        raw = F.softplus(self.rel_curvature_raw[torch.remainder(r_idx, self.num_relations)])
        return _clamp_relation_curvature(raw, self.c, self.rel_curvature_max)

    def set_relation_curvature_bounds(self, curvature_max=None):
        if curvature_max is not None:
            self.rel_curvature_max = float(curvature_max)

    def _query(self, entity_embedding, rel_embedding, triplets):
        raise NotImplementedError

    def forward(self, entity_embedding, rel_embedding, triplets, mode="train"):
        q = self._query(entity_embedding, rel_embedding, triplets)
        rel_c = self._relation_curvature(triplets[:, 1])
        scores = _chunked_hyperbolic_dist_score(
            q, entity_embedding, self.entity_bias, self.c, self.query_chunk_size, self.candidate_chunk_size,
            score_scale=self.score_scale_raw, score_margin=self.score_margin, query_curvature=rel_c,
            use_hyperbolic_distance=self.use_relation_specific_curvature, _raw_scale=True)
        if self.entity_bias is not None:
            scores = scores + self.entity_bias[triplets[:, 0]].unsqueeze(1)
        return scores

    def loss(self, entity_embedding, rel_embedding, triplets, reduction="mean"):
        q = self._query(entity_embedding, rel_embedding, triplets)
        rel_c = self._relation_curvature(triplets[:, 1])
        return _chunked_hyperbolic_ce_loss(
            q, entity_embedding, triplets[:, 2], self.c, self.candidate_chunk_size, candidate_bias=self.entity_bias,
            q_chunk_size=self.query_chunk_size, score_scale=self._score_scale(), score_margin=self.score_margin,
            query_curvature=rel_c, use_hyperbolic_distance=self.use_relation_specific_curvature,
            reduction=reduction)


class HyperbolicMuRP(_EntityDecoderBase):
    """hyperbolic_decoder.py:647-817."""

    def __init__(self, num_entities, num_relations, embedding_dim, c=0.01, dropout=0.0, query_chunk_size=128,
                 candidate_chunk_size=256, init_scale=1e-3, score_scale_init=1.0, score_margin_init=1.0,
                 use_entity_euclidean_bias=False, use_relation_specific_curvature=False):
        super().__init__()
        self._init_common(num_entities, num_relations, embedding_dim, c, dropout, query_chunk_size,
                          candidate_chunk_size, score_scale_init, score_margin_init, use_entity_euclidean_bias,
                          use_relation_specific_curvature)
        self.rot_proj = nn.Linear(embedding_dim, embedding_dim)
        self.trans_proj = nn.Linear(embedding_dim, embedding_dim)
        for lin in (self.rot_proj, self.trans_proj):
            nn.init.uniform_(lin.weight, -init_scale, init_scale)
            nn.init.zeros_(lin.bias)
        self._init_tail(num_entities, num_relations, c, score_scale_init, score_margin_init, dropout,
                        use_entity_euclidean_bias, use_relation_specific_curvature)

    def _query(self, ent, rel, trip):
        """hyperbolic_decoder.py:745-764."""
        c = self.c
        r_idx = trip[:, 1]
        s_emb = HyperbolicOps.project_to_ball(ent[trip[:, 0]], c)
        s_tan = self.dropout(HyperbolicOps.log_map_zero(s_emb, c))
        rr = rel[r_idx]
        rot_s = HyperbolicOps.exp_map_zero((_ag.linear(self.rot_proj, rr) * s_tan).contiguous(), c)
        t_r = HyperbolicOps.exp_map_zero(_ag.linear(self.trans_proj, rr).contiguous(), c)
        return HyperbolicOps.mobius_add(HyperbolicOps.project_to_ball(rot_s, c),
                                        HyperbolicOps.project_to_ball(t_r, c), c)


class HyperbolicRotH(_EntityDecoderBase):
    """hyperbolic_decoder.py:931-1138."""

    def __init__(self, num_entities, num_relations, embedding_dim, c=0.01, dropout=0.0, query_chunk_size=128,
                 candidate_chunk_size=256, init_scale=1e-3, score_scale_init=1.0, score_margin_init=1.0,
                 use_entity_euclidean_bias=False, use_relation_specific_curvature=False):
        super().__init__()
        assert embedding_dim % 2 == 0, "embedding_dim must be even (required for Givens rotation)"
        self._init_common(num_entities, num_relations, embedding_dim, c, dropout, query_chunk_size,
                          candidate_chunk_size, score_scale_init, score_margin_init, use_entity_euclidean_bias,
                          use_relation_specific_curvature)
        self.half_dim = embedding_dim // 2
        self.rot_proj = nn.Linear(embedding_dim, self.half_dim)
        self.trans_proj = nn.Linear(embedding_dim, embedding_dim)
        self.reshape_fc1 = nn.Linear(embedding_dim, embedding_dim)
        self.reshape_fc2 = nn.Linear(embedding_dim, embedding_dim)
        for lin in (self.rot_proj, self.trans_proj, self.reshape_fc1, self.reshape_fc2):
            nn.init.uniform_(lin.weight, -init_scale, init_scale)
            nn.init.zeros_(lin.bias)
        self._init_tail(num_entities, num_relations, c, score_scale_init, score_margin_init, dropout,
                        use_entity_euclidean_bias, use_relation_specific_curvature)

    givens_rotation = staticmethod(givens_rotation)

    def _reshape_tangent(self, x):
        return x + _ag.linear(self.reshape_fc2, F.relu(_ag.linear(self.reshape_fc1, x)))

    def _query(self, ent, rel, trip):
        """hyperbolic_decoder.py:1065-1085.  In eval mode (dropout = identity) one HIP launch
        (regcn_roth_query_f32); with active dropout the same op sequence on torch."""
        if not (self.training and self.dropout.p > 0) and not getattr(self, "_torch_query", False) \
                and not _grad_path(self, ent, rel):
            d = ent.shape[1]
            q = torch.empty(trip.shape[0], d, device=ent.device, dtype=torch.float32)
            f = _lib.fptr
            lins = (self.reshape_fc1, self.reshape_fc2, self.rot_proj, self.trans_proj)
            ws = [packed_t(l.weight) for l in lins]
            bs = [l.bias.detach() for l in lins]
            _lib.call("regcn_roth_query_f32", f(ent.contiguous(), "entity_embedding"),
                      f(rel.detach().contiguous(), "rel_embedding"), _lib.dptr(trip.contiguous(), torch.int64),
                      trip.shape[0], trip.shape[0], 0, f(ws[0]), f(bs[0]), f(ws[1]), f(bs[1]), f(ws[2]), f(bs[2]),
                      f(ws[3]), f(bs[3]), d, _cf(self.c), f(q), _lib.stream())
            return q
        c = self.c
        r_idx = trip[:, 1]
        s_emb = HyperbolicOps.project_to_ball(ent[trip[:, 0]], c)
        s_tan = self._reshape_tangent(self.dropout(HyperbolicOps.log_map_zero(s_emb, c)))
        rr = rel[r_idx]  # one gather (and one index backward) for both projections
        rot_s = HyperbolicOps.exp_map_zero(givens_rotation(s_tan, _ag.linear(self.rot_proj, rr)).contiguous(), c)
        t_r = HyperbolicOps.exp_map_zero(_ag.linear(self.trans_proj, rr).contiguous(), c)
        return HyperbolicOps.mobius_add(HyperbolicOps.project_to_ball(rot_s, c),
                                        HyperbolicOps.project_to_ball(t_r, c), c)


class HyperbolicAttH(_EntityDecoderBase):
    """hyperbolic_decoder.py:1283-1512."""

    def __init__(self, num_entities, num_relations, embedding_dim, c=0.01, dropout=0.0, query_chunk_size=128,
                 candidate_chunk_size=256, init_scale=1e-3, score_scale_init=1.0, score_margin_init=1.0,
                 use_entity_euclidean_bias=False, use_relation_specific_curvature=False):
        super().__init__()
        assert embedding_dim % 2 == 0, "embedding_dim must be even"
        self._init_common(num_entities, num_relations, embedding_dim, c, dropout, query_chunk_size,
                          candidate_chunk_size, score_scale_init, score_margin_init, use_entity_euclidean_bias,
                          use_relation_specific_curvature)
        self.half_dim = embedding_dim // 2
        self.rot_proj = nn.Linear(embedding_dim, self.half_dim)
        self.ref_proj = nn.Linear(embedding_dim, self.half_dim)
        self.trans_proj = nn.Linear(embedding_dim, embedding_dim)
        self.attn_proj = nn.Linear(embedding_dim, 2 * embedding_dim)
        for lin in (self.rot_proj, self.ref_proj, self.trans_proj, self.attn_proj):
            nn.init.uniform_(lin.weight, -init_scale, init_scale)
            nn.init.zeros_(lin.bias)
        self._init_tail(num_entities, num_relations, c, score_scale_init, score_margin_init, dropout,
                        use_entity_euclidean_bias, use_relation_specific_curvature)

    givens_rotation = staticmethod(givens_rotation)
    givens_reflection = staticmethod(givens_reflection)

    def _query(self, ent, rel, trip):
        """hyperbolic_decoder.py:1414-1448."""
        c = self.c
        r_idx = trip[:, 1]
        s_emb = HyperbolicOps.project_to_ball(ent[trip[:, 0]], c)
        s_tan = self.dropout(HyperbolicOps.log_map_zero(s_emb, c))
        rr = rel[r_idx]
        rot_s = givens_rotation(s_tan, _ag.linear(self.rot_proj, rr))
        ref_s = givens_reflection(s_tan, _ag.linear(self.ref_proj, rr))
        a_r = torch.sigmoid(torch.sum(_ag.linear(self.attn_proj, rr) * torch.cat([s_tan, rr], dim=-1), dim=-1, keepdim=True))
        mixed = HyperbolicOps.exp_map_zero((a_r * rot_s + (1.0 - a_r) * ref_s).contiguous(), c)
        t_r = HyperbolicOps.exp_map_zero(_ag.linear(self.trans_proj, rr).contiguous(), c)
        return HyperbolicOps.mobius_add(HyperbolicOps.project_to_ball(mixed, c),
                                        HyperbolicOps.project_to_ball(t_r, c), c)


def roth_pair_fusable(dec, rdec, ent):
    """The RotH entity decoder and the RotHRel relation decoder of an eval predict can run as
    the two-launch front (roth_pair_predict): eval-mode dropout, proxy score (no relation
    curvature), no per-query entity bias, one curvature, d <= 256 on a HIP device."""
    return (isinstance(dec, HyperbolicRotH) and isinstance(rdec, HyperbolicRotHRel) and ent.is_cuda
            and not (dec.training and dec.dropout.p > 0) and not (rdec.training and rdec.dropout.p > 0)
            and not _grad_path(dec, ent) and not _grad_path(rdec, ent)
            and dec.entity_bias is None and not dec.use_relation_specific_curvature
            and _cf(dec.c) == _cf(rdec.c) and ent.shape[1] <= 256 and ent.shape[1] % 4 == 0)


def roth_pair_queries(dec, rdec, ent, rel, test_triplets, num_rels):
    """regcn_roth_queries_f32: the entity (RotH) and relation (RotHRel) queries of a predict,
    the relation candidates exp0(R) and all_triples, in one launch.  Returns
    (all_triples, q_ent, q_rel, cand)."""
    n, d = test_triplets.shape[0], ent.shape[1]
    B, R2 = 2 * n, rel.shape[0]
    dev = ent.device
    f32 = torch.float32
    q_ent = torch.empty(B, d, device=dev, dtype=f32)
    q_rel = torch.empty(B, d, device=dev, dtype=f32)
    cand = torch.empty(R2, d, device=dev, dtype=f32)
    all_triples = torch.empty(B, 3, device=dev, dtype=torch.int64)
    a = _lib.addr
    qd = _lib.RothQueriesDesc()
    qd.ent, qd.rel, qd.trip = a(ent), a(rel), a(test_triplets, torch.int64)
    qd.n_test, qd.B, qd.num_rels, qd.d, qd.c = n, B, int(num_rels), d, _cf(dec.c)
    qd.w1, qd.b1 = a(packed_k4(dec.reshape_fc1.weight)), a(dec.reshape_fc1.bias.detach())
    qd.w2, qd.b2 = a(packed_k4(dec.reshape_fc2.weight)), a(dec.reshape_fc2.bias.detach())
    qd.w_rot, qd.b_rot = a(packed_k4(dec.rot_proj.weight)), a(dec.rot_proj.bias.detach())
    qd.w_trans, qd.b_trans = a(packed_k4(dec.trans_proj.weight)), a(dec.trans_proj.bias.detach())
    qd.rw1, qd.rb1 = a(packed_k4(rdec.reshape_fc1.weight)), a(rdec.reshape_fc1.bias.detach())
    qd.rw2, qd.rb2 = a(packed_k4(rdec.reshape_fc2.weight)), a(rdec.reshape_fc2.bias.detach())
    qd.global_rot = a(rdec.global_rot.detach())
    qd.q_ent, qd.q_rel, qd.n_cand, qd.cand = a(q_ent), a(q_rel), R2, a(cand)
    qd.all_triples = a(all_triples, torch.int64)
    _lib.check(_lib.lib().regcn_roth_queries_f32(ctypes.byref(qd), _lib.stream()), "regcn_roth_queries_f32")
    return all_triples, q_ent, q_rel, cand


def roth_pair_scores(dec, rdec, ent, q_ent, q_rel, cand):
    """regcn_hyp_score_jobs_f32: the entity scores (q_ent against every entity) and the
    relation scores (q_rel against the candidates, + rel_bias) in one launch."""
    B, d = q_ent.shape
    dev = ent.device
    score = torch.empty(B, ent.shape[0], device=dev, dtype=torch.float32)
    score_rel = torch.empty(B, cand.shape[0], device=dev, dtype=torch.float32)
    a = _lib.addr
    jobs = (_lib.ScoreJob * 2)()
    for j, (q, cd, bias, m, out) in enumerate(((q_ent, ent, None, dec, score),
                                               (q_rel, cand, rdec.rel_bias, rdec, score_rel))):
        jobs[j].q, jobs[j].cand, jobs[j].bias = a(q), a(cd), a(bias.detach() if bias is not None else None)
        jobs[j].scale = a(_scalar(m.score_scale_raw, q))
        jobs[j].margin = a(_scalar(m.score_margin, q))
        jobs[j].B, jobs[j].N, jobs[j].d, jobs[j].c = B, cd.shape[0], d, _cf(dec.c)
        jobs[j].flags, jobs[j].out = _lib.SCORE_RAW_SCALE, a(out)
    _lib.check(_lib.lib().regcn_hyp_score_jobs_f32(jobs, 2, _lib.stream()), "regcn_hyp_score_jobs_f32")
    return score, score_rel


def roth_pair_predict(dec, rdec, ent, rel, test_triplets, num_rels, parts=None):
    """The decoders of HyperbolicRecurrentRGCN.predict (hyperbolic_model.py:915-939) for RotH +
    RotHRel in two launches on the calling stream (roth_pair_queries, roth_pair_scores).
    Returns (all_triples, score, score_rel), the values of torch.cat + decoder_ob.forward +
    rdecoder.forward.  `parts` (a dict) receives the queries and the relation candidates."""
    ent = ent.contiguous()
    all_triples, q_ent, q_rel, cand = roth_pair_queries(dec, rdec, ent, rel.detach().contiguous(),
                                                        test_triplets.contiguous(), num_rels)
    score, score_rel = roth_pair_scores(dec, rdec, ent, q_ent, q_rel, cand)
    if parts is not None:
        parts.update(q_ent=q_ent, q_rel=q_rel, cand=cand)
    return all_triples, score, score_rel


class _RelDecoderBase(nn.Module):
    def _score_scale(self):
        return F.softplus(self.score_scale_raw) + SCORE_SCALE_EPSILON

    def forward(self, entity_embedding, rel_embedding, triplets, mode="train"):
        q = self._query(entity_embedding, triplets)
        rel_hyp = HyperbolicOps.exp_map_zero(rel_embedding.contiguous(), self.c)
        return _chunked_hyperbolic_dist_score(q, rel_hyp, self.rel_bias, self.c, self.query_chunk_size,
                                              self.candidate_chunk_size, **self._score_kw())

    def loss(self, entity_embedding, rel_embedding, triplets, reduction="mean"):
        q = self._query(entity_embedding, triplets)
        rel_hyp = HyperbolicOps.exp_map_zero(rel_embedding.contiguous(), self.c)
        return _chunked_hyperbolic_ce_loss(q, rel_hyp, triplets[:, 1], self.c, self.candidate_chunk_size,
                                           candidate_bias=self.rel_bias, q_chunk_size=self.query_chunk_size,
                                           reduction=reduction, **self._score_kw())

    def _score_kw(self):
        return dict(score_scale=self._score_scale(), score_margin=self.score_margin)


class HyperbolicMuRPRel(_RelDecoderBase):
    """hyperbolic_decoder.py:820-928 (no score scale/margin in the reference)."""

    def __init__(self, num_relations, embedding_dim, c=0.01, dropout=0.0, query_chunk_size=128,
                 candidate_chunk_size=256):
        super().__init__()
        self.num_relations, self.embedding_dim, self.c = num_relations, embedding_dim, c
        self.query_chunk_size, self.candidate_chunk_size = query_chunk_size, candidate_chunk_size
        self.W_s = nn.Parameter(torch.Tensor(embedding_dim, embedding_dim))
        nn.init.xavier_uniform_(self.W_s)
        self.W_o = nn.Parameter(torch.Tensor(embedding_dim, embedding_dim))
        nn.init.xavier_uniform_(self.W_o)
        self.rel_bias = nn.Parameter(torch.zeros(num_relations * 2))
        self.dropout = nn.Dropout(dropout)

    def _score_kw(self):
        return {}

    def _query(self, ent, trip):
        c = self.c
        s_tan = self.dropout(HyperbolicOps.log_map_zero(ent[trip[:, 0]], c))
        o_tan = self.dropout(HyperbolicOps.log_map_zero(ent[trip[:, 2]], c))
        return HyperbolicOps.exp_map_zero((torch.mm(s_tan, self.W_s) + torch.mm(o_tan, self.W_o)).contiguous(), c)


class HyperbolicRotHRel(_RelDecoderBase):
    """hyperbolic_decoder.py:1141-1280."""

    def __init__(self, num_relations, embedding_dim, c=0.01, dropout=0.0, query_chunk_size=128,
                 candidate_chunk_size=256, init_scale=1e-3, score_scale_init=1.0, score_margin_init=1.0):
        super().__init__()
        assert embedding_dim % 2 == 0, "embedding_dim must be even"
        self.num_relations, self.embedding_dim, self.half_dim, self.c = num_relations, embedding_dim, \
            embedding_dim // 2, c
        self.query_chunk_size, self.candidate_chunk_size = query_chunk_size, candidate_chunk_size
        self.global_rot = nn.Parameter(torch.Tensor(self.half_dim))
        nn.init.uniform_(self.global_rot, -math.pi, math.pi)
        self.reshape_fc1 = nn.Linear(embedding_dim, embedding_dim)
        self.reshape_fc2 = nn.Linear(embedding_dim, embedding_dim)
        for lin in (self.reshape_fc1, self.reshape_fc2):
            nn.init.uniform_(lin.weight, -init_scale, init_scale)
            nn.init.zeros_(lin.bias)
        self.rel_bias = nn.Parameter(torch.zeros(num_relations * 2))
        self.score_scale_raw = nn.Parameter(torch.tensor(float(score_scale_init)))
        self.score_margin = nn.Parameter(torch.tensor(float(score_margin_init)))
        self.dropout = nn.Dropout(dropout)

    givens_rotation = staticmethod(givens_rotation)

    def forward(self, entity_embedding, rel_embedding, triplets, mode="train"):
        """Eval mode: queries and the exp0 candidates in one launch (regcn_roth_rel_query_f32),
        then the scorer with softplus(score_scale_raw) applied on the device."""
        if (self.training and self.dropout.p > 0) or _grad_path(self, entity_embedding, rel_embedding):
            return super().forward(entity_embedding, rel_embedding, triplets, mode)
        B, d = triplets.shape[0], entity_embedding.shape[1]
        R2 = rel_embedding.shape[0]
        q = torch.empty(B, d, device=entity_embedding.device, dtype=torch.float32)
        cand = torch.empty(R2, d, device=entity_embedding.device, dtype=torch.float32)
        f = _lib.fptr
        _lib.call("regcn_roth_rel_query_f32", f(entity_embedding.contiguous(), "entity_embedding"),
                  _lib.dptr(triplets.contiguous(), torch.int64), B, B, 0, f(packed_t(self.reshape_fc1.weight)),
                  f(self.reshape_fc1.bias.detach()), f(packed_t(self.reshape_fc2.weight)),
                  f(self.reshape_fc2.bias.detach()), f(self.global_rot.detach()),
                  f(rel_embedding.detach().contiguous(), "rel_embedding"), R2, d, _cf(self.c), f(q), f(cand),
                  _lib.stream())
        return _chunked_hyperbolic_dist_score(q, cand, self.rel_bias, self.c, self.query_chunk_size,
                                              self.candidate_chunk_size, score_scale=self.score_scale_raw,
                                              score_margin=self.score_margin, _raw_scale=True)

    def _query(self, ent, trip):
        """hyperbolic_decoder.py:1223-1234."""
        c = self.c
        o_emb = ent[trip[:, 2]].contiguous()
        s_tan = self.dropout(HyperbolicOps.log_map_zero(ent[trip[:, 0]], c))
        s_tan = s_tan + _ag.linear(self.reshape_fc2, F.relu(_ag.linear(self.reshape_fc1, s_tan)))
        rot_s = HyperbolicOps.exp_map_zero(givens_rotation(s_tan, self.global_rot).contiguous(), c)
        return HyperbolicOps.mobius_add(-rot_s, o_emb, c)


class HyperbolicAttHRel(_RelDecoderBase):
    """hyperbolic_decoder.py:1515-1679."""

    def __init__(self, num_relations, embedding_dim, c=0.01, dropout=0.0, query_chunk_size=128,
                 candidate_chunk_size=256, init_scale=1e-3, score_scale_init=1.0, score_margin_init=1.0):
        super().__init__()
        assert embedding_dim % 2 == 0, "embedding_dim must be even"
        self.num_relations, self.embedding_dim, self.half_dim, self.c = num_relations, embedding_dim, \
            embedding_dim // 2, c
        self.query_chunk_size, self.candidate_chunk_size = query_chunk_size, candidate_chunk_size
        self.global_rot = nn.Parameter(torch.Tensor(self.half_dim))
        nn.init.uniform_(self.global_rot, -math.pi, math.pi)
        self.global_ref = nn.Parameter(torch.Tensor(self.half_dim))
        nn.init.uniform_(self.global_ref, -math.pi, math.pi)
        self.attn_weight = nn.Parameter(torch.Tensor(2 * embedding_dim))
        nn.init.uniform_(self.attn_weight, -init_scale, init_scale)
        self.rel_bias = nn.Parameter(torch.zeros(num_relations * 2))
        self.score_scale_raw = nn.Parameter(torch.tensor(float(score_scale_init)))
        self.score_margin = nn.Parameter(torch.tensor(float(score_margin_init)))
        self.dropout = nn.Dropout(dropout)

    givens_rotation = staticmethod(givens_rotation)
    givens_reflection = staticmethod(givens_reflection)

    def _query(self, ent, trip):
        """hyperbolic_decoder.py:1605-1628."""
        c = self.c
        o_emb = ent[trip[:, 2]].contiguous()
        s_tan = self.dropout(HyperbolicOps.log_map_zero(ent[trip[:, 0]], c))
        o_tan = HyperbolicOps.log_map_zero(o_emb, c)
        a = torch.sigmoid(torch.mv(torch.cat([s_tan, o_tan], dim=-1), self.attn_weight)).unsqueeze(1)
        mixed = a * givens_rotation(s_tan, self.global_rot) + (1.0 - a) * givens_reflection(s_tan, self.global_ref)
        rot = HyperbolicOps.exp_map_zero(mixed.contiguous(), c)
        return HyperbolicOps.mobius_add(-rot, o_emb, c)


class HyperbolicConvTransE(nn.Module):
    """hyperbolic_decoder.py:310-413 (tangent-space ConvTransE; host torch convolution,
    HIP log0; the all-entity product is a plain GEMM)."""

    def __init__(self, num_entities, embedding_dim, c=0.01, input_dropout=0.0, hidden_dropout=0.0,
                 feature_map_dropout=0.0, channels=50, kernel_size=3):
        super().__init__()
        self.num_entities, self.embedding_dim, self.c = num_entities, embedding_dim, c
        self.inp_drop = nn.Dropout(input_dropout)
        self.hidden_drop = nn.Dropout(hidden_dropout)
        self.feature_map_drop = nn.Dropout(feature_map_dropout)
        self.conv1 = nn.Conv1d(2, channels, kernel_size, stride=1, padding=int(math.floor(kernel_size / 2)))
        self.bn0 = nn.BatchNorm1d(2)
        self.bn1 = nn.BatchNorm1d(channels)
        self.bn2 = nn.BatchNorm1d(embedding_dim)
        self.fc = nn.Linear(embedding_dim * channels, embedding_dim)
        self.register_parameter("b", Parameter(torch.zeros(num_entities)))

    def forward(self, entity_embedding, rel_embedding, triplets, mode="train"):
        et = HyperbolicOps.log_map_zero(entity_embedding.contiguous(), self.c)
        et = 0.9 * torch.tanh(et) + 0.1 * et
        B = len(triplets)
        x = torch.cat([et[triplets[:, 0]].unsqueeze(1), rel_embedding[triplets[:, 1]].unsqueeze(1)], 1)
        x = self.feature_map_drop(F.relu(_ag.batch_norm(self.bn1, self.conv1(self.inp_drop(_ag.batch_norm(self.bn0, x))))))
        x = self.hidden_drop(_ag.linear(self.fc, x.view(B, -1)))
        if B > 1:
            x = _ag.batch_norm(self.bn2, x)
        return torch.mm(F.relu(x), et.transpose(1, 0)) + self.b


class HyperbolicConvTransR(nn.Module):
    """hyperbolic_decoder.py:416-510."""

    def __init__(self, num_relations, embedding_dim, c=0.01, input_dropout=0.0, hidden_dropout=0.0,
                 feature_map_dropout=0.0, channels=50, kernel_size=3):
        super().__init__()
        self.num_relations, self.embedding_dim, self.c = num_relations, embedding_dim, c
        self.inp_drop = nn.Dropout(input_dropout)
        self.hidden_drop = nn.Dropout(hidden_dropout)
        self.feature_map_drop = nn.Dropout(feature_map_dropout)
        self.conv1 = nn.Conv1d(2, channels, kernel_size, stride=1, padding=int(math.floor(kernel_size / 2)))
        self.bn0 = nn.BatchNorm1d(2)
        self.bn1 = nn.BatchNorm1d(channels)
        self.bn2 = nn.BatchNorm1d(embedding_dim)
        self.fc = nn.Linear(embedding_dim * channels, embedding_dim)
        self.register_parameter("b", Parameter(torch.zeros(num_relations * 2)))

    def forward(self, entity_embedding, rel_embedding, triplets, mode="train"):
        et = HyperbolicOps.log_map_zero(entity_embedding.contiguous(), self.c)
        et = 0.9 * torch.tanh(et) + 0.1 * et
        B = len(triplets)
        x = torch.cat([et[triplets[:, 0]].unsqueeze(1), et[triplets[:, 2]].unsqueeze(1)], 1)
        x = self.feature_map_drop(F.relu(_ag.batch_norm(self.bn1, self.conv1(self.inp_drop(_ag.batch_norm(self.bn0, x))))))
        x = _ag.batch_norm(self.bn2, self.hidden_drop(_ag.linear(self.fc, x.view(B, -1))))
        return torch.mm(F.relu(x), rel_embedding.transpose(1, 0)) + self.b
