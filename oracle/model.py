"""Recurrent encoders and decoders restated (oracle; test infrastructure only).

State comes from a state_dict carrying the reference's key names
(SURVEY.md Appendix B), so a product model's `state_dict()` or a golden
fixture's `sd_*` arrays feed it directly.
"""
import math

import torch
import torch.nn.functional as F

from . import ops
from .layers import euclid_union_layer, lorentz_layer, union_layer

SCORE_EPS = 1e-6


def gru_cell(x, h, sd, prefix):
    """torch.nn.GRUCell semantics (gate order r, z, n), used at
    hyperbolic_model.py:408, :818, :823 and src/rrgcn.py:133, :169, :173."""
    gi = F.linear(x, sd[prefix + "weight_ih"], sd[prefix + "bias_ih"])
    gh = F.linear(h, sd[prefix + "weight_hh"], sd[prefix + "bias_hh"])
    ir, iz, inn = gi.chunk(3, 1)
    hr, hz, hn = gh.chunk(3, 1)
    r = torch.sigmoid(ir + hr)
    z = torch.sigmoid(iz + hz)
    n = torch.tanh(inn + r * hn)
    return (1 - z) * n + z * h


def rel_context(ht, g, num_rels2):
    """hyperbolic_model.py:802-812 / src/rrgcn.py:161-166: x_input[r] = mean of the
    rows of entities touching r in this snapshot; absent relations stay 0."""
    x_input = torch.zeros(num_rels2, ht.shape[1], dtype=ht.dtype)
    temp = ht[torch.as_tensor(g["r_to_e"]).long()]
    for (a, b), r in zip(g["r_len"], g["uniq_r"]):
        x_input[int(r)] = torch.mean(temp[int(a):int(b)], dim=0)
    return x_input


def static_radius(sd, cfg):
    """hyperbolic_model.py:715-720."""
    r = torch.clamp(sd["radius_static"], min=cfg["radius_min"], max=cfg["radius_max"])
    return torch.clamp(r, max=1.0 / math.sqrt(cfg["c"]) - 1e-6)


def radius_evolution(h, r_static, sd, cfg, stats=None):
    """TemporalRadiusEvolution.forward, hyperbolic_ops.py:395-435 (`stats`: a dict to receive
    its last_evolution_stats, :426-434)."""
    c = cfg["c"]
    t = ops.log0(h, c)
    delta = F.linear(t, sd["temporal_radius_evolution.radius_mlp.weight"],
                     sd["temporal_radius_evolution.radius_mlp.bias"]).squeeze(-1)
    delta = torch.clamp(delta, -cfg["radius_epsilon"], cfg["radius_epsilon"]).unsqueeze(-1)
    dyn = ops.get_radius(h).unsqueeze(-1)
    beta = cfg["radius_anchor_beta"]
    base = beta * r_static.unsqueeze(-1) + (1.0 - beta) * dyn
    if stats is not None:
        stats.update(delta_mean=delta.mean().item(), delta_std=delta.std().item(),
                     dynamic_radius_mean=dyn.mean().item(), static_radius_mean=r_static.mean().item(),
                     base_radius_mean=base.mean().item(), anchor_beta=beta, epsilon=cfg["radius_epsilon"])
    return ops.apply_radius(h, base + delta, c)


def hyperbolic_forward(sd, cfg, glist, analysis=None):
    """HyperbolicRecurrentRGCN.forward, hyperbolic_model.py:722-890 (eval, no static
    graph, no EST).  Returns (history_embs, h_0).  `analysis` (a dict, the --run-analysis
    path): receives "gates" (each timestep's time_weight, :852-856), "time_gate_values"
    (their means) and "evolution" (the last radius-evolution stats, hyperbolic_ops.py:426-434)."""
    c, ln = cfg["c"], cfg["layer_norm"]
    R2 = sd["emb_rel"].shape[0]
    dyn = sd["dynamic_emb"]
    h = ops.exp0(F.normalize(dyn) if ln else dyn, c)                       # :779-780
    h = ops.apply_radius(h, static_radius(sd, cfg), c)                     # :782
    embs, h0 = [], None
    for i, g in enumerate(glist):
        ht = ops.log0(h, c)                                                # :802
        x_in = torch.cat([sd["emb_rel"], rel_context(ht, g, R2)], dim=1)
        h0 = gru_cell(x_in, sd["emb_rel"] if i == 0 else h0, sd, "relation_gru.")
        h0 = F.normalize(h0) if ln else h0                                 # :819, :824
        cur = h
        prev = None
        for li in range(cfg["n_layers"]):
            p = "rgcn.layers.%d." % li
            skip = None
            if cfg.get("skip_connect") and li > 0 and (p + "skip_weight") in sd:
                skip = (sd[p + "skip_weight"], sd[p + "skip_bias"], prev)
            if cfg["encoder"] == "hyperbolic_uvrgcn":
                new = union_layer(g, cur, h0, sd[p + "weight_neighbor"], sd[p + "loop_weight"],
                                  sd[p + "evolve_loop_weight"], c, cfg["radius_msg_gamma"])
            elif cfg["encoder"] == "lgcn":
                nb = min(cfg["n_bases"], R2) if cfg["n_bases"] > 0 else R2
                new = lorentz_layer(g, cur, h0, sd[p + "weight"], sd[p + "loop_weight"],
                                    sd[p + "evolve_loop_weight"], c, nb, skip=skip)
            else:
                raise NotImplementedError(cfg["encoder"])
            prev, cur = cur, new
        cur = ops.project(cur, c)                                          # :829
        if ln:
            cur = ops.exp0(F.normalize(ops.log0(cur, c)), c)               # :832-835
        ct = torch.clamp(ops.log0(cur, c), -10.0, 10.0)                    # :841-846
        pt = torch.clamp(ops.log0(h, c), -10.0, 10.0)
        tw = torch.sigmoid(torch.mm(pt, sd["time_gate_weight"]) + sd["time_gate_bias"])
        if analysis is not None:
            analysis.setdefault("gates", []).append(tw)
            analysis.setdefault("time_gate_values", []).append(tw.mean().item())
        h = ops.project(ops.exp0(tw * ct + (1 - tw) * pt, c), c)           # :859-860
        sr = static_radius(sd, cfg)
        if cfg.get("use_residual_evolution", True):
            h = radius_evolution(h, sr, sd, cfg,
                                 None if analysis is None else analysis.setdefault("evolution", {}))  # :866-867
        else:
            h = ops.apply_radius(h, sr, c)                                 # :869
        embs.append(h)
    return embs, h0


# ----------------------------------------------------------------------------- decoders

def dist_score(q, cand, bias, c, scale=None, margin=0.0, c_r=None, use_dist=False, chunk=64):
    """_chunked_hyperbolic_dist_score, hyperbolic_decoder.py:89-179, chunked over
    queries only (the chunking does not change the math, :104-106)."""
    B, d = q.shape
    N = cand.shape[0]
    out = q.new_zeros(B, N)
    for a in range(0, B, chunk):
        b = min(B, a + chunk)
        qe = q[a:b].unsqueeze(1).expand(b - a, N, d).reshape(-1, d)
        ce = cand.unsqueeze(0).expand(b - a, N, d).reshape(-1, d)
        if use_dist:
            if c_r is not None:                                            # :146-161
                ceff = c_r[a:b].reshape(-1, 1, 1).expand(b - a, N, 1).reshape(-1, 1).to(q.dtype)
                sc = torch.sqrt(ceff + SCORE_EPS)
                x2 = torch.sum(qe * qe, -1, keepdim=True)
                y2 = torch.sum(ce * ce, -1, keepdim=True)
                xy = torch.sum(qe * ce, -1, keepdim=True)
                num = (1 - 2 * ceff * xy + ceff * y2) * (-qe) + (1 - ceff * x2) * ce
                den = 1 - 2 * ceff * xy + (ceff ** 2) * x2 * y2
                n = torch.norm(num / (den + SCORE_EPS), p=2, dim=-1, keepdim=True).clamp(min=SCORE_EPS)
                n = torch.min(n, 1.0 / (sc + SCORE_EPS) - SCORE_EPS)
                dist = (2.0 / (sc + SCORE_EPS)) * torch.atanh((sc * n).clamp(max=1.0 - SCORE_EPS))
            else:
                dist = ops.hyperbolic_distance(qe, ce, c)                  # :163
            blk = margin - dist.reshape(b - a, N)
        else:
            diff = ops.mobius_add(-qe, ce, c)                              # :166-168
            blk = margin - torch.sum(diff ** 2, dim=-1).reshape(b - a, N)
        if scale is not None:
            blk = scale * blk
        if bias is not None:
            blk = blk + bias.unsqueeze(0)
        out[a:b] = blk
    return out


def ce_loss(q, cand, target, c, bias=None, scale=None, margin=0.0, c_r=None, use_dist=False):
    """_chunked_hyperbolic_ce_loss, hyperbolic_decoder.py:182-307 == cross entropy of
    the full logits (query_bias cancels and is ignored, :204-205)."""
    logits = dist_score(q, cand, bias, c, scale, margin, c_r, use_dist)
    return F.cross_entropy(logits, target.long())


def givens_rotation(x, ang):
    """hyperbolic_decoder.py:1032-1051 (interleaved pairs)."""
    if ang.dim() == 1:
        ang = ang.unsqueeze(0).expand(x.shape[0], -1)
    x1, x2 = x[:, 0::2], x[:, 1::2]
    co, si = torch.cos(ang), torch.sin(ang)
    return torch.stack([co * x1 - si * x2, si * x1 + co * x2], 2).reshape(x.shape)


def givens_reflection(x, ang):
    """hyperbolic_decoder.py:1392-1401."""
    if ang.dim() == 1:
        ang = ang.unsqueeze(0).expand(x.shape[0], -1)
    x1, x2 = x[:, 0::2], x[:, 1::2]
    co, si = torch.cos(ang), torch.sin(ang)
    return torch.stack([co * x1 + si * x2, si * x1 - co * x2], 2).reshape(x.shape)


def _lin(sd, p, x):
    return F.linear(x, sd[p + ".weight"], sd[p + ".bias"])


def _scale(sd, p):
    return F.softplus(sd[p + "score_scale_raw"]) + SCORE_EPS


def _rel_curvature(sd, p, r_idx, c, num_rel2):
    """hyperbolic_decoder.py:66-86, :1015-1022 (warmup bound = constructor c)."""
    key = p + "rel_curvature_raw"
    if key not in sd:
        return None
    raw = F.softplus(sd[key][torch.remainder(r_idx, num_rel2)])
    upper = torch.min(torch.tensor(0.999 * c), torch.tensor(float(c)))
    return torch.max(torch.min(raw, upper), torch.tensor(1e-5))


def entity_decoder(name, sd, emb, rel, trip, c):
    """HyperbolicMuRP/RotH/AttH.forward (hyperbolic_decoder.py:733-779, :1053-1099,
    :1403-1462) and HyperbolicConvTransE.forward (:360-413), eval mode."""
    p = "decoder_ob."
    s_idx, r_idx = trip[:, 0].long(), trip[:, 1].long()
    if name == "hyperbolic_convtranse":
        return _conv_decoder(sd, p, emb, rel, trip, c, relation=False)
    s_emb = ops.project(emb[s_idx], c)
    s_tan = ops.log0(s_emb, c)
    rr = rel[r_idx]
    if name == "roth":
        s_tan = s_tan + _lin(sd, p + "reshape_fc2", F.relu(_lin(sd, p + "reshape_fc1", s_tan)))
        q0 = ops.exp0(givens_rotation(s_tan, _lin(sd, p + "rot_proj", rr)), c)
    elif name == "murp":
        q0 = ops.exp0(_lin(sd, p + "rot_proj", rr) * s_tan, c)
    elif name == "atth":
        rot = givens_rotation(s_tan, _lin(sd, p + "rot_proj", rr))
        ref = givens_reflection(s_tan, _lin(sd, p + "ref_proj", rr))
        a = torch.sigmoid(torch.sum(_lin(sd, p + "attn_proj", rr) * torch.cat([s_tan, rr], -1),
                                    -1, keepdim=True))
        q0 = ops.exp0(a * rot + (1.0 - a) * ref, c)
    else:
        raise NotImplementedError(name)
    t_r = ops.project(ops.exp0(_lin(sd, p + "trans_proj", rr), c), c)
    q = ops.mobius_add(ops.project(q0, c), t_r, c)
    nrel2 = sd[p + "rel_curvature_raw"].shape[0] if (p + "rel_curvature_raw") in sd else 1
    c_r = _rel_curvature(sd, p, r_idx, c, nrel2)
    bias = sd.get(p + "entity_bias")
    sc = dist_score(q, emb, bias, c, _scale(sd, p), sd[p + "score_margin"], c_r,
                    use_dist=c_r is not None)
    if bias is not None:
        sc = sc + bias[s_idx].unsqueeze(1)
    return sc


def relation_decoder(name, sd, emb, rel, trip, c):
    """HyperbolicMuRPRel/RotHRel/AttHRel.forward (hyperbolic_decoder.py:859-895,
    :1211-1247, :1593-1639) and HyperbolicConvTransR.forward (:464-510), eval mode."""
    p = "rdecoder."
    if name == "hyperbolic_convtranse":
        return _conv_decoder(sd, p, emb, rel, trip, c, relation=True)
    s_emb, o_emb = emb[trip[:, 0].long()], emb[trip[:, 2].long()]
    s_tan = ops.log0(s_emb, c)
    rel_hyp = ops.exp0(rel, c)
    if name == "murp":
        q = ops.exp0(torch.mm(s_tan, sd[p + "W_s"]) + torch.mm(ops.log0(o_emb, c), sd[p + "W_o"]), c)
        return dist_score(q, rel_hyp, sd[p + "rel_bias"], c)
    if name == "roth":
        s_tan = s_tan + _lin(sd, p + "reshape_fc2", F.relu(_lin(sd, p + "reshape_fc1", s_tan)))
        rot = ops.exp0(givens_rotation(s_tan, sd[p + "global_rot"]), c)
    elif name == "atth":
        o_tan = ops.log0(o_emb, c)
        a = torch.sigmoid(torch.mv(torch.cat([s_tan, o_tan], -1), sd[p + "attn_weight"])).unsqueeze(1)
        rot = ops.exp0(a * givens_rotation(s_tan, sd[p + "global_rot"])
                       + (1.0 - a) * givens_reflection(s_tan, sd[p + "global_ref"]), c)
    else:
        raise NotImplementedError(name)
    q = ops.mobius_add(-rot, o_emb, c)
    return dist_score(q, rel_hyp, sd[p + "rel_bias"], c, _scale(sd, p), sd[p + "score_margin"])


def _bn(x, sd, p):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"],
                        sd[p + ".bias"], False, 0.0, 1e-5)


def _conv_decoder(sd, p, emb, rel, trip, c, relation, hyperbolic=True):
    """Conv decoders in eval mode: hyperbolic_decoder.py:360-510 (hyperbolic=True) and
    src/decoder.py:29-100 (hyperbolic=False)."""
    if hyperbolic:
        ent = ops.log0(emb, c)
        ent = 0.9 * torch.tanh(ent) + 0.1 * ent                           # :379
    else:
        ent = torch.tanh(emb)
    B = trip.shape[0]
    e1 = ent[trip[:, 0].long()].unsqueeze(1)
    other = ent[trip[:, 2].long()].unsqueeze(1) if relation else rel[trip[:, 1].long()].unsqueeze(1)
    x = _bn(torch.cat([e1, other], 1), sd, p + "bn0")
    x = F.conv1d(x, sd[p + "conv1.weight"], sd[p + "conv1.bias"], padding=1)
    x = F.relu(_bn(x, sd, p + "bn1"))
    x = F.linear(x.view(B, -1), sd[p + "fc.weight"], sd[p + "fc.bias"])
    if relation or B > 1:
        x = _bn(x, sd, p + "bn2")
    x = F.relu(x)
    if relation:
        out = torch.mm(x, rel.t())
    else:
        out = torch.mm(x, ent.t())
    if hyperbolic:
        out = out + sd[p + "b"]
    return out


def hyperbolic_predict(sd, cfg, glist, test_triplets):
    """HyperbolicRecurrentRGCN.predict, hyperbolic_model.py:892-939."""
    R = sd["emb_rel"].shape[0] // 2
    inv = test_triplets[:, [2, 1, 0]].clone()
    inv[:, 1] += R
    all_tr = torch.cat([test_triplets, inv])
    embs, h0 = hyperbolic_forward(sd, cfg, glist)
    emb = embs[-1]
    c = cfg["c"]
    if cfg["layer_norm"]:
        emb = ops.exp0(F.normalize(ops.log0(emb, c)), c)
    score = entity_decoder(cfg["decoder"], sd, emb, h0, all_tr, c)
    score_rel = relation_decoder(cfg["decoder"], sd, emb, h0, all_tr, c)
    return all_tr, score, score_rel, embs, h0


def euclid_forward(sd, cfg, glist):
    """RecurrentRGCN.forward, src/rrgcn.py:142-180 (uvrgcn, no static graph)."""
    ln = cfg["layer_norm"]
    R2 = sd["emb_rel"].shape[0]
    h = F.normalize(sd["dynamic_emb"]) if ln else sd["dynamic_emb"]
    embs, h0 = [], None
    for i, g in enumerate(glist):
        x_in = torch.cat([sd["emb_rel"], rel_context(h, g, R2)], dim=1)
        h0 = gru_cell(x_in, sd["emb_rel"] if i == 0 else h0, sd, "relation_cell_1.")
        h0 = F.normalize(h0) if ln else h0
        cur = h
        for li in range(cfg["n_layers"]):
            p = "rgcn.layers.%d." % li
            cur = euclid_union_layer(g, cur, h0, sd[p + "weight_neighbor"], sd[p + "loop_weight"],
                                     sd[p + "evolve_loop_weight"])
        cur = F.normalize(cur) if ln else cur
        tw = torch.sigmoid(torch.mm(h, sd["time_gate_weight"]) + sd["time_gate_bias"])
        h = tw * cur + (1 - tw) * h
        embs.append(h)
    return embs, h0


def euclid_predict(sd, cfg, glist, test_triplets):
    """RecurrentRGCN.predict, src/rrgcn.py:183-194 with ConvTransE/ConvTransR."""
    R = sd["emb_rel"].shape[0] // 2
    inv = test_triplets[:, [2, 1, 0]].clone()
    inv[:, 1] += R
    all_tr = torch.cat([test_triplets, inv])
    embs, h0 = euclid_forward(sd, cfg, glist)
    emb = F.normalize(embs[-1]) if cfg["layer_norm"] else embs[-1]
    score = _conv_decoder(sd, "decoder_ob.", emb, h0, all_tr, None, False, hyperbolic=False)
    score_rel = _conv_decoder(sd, "rdecoder.", emb, h0, all_tr, None, True, hyperbolic=False)
    return all_tr, score, score_rel, embs, h0


# ----------------------------------------------------------------------------- ranking

def sort_and_rank(score, target):
    """rgcn/utils.py:21-25 (0-based position of the target in a descending sort)."""
    _, idx = torch.sort(score, dim=1, descending=True)
    return torch.nonzero(idx == target.view(-1, 1), as_tuple=False)[:, 1].view(-1)


def filter_score(triples, score, all_ans, rel_predict=False):
    """rgcn/utils.py:51-75: other true answers of the same snapshot -> -1e7."""
    score = score.clone()
    for i, (h, r, t) in enumerate(triples.tolist()):
        if rel_predict:
            ans = set(all_ans[h][t])
            ans.discard(r)
        else:
            ans = set(all_ans[h][r])
            ans.discard(t)
        if ans:
            score[i, torch.tensor(sorted(ans))] = -10000000
    return score


def total_rank(triples, score, all_ans, rel_predict=False):
    """rgcn/utils.py:136-166 (batching by eval_bz does not change the result)."""
    col = 1 if rel_predict else 2
    target = triples[:, col]
    rank = sort_and_rank(score, target) + 1
    frank = sort_and_rank(filter_score(triples, score, all_ans, rel_predict), target) + 1
    return (torch.mean(1.0 / frank.float()).item(), torch.mean(1.0 / rank.float()).item(),
            rank, frank)


def answers_for_filter(snap, num_rels, rel_p=False):
    """rgcn/utils.py:237-283 (load_all_answers_for_filter for one snapshot)."""
    ans = {}
    for s, r, o in snap.tolist():
        if rel_p:
            ans.setdefault(s, {}).setdefault(o, set()).add(r)
            ans.setdefault(o, {}).setdefault(s, set()).add(r + num_rels)
        else:
            ans.setdefault(o, {}).setdefault(r + num_rels, set()).add(s)
            ans.setdefault(s, {}).setdefault(r, set()).add(o)
    return ans


def hyperbolic_get_loss(sd, cfg, glist, triples, radius_target):
    """HyperbolicRecurrentRGCN.get_loss, hyperbolic_model.py:941-1088 (dropout off, no static
    graph): entity and relation cross entropy over the triples and their inverses, the
    radius MSE on the entities in the batch.  Returns (loss_ent, loss_rel, loss_static,
    loss_radius)."""
    R = sd["emb_rel"].shape[0] // 2
    inv = triples[:, [2, 1, 0]].clone()
    inv[:, 1] += R
    all_tr = torch.cat([triples, inv])                                     # :982-985
    embs, h0 = hyperbolic_forward(sd, cfg, glist)
    emb = embs[-1]
    c = cfg["c"]
    if cfg["layer_norm"]:
        emb = ops.exp0(F.normalize(ops.log0(emb, c)), c)                   # :991-995
    le = F.cross_entropy(entity_decoder(cfg["decoder"], sd, emb, h0, all_tr, c), all_tr[:, 2].long())
    lr = F.cross_entropy(relation_decoder(cfg["decoder"], sd, emb, h0, all_tr, c), all_tr[:, 1].long())
    ids = torch.unique(all_tr[:, [0, 2]].reshape(-1))
    lrad = cfg.get("radius_lambda", 0.02) * F.mse_loss(static_radius(sd, cfg)[ids],
                                                       torch.as_tensor(radius_target)[ids].to(emb.dtype))
    return le, lr, torch.zeros(1, dtype=emb.dtype), lrad


def euclid_get_loss(sd, cfg, glist, triples):
    """RecurrentRGCN.get_loss, src/rrgcn.py:196-248 (no static graph)."""
    R = sd["emb_rel"].shape[0] // 2
    inv = triples[:, [2, 1, 0]].clone()
    inv[:, 1] += R
    all_tr = torch.cat([triples, inv])
    embs, h0 = euclid_forward(sd, cfg, glist)
    emb = F.normalize(embs[-1]) if cfg["layer_norm"] else embs[-1]
    le = F.cross_entropy(_conv_decoder(sd, "decoder_ob.", emb, h0, all_tr, None, False, hyperbolic=False),
                         all_tr[:, 2].long())
    lr = F.cross_entropy(_conv_decoder(sd, "rdecoder.", emb, h0, all_tr, None, True, hyperbolic=False),
                         all_tr[:, 1].long())
    return le, lr, torch.zeros(1, dtype=emb.dtype)
