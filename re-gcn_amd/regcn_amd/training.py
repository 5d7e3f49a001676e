"""Differentiable forward of the recurrent encoder (training path).

The inference forward fuses a whole layer (gather + GEMMs + epilogue [+ timestep]) into one
launch and keeps no intermediates.  Training needs them, so this path composes the
autograd functions of autograd.py -- HIP kernels forward and backward for the row maps,
the union / Lorentz message aggregation and (in the decoders) the all-entity cross
entropy -- with the split-K products (autograd.mm_weight / linear), the fused layer tail
(autograd.tail: clamp, self loop, skip / time gates, rrelu) and the remaining glue (dropout,
normalize, GRUCell) as device torch ops.  The op sequence is the reference's:

  HyperbolicUnionRGCNLayer.forward   hyperbolic_layers.py:242-323
  LorentzRGCNLayer.forward           hyperbolic_layers.py:627-694
  HyperbolicRecurrentRGCN.forward    hyperbolic_model.py:722-890
"""
import torch
import torch.nn.functional as F

from . import _lib
from . import analysis
from . import autograd as A

RRELU_SLOPE = (1.0 / 8 + 1.0 / 3) / 2  # F.rrelu(x) with training=False (hyperbolic_model.py:120)


def _pos_rows(g, device):
    """uint8 per row: 1 where the row has in-edges (hyperbolic_layers.py:273-280), cached."""
    pos = g.__dict__.get("_pos_u8")
    if pos is None or pos.device != device:
        pos = (g.in_degrees() > 0).to(device=device, dtype=torch.uint8).contiguous()
        _lib.publish()
        g.__dict__["_pos_u8"] = pos
    return pos


def _loop_product(x, layer):
    """x [W_loop | W_evolve] (V x 2d): one GEMM forward, one for dx, one split-K for dW."""
    return A.mm_weight(x, torch.cat([layer.loop_weight, layer.evolve_loop_weight], dim=1))


def _layer_tail(layer, g, h_new, x, prev_h, c):
    """clamp -> + loop [-> skip blend] -> clamp -> rrelu -> dropout -> exp0
    (hyperbolic_layers.py:296-321, :672-694); everything up to rrelu is one fused launch
    (A.tail), fed by ONE product x [W_loop | W_evolve] (rows with / without in-edges pick a
    half) instead of two."""
    loop = pos = z = bias = prev_t = None
    if layer.self_loop:
        loop = _loop_product(x, layer)
        pos = _pos_rows(g, x.device)
    if layer.skip_connect and prev_h is not None:
        prev_t = A.log0(prev_h, c)
        z, bias = A.mm_weight(prev_t, layer.skip_weight), layer.skip_bias
    h_new = A.tail(h_new, loop, pos, z, bias, prev_t,
                   A.TAIL_CLAMP_IN | A.TAIL_CLAMP_OUT | A.TAIL_LEAKY, RRELU_SLOPE)
    if layer.dropout is not None:
        h_new = layer.dropout(h_new)
    return A.exp0(h_new, c)


def union_layer(layer, g, h, rel, prev_h=None):
    """msg = ((x_src + rel) W_n) w_e summed and normalised == (norm sum_e w_e (x_src + rel)) W_n."""
    c = float(layer.c)
    x = A.log0(h, c)
    r = A.get_radius(h)
    agg = A.mm_weight(A.union_aggregate(x, r, rel.contiguous(), g, layer.radius_msg_gamma), layer.weight_neighbor)
    return _layer_tail(layer, g, agg, x, prev_h, c)


def lorentz_layer(layer, g, h, rel, prev_h=None):
    c = float(layer.c)
    x = A.log0(h, c)
    d = x.shape[1]
    rel_d = torch.zeros(layer.num_rels, d, device=x.device) if rel is None else rel[:, :d].contiguous()
    agg = A.lorentz_aggregate(x, rel_d, layer.weight, g, layer.num_bases, c)
    return _layer_tail(layer, g, agg, x, prev_h, c)


def cell_forward(cell, g, h, rel_embs, lorentz):
    """HyperbolicRGCNCell (no prev_h, hyperbolic_model.py:142-154) / LorentzRGCNCell
    (prev_h = the layer input, hyperbolic_layers.py:719-743)."""
    prev = None
    for i, layer in enumerate(cell.layers):
        if lorentz:
            new = lorentz_layer(layer, g, h, rel_embs[i], prev_h=prev)
        else:
            new = union_layer(layer, g, h, rel_embs[i])
        prev, h = h, new
    return h


class _RelationContext(torch.autograd.Function):
    """x_input[r] = mean of x over r's r_to_e span, 0 for absent relations
    (hyperbolic_model.py:802-812), forward and backward on the segment-mean kernel
    (regcn_segment_mean_f32): deterministic (fixed summation orders, no atomics).

    forward: the forward relations' spans (hyperbolic_model.relation_context; an inverse
    relation's span repeats its forward relation's entities, so its mean is a copy).
    backward: dx[e] = sum over the forward relations r whose span holds e of
    (dy[r] + dy[r + R]) / count[r] -- a gather-sum over each entity's relation list (the
    entity-sorted transpose of the spans, built once per snapshot and cached)."""

    @staticmethod
    def forward(ctx, x, g, R2):
        from .hyperbolic_model import relation_context as rc_fwd
        ctx.g, ctx.R2, ctx.V = g, R2, x.shape[0]
        return rc_fwd(x.detach().contiguous(), g, R2)

    @staticmethod
    def backward(ctx, dy):
        from . import _lib
        g, R2, V = ctx.g, ctx.R2, ctx.V
        R = R2 // 2
        wk = g.work()
        d = dy.shape[1]
        tr = _entity_relation_lists(g, V, R)
        gr = (dy[:R] + dy[R:]) / torch.clamp(wk["rel_count"][:R], min=1.0).unsqueeze(-1)
        dx = torch.zeros(V, d, device=dy.device, dtype=torch.float32)
        ch = tr["chunks"]
        if ch.shape[0]:
            _lib.call("regcn_segment_mean_f32", _lib.fptr(gr.contiguous(), "grad"), _lib.iptr(tr["rel"]),
                      _lib.fptr(tr["ones"]), _lib.iptr(ch), ch.shape[0], None, 0, d, None, d, _lib.fptr(dx),
                      _lib.stream())
        return dx, None, None


def _entity_relation_lists(g, V, R):
    """Per entity, the forward relations whose r_to_e span holds it (entity-sorted, stable),
    as chunk records {entity, begin, end, -1} over that list (one chunk per entity: an entity
    touches at most R relations); cached on the graph."""
    tr = g.__dict__.get("_ent_rel")
    if tr is not None:
        return tr
    wk = g.work()
    dev = wk["rel_idx"].device
    cnt = wk["rel_count"][:R].long()
    n_fwd = int(wk["rel_idx"].numel()) // 2
    ent = wk["rel_idx"][:n_fwd].long()
    rel = torch.repeat_interleave(torch.arange(R, device=dev), cnt)
    order = torch.sort(ent, stable=True).indices
    ent_s, rel_s = ent[order], rel[order].to(torch.int32)
    per = torch.bincount(ent_s, minlength=V)
    ptr = torch.zeros(V + 1, device=dev, dtype=torch.long)
    ptr[1:] = torch.cumsum(per, 0)
    rows = torch.nonzero(per > 0).flatten()
    chunks = torch.stack([rows, ptr[rows], ptr[rows + 1], torch.full_like(rows, -1)], 1).to(torch.int32).contiguous()
    tr = {"rel": rel_s.contiguous() if rel_s.numel() else torch.zeros(1, device=dev, dtype=torch.int32),
          "chunks": chunks, "ones": torch.ones(V, device=dev, dtype=torch.float32)}
    _lib.publish()
    g.__dict__["_ent_rel"] = tr
    return tr


def relation_context(x, g, R2):
    """x_input[r] = mean of the rows of r's r_to_e span, 0 for absent relations
    (hyperbolic_model.py:802-812), HIP forward and backward (_RelationContext)."""
    if g.work()["rel_idx"].numel() == 0:
        return torch.zeros(R2, x.shape[1], device=x.device, dtype=x.dtype) + 0.0 * x.sum()
    return _RelationContext.apply(x, g, R2)


def model_forward(model, g_list):
    """HyperbolicRecurrentRGCN.forward with autograd (hyperbolic_model.py:722-890)."""
    c = model._c_float()
    # a learned curvature enters the model-level maps as the clamped exp(log_c) tensor, so its
    # gradient flows (hyperbolic_model.py:753-756); the layers and the radius evolution keep
    # their constructor-time float (hyperbolic_layers.py:195, hyperbolic_ops.py:385)
    ct = model.get_curvature() if model.learn_curvature else c
    dev = model.dynamic_emb.device
    R2 = model.num_rels * 2
    r_static = model._static_radius(c)
    dyn = model.dynamic_emb
    h = A.exp0(F.normalize(dyn) if model.layer_norm else dyn, ct)                      # :775-780
    h = A.apply_radius(h, r_static, c)                                                 # :782
    trev = model.temporal_radius_evolution
    lorentz = model.encoder_name == "lgcn"
    ana = model.run_analysis
    if ana and model.training:                                                         # :791-792
        analysis.log_embedding(model, h, "init_embeddings", c)
    history, h0, gate_list, gate_means = [], None, [], []
    for i, g in enumerate(g_list):
        g = g.to(dev)
        x_prev = A.log0(h, ct)                                                         # :802
        x_in = torch.cat([model.emb_rel, relation_context(x_prev, g, R2)], dim=1)
        h0 = model.relation_gru(x_in, model.emb_rel if i == 0 else h0)                 # :815-823
        if model.layer_norm:
            h0 = F.normalize(h0)
        cur = cell_forward(model.rgcn, g, h, [h0] * len(model.rgcn.layers), lorentz)   # :828
        cur = A.project(cur, c)                                                        # :829
        if model.layer_norm:
            cur = A.exp0(F.normalize(A.log0(cur, ct)), ct)                            # :832-835
        pt = torch.clamp(x_prev, -10.0, 10.0)                                          # :841-846
        z = A.mm_weight(pt, model.time_gate_weight)                                    # tw = sigmoid(z + b)
        if ana:                                                                        # :852-856
            with torch.no_grad():
                gate_list.append(torch.sigmoid(z.detach() + model.time_gate_bias.detach()))
                gate_means.append(gate_list[-1].mean())
        mix = A.tail(A.log0(cur, ct), z=z, bias=model.time_gate_bias, p=pt, flags=A.TAIL_CLAMP_IN)
        h = A.project(A.exp0(mix, ct), c)                                              # :859-860
        if model.use_residual_evolution:
            t = A.log0(h, trev.c)                                                      # hyperbolic_ops.py:395-435
            delta = torch.clamp(A.linear(trev.radius_mlp, t).squeeze(-1), -trev.epsilon, trev.epsilon)
            dyn = A.get_radius(h)
            base = trev.anchor_beta * r_static + (1.0 - trev.anchor_beta) * dyn
            h = A.apply_radius(h, base + delta, trev.c)
            if ana:  # TemporalRadiusEvolution's stats of this evolution (hyperbolic_ops.py:426-434)
                with torch.no_grad():
                    trev.last_evolution_stats = analysis.evolution_terms(
                        delta.detach(), dyn.detach(), base.detach(), r_static.detach(), trev.anchor_beta, trev.epsilon)
        else:
            h = A.apply_radius(h, r_static, c)                                         # :869
        if ana:
            analysis.log_timestep(i, gate_means[-1], trev.__dict__.get("_ev"))
        history.append(h)
    if ana:                                                                            # :887-888
        dict.__setitem__(model.training_stats, "time_gate_values", torch.stack(gate_means) if gate_means else [])
    return history, None, h0, gate_list, []


def euclid_layer(layer, g, h, rel):
    """UnionRGCNLayer.forward, rgcn/layers.py:222-279 (the cell passes prev_h = [], so no skip):
    norm sum_e (h_src + rel) W_n + loop, rrelu, dropout."""
    zero_r = torch.zeros(h.shape[0], device=h.device)
    node = A.mm_weight(A.union_aggregate(h, zero_r, rel.contiguous(), g, 0.0), layer.weight_neighbor)
    loop = pos = None
    if layer.self_loop:
        loop, pos = _loop_product(h, layer), _pos_rows(g, h.device)
    node = A.tail(node, loop, pos, flags=A.TAIL_LEAKY, slope=RRELU_SLOPE)
    if layer.dropout is not None:
        node = layer.dropout(node)
    return node


def euclid_model_forward(model, g_list):
    """RecurrentRGCN.forward with autograd (src/rrgcn.py:142-180)."""
    dev = model.dynamic_emb.device
    R2 = model.num_rels * 2
    h = F.normalize(model.dynamic_emb) if model.layer_norm else model.dynamic_emb
    history, h0 = [], None
    for i, g in enumerate(g_list):
        g = g.to(dev)
        x_in = torch.cat([model.emb_rel, relation_context(h, g, R2)], dim=1)
        h0 = model.relation_cell_1(x_in, model.emb_rel if i == 0 else h0)
        if model.layer_norm:
            h0 = F.normalize(h0)
        cur = h
        for layer in model.rgcn.layers:
            cur = euclid_layer(layer, g, cur, h0)
        if model.layer_norm:
            cur = F.normalize(cur)
        h = A.tail(cur, z=A.mm_weight(h, model.time_gate_weight), bias=model.time_gate_bias, p=h)  # tw cur + (1 - tw) h
        history.append(h)
    return history, None, h0, [], []


class GraphedSteps:
    """Whole training steps replayed from HIP graphs: one graph per key
    (a training sample: its snapshot shapes fix every launch), captured right after the
    key's first step, which runs eagerly.  The step is launch-bound at ICEWS size (~1,000
    launches of 2-30 us), so a replay removes the host's launch cost; it needs a step free of
    host synchronisation (the radius loss's distinct-entity mask, curvature floats cached per
    version) and an optimizer whose step counter lives on the device (Adam capturable=True).

    All graphs share one memory pool: each is self-contained (it reads the parameters, the
    sample's snapshot graphs and triples, which the caller keeps alive for the key, and
    writes parameters, optimizer state and its returned tensor), so replays may come in any
    order; the returned tensor is valid until the next `run`.  Dropout draws from the
    graph-safe generator (a different mask per replay, as in eager steps)."""

    def __init__(self, device):
        self.device = device
        self.stream = torch.cuda.Stream(device)
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs = {}

    def run(self, key, step):
        """`step()` -> device tensor: one full step (zero_grad, forward, backward, clip,
        optimizer step).  Runs it eagerly the first time `key` is seen and captures it for the
        later calls, which replay.  Ordered after the calling stream's prior work."""
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            g = self.graphs.get(key)
            if g is not None:
                g[0].replay()
                out = g[1]
            else:
                out = step()  # eager: lazily built caches (transposed edge lists, ...) exist after it
                gph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gph, pool=self.pool, stream=self.stream):
                    static = step()
                self.graphs[key] = (gph, static)
        cur.wait_stream(self.stream)
        return out
