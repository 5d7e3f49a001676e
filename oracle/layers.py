"""Message-passing layers restated (oracle; test infrastructure only).

Mirrors the reference op sequence: per-edge messages are materialised (E x d),
the Union layer runs the per-edge GEMM, and messages are segment-summed into
their destination with zero fill for nodes without in-edges (DGL
update_all + fn.sum semantics).

`g` is a dict as produced by oracle.graph.build_sub_graph (src/dst/type in
the reference's edge order, in_deg, norm).
"""
import torch

from . import ops


def _t(a, dtype=None):
    t = torch.as_tensor(a)
    return t.to(dtype) if dtype is not None else t


def _self_loop(x, g, w_loop, w_evolve):
    """hyperbolic_layers.py:273-280 / rgcn/layers.py:226-233: W_loop for nodes
    with in-degree > 0, W_evolve otherwise."""
    loop = torch.mm(x, w_evolve)
    mask = _t(g["in_deg"]) > 0
    loop[mask] = torch.mm(x, w_loop)[mask]
    return loop


def _segment_sum(msg, dst, n):
    out = torch.zeros((n,) + tuple(msg.shape[1:]), dtype=msg.dtype)
    out.index_add_(0, dst, msg)
    return out


def _chunks(n, chunk):
    chunk = chunk or max(n, 1)
    return [slice(i, min(i + chunk, n)) for i in range(0, n, chunk)]


def union_layer(g, h, rel, w_n, w_loop, w_evolve, c, gamma, skip=None, self_loop=True, edge_chunk=None):
    """HyperbolicUnionRGCNLayer.forward, hyperbolic_layers.py:242-323 (eval mode).

    msg_e = ((x_src + rel[type]) @ W_n) * exp(-gamma |r_src - r_dst|)   (:222-236)
    agg   = norm * sum_e msg_e                                         (:238-240, :290)
    out   = exp0(leaky(clamp(clamp(agg) + loop)))                      (:296-321)
    skip  = (w_skip, b_skip, prev_h): gate = sigmoid(log0(prev) @ w_skip + b) (:283-303)
    edge_chunk: the per-edge messages materialised this many edges at a time (the same
    per-edge arithmetic, summed chunk by chunk; for hub rows of millions of edges).
    """
    src, dst, et = _t(g["src"]).long(), _t(g["dst"]).long(), _t(g["type"]).long()
    n = h.shape[0]
    x = ops.log0(h, c)
    rad = ops.get_radius(h).unsqueeze(-1)
    if self_loop:
        loop = _self_loop(x, g, w_loop, w_evolve)
    if skip is not None:
        w_skip, b_skip, prev_h = skip
        prev_t = ops.log0(prev_h, c)
        sg = torch.sigmoid(torch.mm(prev_t, w_skip) + b_skip)
    agg = torch.zeros(n, x.shape[1], dtype=x.dtype)
    for sl in _chunks(src.numel(), edge_chunk):
        s_, d_ = src[sl], dst[sl]
        msg = torch.nn.functional.linear(x[s_] + rel[et[sl]], w_n.t())
        wgt = torch.exp(-gamma * torch.abs(rad[s_] - rad[d_])).squeeze(-1)
        agg.index_add_(0, d_, msg * wgt.unsqueeze(-1))
    agg = agg * _t(g["norm"]).float().view(-1, 1)
    hn = torch.clamp(agg, -10.0, 10.0)
    if self_loop:
        hn = hn + loop
    if skip is not None:
        hn = sg * hn + (1 - sg) * prev_t
    hn = torch.clamp(hn, -10.0, 10.0)
    return ops.exp0(ops.leaky(hn), c)


def euclid_union_layer(g, h, rel, w_n, w_loop, w_evolve, self_loop=True):
    """UnionRGCNLayer.forward, rgcn/layers.py:222-279 (eval mode, no skip):
    node = norm * sum_e (h_src + rel[type]) @ W_n + loop, then rrelu."""
    src, dst, et = _t(g["src"]).long(), _t(g["dst"]).long(), _t(g["type"]).long()
    n = h.shape[0]
    if self_loop:
        loop = _self_loop(h, g, w_loop, w_evolve)
    msg = torch.mm(h[src] + rel[et], w_n)
    node = _segment_sum(msg, dst, n) * _t(g["norm"]).float().view(-1, 1)
    if self_loop:
        node = node + loop
    return ops.leaky(node)


def lorentz_layer(g, h, rel, weight, w_loop, w_evolve, c, num_bases, skip=None, self_loop=True, edge_chunk=None):
    """LorentzRGCNLayer.forward, hyperbolic_layers.py:627-694 (eval mode).

    msg: m = blockdiag_k(W[type]_k (s x s)) . x_src + rel[type]; p = exp0(m);
         L = to_lorentz(p)                                       (:589-611)
    reduce: per destination the weighted Lorentz centroid with mailbox
         weights norm_dst / (sum + 1e-6), renormalised inside the centroid
         (:613-625, hyperbolic_ops.py:562-581); zero in-degree -> 0.
    then to_poincare -> log0 -> clamp -> +loop [skip blend] -> clamp -> leaky -> exp0.
    edge_chunk: as union_layer.
    """
    src, dst, et = _t(g["src"]).long(), _t(g["dst"]).long(), _t(g["type"]).long()
    n, d = h.shape
    s = d // num_bases
    x = ops.log0(h, c)
    if self_loop:
        loop = _self_loop(x, g, w_loop, w_evolve)
    if skip is not None:
        w_skip, b_skip, prev_h = skip
        prev_t = ops.log0(prev_h, c)
        sg = torch.sigmoid(torch.mm(prev_t, w_skip) + b_skip)
    # mailbox weights (:620): all messages of one destination carry norm_dst
    nd = _t(g["norm"]).float()[dst]
    w1 = nd / (_segment_sum(nd, dst, n)[dst] + 1e-6)
    w2 = w1 / (_segment_sum(w1, dst, n)[dst] + 1e-6)            # hyperbolic_ops.py:576
    cen = torch.zeros(n, d + 1, dtype=x.dtype)
    for sl in _chunks(src.numel(), edge_chunk):
        e_ = et[sl]
        wt = weight.index_select(0, e_).view(-1, s, s)
        node = x[src[sl]].view(-1, 1, s)
        m = torch.bmm(node, wt).view(-1, d)
        if rel is not None:
            m = m + rel.index_select(0, e_)[:, :d]
        L = ops.to_lorentz(ops.exp0(m, c), c)
        cen.index_add_(0, dst[sl], w2[sl].unsqueeze(-1).to(L.dtype) * L)   # :577
    ip = ops.lorentz_inner(cen, cen, keepdim=True)                 # :579
    cen = cen / torch.sqrt(torch.clamp(-ip * c, min=1e-6))         # :580-581
    cen[_t(g["in_deg"]) == 0] = 0.0                                # DGL zero fill
    hn = ops.log0(ops.to_poincare(cen, c), c)
    hn = torch.clamp(hn, -10.0, 10.0)
    if self_loop:
        hn = hn + loop
    if skip is not None:
        hn = sg * hn + (1 - sg) * prev_t
    hn = torch.clamp(hn, -10.0, 10.0)
    return ops.exp0(ops.leaky(hn), c)
