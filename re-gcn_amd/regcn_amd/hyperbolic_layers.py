"""Hyperbolic message-passing layers on HIP (mirror of hyperbolic_src/hyperbolic_layers.py).

Constructor arguments, parameter names/shapes (hence state_dict keys) and forward
signatures follow the reference; forward runs three gfx950 kernels per layer:
  1. row prologue x = log0(h), r = |h| (skipped when the producer already emitted them);
  2. CSR gather + segment reduce (csrc/aggregate.hip);
  3. MFMA layer tail: neighbour/self-loop/skip GEMMs + clamp/rrelu/dropout/exp0 and the
     next layer's prologue, fused (csrc/rowgemm.hip).
With autograd on (training) the model runs training.py instead, the differentiable
composition of the same layers; FHNN/HGAT encoders are outside this build's scope.
"""
import ctypes
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .parallel import ShardedGraph
from .tangent import attach, tangent_of
from .weights import packed, packed_kp
from .graph import hub_block_work

EPS = 1e-6
TRACE = None  # int64 HIP tensor (>= 8 x workgroups) to record k_layer phase timestamps (profiling)
# Snapshots with at least this many rows run a layer as the agg gather + the 64-row MFMA tail
# (regcn_layer_rowtail_f32, csrc/rowtail.hip) instead of the fused 16-row kernel; 0 disables.
ROWTAIL_MIN_ROWS = int(os.environ.get("REGCN_ROWTAIL_MIN_ROWS", "65536"))
# ... and a view (a rank's rows of a partitioned snapshot) of at least this many rows
ROWTAIL_MIN_VIEW_ROWS = int(os.environ.get("REGCN_ROWTAIL_MIN_VIEW_ROWS", "1024"))
# ... in this many row chunks: the gather of chunk i + 1 runs on a side stream beside the tail of
# chunk i (the L2-bound gather beside the MFMA-bound tail); 1 = one stream, no pipelining
ROWTAIL_CHUNKS = int(os.environ.get("REGCN_ROWTAIL_CHUNKS", "1"))
# Inline tiles with at least this many items take their relation half as one MFMA product per
# tile (regcn_layer_desc.crel_tiles, csrc/rowtail.hip k_gather_crel); 0 disables.  Config-5 sweep
# (profiles/r5_crel_sweep.log, gather call ms): off 1.623, 512 1.657, 1024 1.596, 2048 1.580, 4096 1.667
CREL_MIN_ITEMS = int(os.environ.get("REGCN_CREL_MIN_ITEMS", "2048"))
# ... when at least this many tiles qualify: a crel workgroup is one tile's long chain, so a launch
# of fewer big tiles than the chip's crel slots (3 per CU) lasts one chain while most CUs idle --
# a rank's view of an owner-partitioned config-5 snapshot has ~220 (profiles/r5_owner_sim_kernels_*)
# (8-rank simulation: predicted 8.19 -> 8.13 ms with 768, profiles/r5_crel_min_tiles_sim.txt)
CREL_MIN_TILES = int(os.environ.get("REGCN_CREL_MIN_TILES", "768"))
# A rank's pipeline-chunk tails (owner partition) on this many streams (1: one after another)
CHUNK_TAIL_STREAMS = int(os.environ.get("REGCN_CHUNK_TAIL_STREAMS", "2"))
# a fused-step cell's inner layer on the 64-row tail skips its Poincare rows h (the next layer
# reads x = log0 h and |h| only): 800 MB less written per timestep at config 5
INNER_SKIP_H = os.environ.get("REGCN_INNER_SKIP_H", "1") != "0"


def _rowtail_chunks(g, k):
    """[(tile0, tile1, row0, row1)]: k chunks of the rows list, cut at tile starts (each chunk's
    gather covers exactly the in-edge rows its tail needs), the rows without in-edges in the
    last; cached on the graph (one host copy of the tile starts)."""
    hit = g.__dict__.get("_rt_chunks")
    if hit is not None and hit[0] == k:
        return hit[1]
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        return None  # no host copy inside a capture: this launch runs unchunked
    wk = g.work()
    n_t, n_rows = int(g.n_pos_tiles), int(wk["rows"].shape[0])
    starts = wk["tiles"][:n_t, 0].cpu().tolist() if n_t else []
    k = max(1, min(k, n_t)) if n_t else 1
    tb = [round(i * n_t / k) for i in range(k + 1)]
    rb = [starts[t] if t < n_t else n_rows for t in tb]
    rb[0], rb[-1] = 0, n_rows
    out = [(tb[i], tb[i + 1], rb[i], rb[i + 1]) for i in range(k)]
    g.__dict__["_rt_chunks"] = (k, out)
    return out


_RT_STREAMS = {}


def _rowtail_stream(dev):
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    st = _RT_STREAMS.get(key)
    if st is None:
        st = _RT_STREAMS[key] = torch.cuda.Stream(dev)
    return st


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


def _heavy_aggregate(mode, g, x, r, rel, w_rel, nb, gamma, c):
    """Pre-aggregate the rows over the fused kernel's edge budget (chunked kernels);
    returns the V x d buffer holding them, or None when the snapshot has none."""
    if not g.n_heavy:
        return None
    wk = g.work()
    V, d = x.shape
    agg = torch.empty_like(x)
    hc, hf = wk["heavy_chunks"], wk["heavy_fixups"]
    stride = d + 4
    part = torch.empty(max(g.heavy_slots, 1), stride, device=x.device, dtype=torch.float32)
    f, i = _lib.fptr, _lib.iptr
    halo = getattr(g, "hub_cols", None)  # a rank's HaloView: remote sources read from its halo rows
    if mode == _lib.AGG_LORENTZ:  # hub rows: edges in type order, same-type runs reuse rel/W from L1
        cs, ct = g.row_type_cols()
        if halo is not None:
            cs, ct, _, hc = halo(cs, ct, None, hc)
        _lib.call("regcn_lorentz_aggregate_f32", f(x), f(rel), f(w_rel), i(cs), i(ct), i(hc),
                  hc.shape[0], i(hf), hf.shape[0], nb, float(c), d, f(part), stride, f(agg), _lib.stream())
    else:  # union / Euclid: relation half over type runs, source half over source runs
        cs, ct = g.row_type_cols()
        ss = g.row_src_cols()
        euclid = mode != _lib.AGG_UNION
        # the source-block lists of the plain view (positions; blocks by the original ids)
        hb = hub_block_work(getattr(g, "hub_owner", g)) if hasattr(g, "row_src_cols") else None
        if hb is not None:  # large snapshot: spans cut at source blocks, XCD-dealt (graph.py)
            hc, hf, n_slots = hb
            part = torch.empty(n_slots, stride, device=x.device, dtype=torch.float32)
        if halo is not None:
            cs, ct, ss, hc = halo(cs, ct, ss, hc)
        _lib.call("regcn_union_aggregate_src_runs_f32", f(x), None if euclid else f(r), f(rel), i(cs), i(ct), i(ss),
                  f(wk["norm"]), i(hc), hc.shape[0], i(hf), hf.shape[0], float(gamma), int(euclid), d, f(part), stride,
                  f(agg), _lib.stream())
    return agg


class StepSpec:
    """Timestep operands fused behind the last layer (regcn_layer_desc step_* fields).
    w_g_param: the time-gate weight itself (the 64-row tail packs it its own way); tw: the
    gate pre-activation rows clamp(x_prev) @ W_g when the cell's first layer computed them
    (the 64-row tail, `gate=` of run_layer), else None."""

    def __init__(self, x_prev, w_g, b_g, r_static, w_r, b_r, eps_r, beta, layer_norm, residual, c_radius,
                 w_g_param=None):
        self.x_prev, self.w_g, self.b_g, self.r_static = x_prev, w_g, b_g, r_static
        self.w_r, self.b_r, self.eps_r, self.beta = w_r, b_r, eps_r, beta
        self.layer_norm, self.residual, self.c_radius = layer_norm, residual, c_radius
        self.w_g_param, self.tw = w_g_param, None
        self.need_h = True  # False: the timestep's Poincare rows h are not written (x, |h| are)
        # False: x = log0 h and |h| are not written (predict's last timestep, whose consumers read
        # h only); the 64-row tail honours it and the returned h carries no tangent cache
        self.need_xr = True


def _use_rowtail(V, n_rows, d, prev_t, drop_mask, pos_only):
    """The 64-row tail serves large snapshots' layers (V rows; a rank's view of one runs its
    own n_rows) without a skip gate or dropout mask."""
    return (ROWTAIL_MIN_ROWS > 0 and V >= ROWTAIL_MIN_ROWS and n_rows >= ROWTAIL_MIN_VIEW_ROWS and prev_t is None
            and drop_mask is None and not pos_only and d % 4 == 0 and d <= 256)


def run_layer(mode, g, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t, w_skip, b_skip, drop_mask, c,
              euclid=False, step=None, agg=None, out=None, pos_only=False, gate=None, need_h=True):
    """One fused layer launch (regcn_layer_f32): inline gather + GEMMs + epilogue, or with
    `step` the timestep too.  Returns (h, x_next, r_next) of the layer (or of the step).
    `g` may be a rank's view of a snapshot (parallel.py): the launch covers its rows only,
    writing them into full-size outputs (`out`, optional preallocated (h, x, r)).
    agg (with mode AGG_NONE): the finished aggregation of every in-degree > 0 row.
    pos_only: the launch covers the rows with in-edges only (rows[:n_pos]).
    Large snapshots run regcn_layer_rowtail_f32 instead (the agg gather, then the 64-row MFMA
    tail); `gate` (a StepSpec, the cell's first layer): that path also writes the timestep's
    gate pre-activation rows into gate.tw for the step layer."""
    if isinstance(g, ShardedGraph):  # multi-GPU partition of the snapshot (parallel.py)
        if agg is not None or out is not None or pos_only:
            raise ValueError("agg/out are managed by the sharded layer")
        return g.run_layer(mode, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, prev_t, w_skip, b_skip,
                           drop_mask, c, euclid=euclid, step=step, gate=gate)
    wk = g.work()
    V, d = x.shape
    n_rows = int(wk["rows"].shape[0])
    a = _lib.addr
    rowtail = _use_rowtail(V, n_rows, d, prev_t, drop_mask, pos_only) and (agg is None or mode == _lib.AGG_NONE)
    if agg is None:
        agg = _heavy_aggregate(mode, g, x, r, rel, w_rel, nb, gamma, c)
    elif mode != _lib.AGG_NONE:
        raise ValueError("a precomputed aggregation needs mode AGG_NONE")
    if g.n_pos == 0:  # an edgeless snapshot: nothing to gather, every row takes the evolve loop
        mode = _lib.AGG_NONE
    if rowtail:
        return _run_rowtail(mode, g, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, c, euclid, step, agg, out,
                            gate, n_rows, need_h=need_h)
    if out is None:
        h = torch.empty_like(x)
        xn = torch.empty_like(x)
        rn = torch.empty(V, device=x.device, dtype=torch.float32)
    else:
        h, xn, rn = out
    pk = [packed(w) for w in (w_n, w_loop, w_evolve, w_skip)]
    desc = _lib.LayerDesc()
    desc.agg_mode = mode
    desc.x = a(x, what="x")
    desc.radius = a(r, what="radius")
    desc.rel = a(rel, what="rel_emb")
    desc.w_rel = a(w_rel, what="weight")
    desc.num_bases = int(nb)
    desc.gamma = float(gamma)
    desc.rowptr = a(wk["rowptr"], torch.int32)
    desc.col_src = a(wk["col_src"], torch.int32)
    desc.col_type = a(wk["col_type"], torch.int32)
    desc.norm = a(wk["norm"])
    desc.budget = g.budget
    desc.tiles = a(wk["tiles"], torch.int32)
    desc.n_pos_tiles = g.n_pos_tiles
    desc.item_ptr = a(wk["item_ptr"], torch.int32)
    items = (wk["item_src"], wk["item_tl"])
    if mode in (_lib.AGG_UNION, _lib.AGG_EUCLID) and getattr(g, "use_item_src_runs", None) and g.use_item_src_runs():
        items = g.item_src_cols()  # a row's duplicate sources gathered once (regcn_layer_desc.item_src_runs)
        desc.item_src_runs = 1
    desc.item_src = a(items[0], torch.int32) if items[0].numel() else None
    desc.item_tl = a(items[1], torch.int32) if items[1].numel() else None
    desc.agg = a(agg)
    desc.w_n, desc.w_loop, desc.w_evolve, desc.w_skip = (a(w) for w in pk)
    desc.prev_t = a(prev_t, what="prev_h")
    desc.b_skip = a(b_skip)
    desc.drop_mask = a(drop_mask)
    desc.rows = a(wk["rows"], torch.int32)
    desc.n_pos, desc.V, desc.d, desc.euclid = g.n_pos, g.n_pos if pos_only else n_rows, d, int(bool(euclid))
    desc.c = float(c)
    if step is None:
        desc.h_out, desc.x_next, desc.r_next = a(h), a(xn), a(rn)
    else:
        desc.fuse_step = 1
        desc.step_x_prev = a(step.x_prev, what="x_prev")
        desc.step_w_g, desc.step_b_g = a(step.w_g), a(step.b_g)
        desc.step_r_static, desc.step_w_r, desc.step_b_r = a(step.r_static), a(step.w_r), a(step.b_r)
        desc.step_eps_r, desc.step_beta = float(step.eps_r), float(step.beta)
        desc.step_layer_norm, desc.step_residual = int(bool(step.layer_norm)), int(bool(step.residual))
        desc.step_c_radius = float(step.c_radius)
        desc.step_h_out, desc.step_x_out, desc.step_r_out = a(h), a(xn), a(rn)
    if TRACE is not None:  # profiling hook: per-workgroup phase timestamps
        desc.trace = a(TRACE, torch.int64)
    _lib.call_layer(desc)
    return h, xn, rn


def run_layer_chunked(mode, g, tail_views, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, c, euclid, step, out,
                      gate, after, send=None):
    """The large-snapshot layer over a rank's rows in pipeline chunks (parallel.ShardedGraph,
    owner partition): the hub pass and the gather run once over `g` (all of the rank's rows),
    then each tail view's 64-row tail, `after(j)` following chunk j's tail (its rows' x and |h|
    are final: the caller all-gathers them while the next chunk's tail runs).  send(j): None or
    the send block chunk j's tail writes as well (parallel.ExchangePlan.send_block)."""
    agg = _heavy_aggregate(mode, g, x, r, rel, w_rel, nb, gamma, c)
    if g.n_pos == 0:
        mode = _lib.AGG_NONE
    return _run_rowtail(mode, g, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, c, euclid, step, agg, out, gate,
                        int(g.work()["rows"].shape[0]), tail_views=tail_views, after=after, send=send)


def _run_rowtail(mode, g, x, r, rel, w_rel, nb, gamma, w_n, w_loop, w_evolve, c, euclid, step, agg, out, gate,
                 n_rows, tail_views=None, after=None, send=None, need_h=True):
    """regcn_layer_rowtail_f32: the inline in-edge rows gathered into `agg` (which holds the hub
    rows already), then the 64-row tail over all rows (csrc/rowtail.hip).  need_h=False (a
    cell's inner layer, whose consumer reads x_next and r_next only): h is not written."""
    wk = g.work()
    V, d = x.shape
    a = _lib.addr
    if out is None:
        h = torch.empty_like(x)
        xn = torch.empty_like(x)
        rn = torch.empty(V, device=x.device, dtype=torch.float32)
    else:
        h, xn, rn = out
    if agg is None and g.n_pos:
        agg = torch.empty_like(x)
    desc = _lib.LayerDesc()
    desc.agg_mode = mode
    desc.x = a(x, what="x")
    desc.radius = a(r, what="radius")
    desc.rel = a(rel, what="rel_emb")
    desc.w_rel = a(w_rel, what="weight")
    desc.num_bases = int(nb)
    desc.gamma = float(gamma)
    desc.rowptr = a(wk["rowptr"], torch.int32)
    desc.col_src = a(wk["col_src"], torch.int32)
    desc.col_type = a(wk["col_type"], torch.int32)
    desc.norm = a(wk["norm"])
    desc.budget = g.budget
    desc.tiles = a(wk["tiles"], torch.int32)
    desc.n_pos_tiles = g.n_pos_tiles
    desc.item_ptr = a(wk["item_ptr"], torch.int32)
    items = (wk["item_src"], wk["item_tl"])
    if mode in (_lib.AGG_UNION, _lib.AGG_EUCLID) and getattr(g, "use_item_src_runs", None) and g.use_item_src_runs():
        items = g.item_src_cols()
        desc.item_src_runs = 1
    desc.item_src = a(items[0], torch.int32) if items[0].numel() else None
    desc.item_tl = a(items[1], torch.int32) if items[1].numel() else None
    desc.w_n, desc.w_loop, desc.w_evolve = (a(packed_kp(w)) for w in (w_n, w_loop, w_evolve))
    desc.rows = a(wk["rows"], torch.int32)
    desc.n_pos, desc.V, desc.d, desc.euclid = g.n_pos, n_rows, d, int(bool(euclid))
    desc.c = float(c)
    keep = []
    cr = _crel(g, mode, rel) if g.n_pos else None
    if cr is not None:  # the big tiles' relation half as one product per tile
        desc.crel_tiles, desc.n_types = cr[0], rel.shape[0]
        desc.crel_item_src, desc.crel_item_tl = a(cr[1][0], torch.int32), a(cr[1][1], torch.int32)
        desc.rel_t = a(cr[2])
        keep.append(cr[2])
    if step is None:
        desc.h_out, desc.x_next, desc.r_next = a(h) if (need_h or not INNER_SKIP_H) else None, a(xn), a(rn)
        if gate is not None and gate.w_g_param is not None:
            if gate.tw is None:
                gate.tw = torch.empty_like(x)
            desc.gate_w, desc.gate_out = a(packed_kp(gate.w_g_param)), a(gate.tw)
    else:
        desc.fuse_step = 1
        desc.step_x_prev = a(step.x_prev, what="x_prev")
        wg = packed_kp(step.w_g_param) if step.w_g_param is not None else None
        if wg is None:
            raise ValueError("the 64-row tail needs StepSpec.w_g_param")
        desc.step_w_g, desc.step_b_g = a(wg), a(step.b_g)
        desc.step_r_static, desc.step_w_r, desc.step_b_r = a(step.r_static), a(step.w_r), a(step.b_r)
        desc.step_eps_r, desc.step_beta = float(step.eps_r), float(step.beta)
        desc.step_layer_norm, desc.step_residual = int(bool(step.layer_norm)), int(bool(step.residual))
        desc.step_c_radius = float(step.c_radius)
        skip = not step.need_h and INNER_SKIP_H
        desc.step_h_out, desc.step_x_out, desc.step_r_out = None if skip else a(h), a(xn), a(rn)
        if not step.need_xr and not skip and send is None:
            desc.step_x_out = desc.step_r_out = None
            xn = rn = None
        if step.tw is not None:
            desc.step_tw = a(step.tw)
            keep.append(step.tw)
    name = "regcn_layer_rowtail_f32(step)" if step is not None else "regcn_layer_rowtail_f32"
    if tail_views is not None:  # gather over g, then one tail per view (run_layer_chunked)
        part = _lib.lib().regcn_layer_rowtail_part_f32
        if mode != _lib.AGG_NONE and g.n_pos_tiles:
            _lib.check(part(ctypes.byref(desc), _lib.fptr(agg), 1, 0, int(g.n_pos_tiles), _lib.stream()),
                       "regcn_layer_rowtail_f32(gather)")
        # chunk tails alternate between the calling stream and a side stream, so chunk j + 1's
        # tail fills the CUs chunk j's drains from (a chunk is ~500 workgroups) while each
        # chunk's completion still orders its exchange (after(j) runs on the chunk's stream)
        cur = torch.cuda.current_stream(x.device)
        lanes = [cur]
        if CHUNK_TAIL_STREAMS > 1 and len(tail_views) > 1:
            side = _rowtail_stream(x.device)
            side.wait_stream(cur)
            lanes.append(side)
        for j, tv in enumerate(tail_views):
            with torch.cuda.stream(lanes[j % len(lanes)]):
                tw = tv.work()
                nr = int(tw["rows"].shape[0])
                sb = send(j) if (send is not None and nr) else None
                if sb is not None:  # the tail also fills chunk j's send block of the halo exchange
                    lo, n, ptr, pos, xs, r1 = sb
                    desc.send_lo, desc.send_n = int(lo), int(n)
                    desc.send_ptr, desc.send_pos = a(ptr, torch.int32), a(pos, torch.int32)
                    desc.send_x, desc.send_r = a(xs), a(r1)
                else:
                    desc.send_lo, desc.send_n, desc.send_ptr, desc.send_pos, desc.send_x, desc.send_r = 0, 0, None, None, None, None
                if nr:
                    keep.append(tw["rows"])
                    desc.rows, desc.n_pos, desc.V = a(tw["rows"], torch.int32), tv.n_pos, nr
                    _lib.check(part(ctypes.byref(desc), _lib.fptr(agg), 2, 0, nr, _lib.stream()), name)
                after(j)
        for ln in lanes[1:]:  # every side-stream read and write joined back (frees on `cur` are safe)
            cur.wait_stream(ln)
        return h, xn, rn
    chunks = _rowtail_chunks(g, ROWTAIL_CHUNKS) if (ROWTAIL_CHUNKS > 1 and g.n_pos_tiles > 1
                                                     and mode != _lib.AGG_NONE) else None
    if chunks is None or len(chunks) < 2:
        # the gather and the tail as two calls (the same two launches regcn_layer_rowtail_f32
        # makes), so a trace times each kernel on its own
        part = _lib.lib().regcn_layer_rowtail_part_f32
        if mode != _lib.AGG_NONE and g.n_pos_tiles:
            _lib.check(part(ctypes.byref(desc), _lib.fptr(agg), 1, 0, int(g.n_pos_tiles), _lib.stream()),
                       "regcn_layer_rowtail_f32(gather)")
        _lib.check(part(ctypes.byref(desc), _lib.fptr(agg), 2, 0, int(n_rows), _lib.stream()), name)
        return h, xn, rn
    # gathers on the side stream, chunk by chunk; each tail chunk waits for its gather only
    part = _lib.lib().regcn_layer_rowtail_part_f32
    cur = torch.cuda.current_stream(x.device)
    side = _rowtail_stream(x.device)
    side.wait_stream(cur)
    events = []
    with torch.cuda.stream(side):
        for t0, t1, _, _ in chunks:
            _lib.check(part(ctypes.byref(desc), _lib.fptr(agg), 1, t0, t1, _lib.stream()), name + "[gather]")
            ev = torch.cuda.Event()
            ev.record(side)
            events.append(ev)
    for (_, _, r0, r1), ev in zip(chunks, events):
        cur.wait_event(ev)
        _lib.check(part(ctypes.byref(desc), _lib.fptr(agg), 2, r0, r1, _lib.stream()), name)
    # the last tail waited for the last gather event, so every side-stream read is joined into
    # `cur` here: x, r, rel and agg may be freed on `cur` afterwards (and, under capture, the
    # fork joins back into the captured stream)
    return h, xn, rn


def _rel_t(rel):
    """rel (R2 x d) transposed into the crel gather's B operand: 16 ceil(d / 16) rows of kpad =
    R2 rounded up to 16 floats, zero padded; cached on the tensor per version (both layers of a
    timestep read the same relation rows)."""
    hit = getattr(rel, "_regcn_relt", None)
    if hit is not None and hit[0] == rel._version:
        return hit[1]
    R2, d = rel.shape
    t = torch.zeros(-(-d // 16) * 16, -(-R2 // 16) * 16, device=rel.device, dtype=torch.float32)
    t[:d, :R2] = rel.t()
    rel._regcn_relt = (rel._version, t)
    return t


def _crel(g, mode, rel):
    """(tiles, (item_src, item_tl) in (row, type) order, rel_t) of the rowtail gather's leading
    tiles up to the last of the first run of tiles with >= CREL_MIN_ITEMS items (tiles come in
    descending row-degree order: the hub rows' item-less tiles, then the big ones), or None:
    union / euclid, R2 <= 512 (a snapshot, or a rank's view of one: parallel.OwnerView /
    HaloView build their own type-ordered items)."""
    if CREL_MIN_ITEMS <= 0 or mode not in (_lib.AGG_UNION, _lib.AGG_EUCLID) or not hasattr(g, "item_type_cols"):
        return None
    if rel.shape[0] > 512 or not g.n_pos_tiles:
        return None
    hit = g.__dict__.get("_crel_tiles")
    if hit is None or hit[0] != CREL_MIN_ITEMS:
        if torch.cuda.is_current_stream_capturing():
            return None  # no host copy inside a capture: this launch gathers per item
        big = np.diff(g.work()["item_ptr"][:g.n_pos_tiles + 1].cpu().numpy()) >= CREL_MIN_ITEMS
        k, first = 0, 0
        if big.any():  # the big tiles follow the hub rows' tiles (no inline items: skipped in-kernel)
            first = int(np.argmax(big))
            rest = np.nonzero(~big[first:])[0]
            k = first + (int(rest[0]) if len(rest) else len(big) - first)
        hit = g.__dict__["_crel_tiles"] = (CREL_MIN_ITEMS, k, first)
    if hit[1] == 0 or hit[1] - hit[2] < CREL_MIN_TILES:
        return None
    return hit[1], g.item_type_cols(), _rel_t(rel)


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

    def forward(self, g, h_hyper, rel_emb, prev_h=None, step=None, pos_only=False, out=None, gate=None,
                need_h=True):
        """hyperbolic_layers.py:242-323 (one fused launch; `step` fuses the timestep;
        pos_only/out/gate/need_h: see run_layer)."""
        if self.activation is None:
            raise NotImplementedError("the fused tail applies rrelu; activation=None is not supported")
        self.rel_emb = rel_emb
        c = float(self.c)
        x, r = tangent_of(h_hyper, c)
        prev_t = None
        if self.skip_connect and prev_h is not None:
            prev_t = tangent_of(prev_h, c)[0]
        wl = self.loop_weight if self.self_loop else None
        we = self.evolve_loop_weight if self.self_loop else None
        h, xn, rn = run_layer(_lib.AGG_UNION, g, x, r, rel_emb.contiguous(), None, 0, self.radius_msg_gamma,
                              self.weight_neighbor, wl, we, prev_t,
                              self.skip_weight if prev_t is not None else None,
                              self.skip_bias.detach() if prev_t is not None else None,
                              _drop_mask(self, x), c, step=step, out=out, pos_only=pos_only, gate=gate,
                              need_h=need_h)
        return attach(h, xn, rn, c) if xn is not None else h  # xn None: StepSpec.need_xr


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

    def forward(self, g, h_hyper, rel_emb=None, prev_h=None, step=None, pos_only=False, out=None, gate=None,
                need_h=True):
        """hyperbolic_layers.py:627-694 (one fused launch; `step` fuses the timestep;
        pos_only/out/gate/need_h: see run_layer)."""
        if self.activation is None:
            raise NotImplementedError("the fused tail applies rrelu; activation=None is not supported")
        if self.submat_in * self.num_bases != self.in_feat:
            # the reference's view(-1, 1, submat_in) fails on this shape too
            raise RuntimeError("in_feat=%d is not divisible by num_bases=%d" % (self.in_feat, self.num_bases))
        self.rel_emb = rel_emb
        c = float(self.c)
        x, r = tangent_of(h_hyper, c)
        V, d = x.shape
        if rel_emb is None:
            rel = torch.zeros(self.num_rels, d, device=x.device, dtype=torch.float32)
        else:
            rel = rel_emb if rel_emb.shape[1] == d else rel_emb[:, :d]
            rel = rel.contiguous()
        prev_t = None
        if self.skip_connect and prev_h is not None:
            prev_t = tangent_of(prev_h, c)[0]
        wl = self.loop_weight if self.self_loop else None
        we = self.evolve_loop_weight if self.self_loop else None
        h, xn, rn = run_layer(_lib.AGG_LORENTZ, g, x, r, rel, self.weight.detach().contiguous(), self.num_bases, 0.0,
                              None, wl, we, prev_t,
                              self.skip_weight if prev_t is not None else None,
                              self.skip_bias.detach() if prev_t is not None else None,
                              _drop_mask(self, x), c, step=step, out=out, pos_only=pos_only, gate=gate,
                              need_h=need_h)
        return attach(h, xn, rn, c) if xn is not None else h  # xn None: StepSpec.need_xr


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

    def forward(self, g, init_ent_emb, init_rel_emb, step=None, pos_only=False, out=None):
        """`step` (StepSpec): run the timestep fused into the last layer's launch and
        return its output instead of the cell output.  pos_only/out (with step): the
        launches cover the rows with in-edges only, the last one writing into `out`."""
        h = init_ent_emb  # node ids are arange(V) (rgcn/utils.py:122): the gather is the identity
        rel_embs = init_rel_emb if isinstance(init_rel_emb, list) else [init_rel_emb] * len(self.layers)
        prev_h = None
        n = len(self.layers)
        for i, layer in enumerate(self.layers):
            last = i == n - 1
            h_new = layer(g, h, rel_embs[i], prev_h=prev_h, step=step if last else None, pos_only=pos_only,
                          out=out if last else None, gate=step if (i == 0 and not last) else None,
                          need_h=last or step is None)
            prev_h = h
            h = h_new
        return h
