"""Packed MFMA B-operand copies of d x d weights (regcn_pack_weight_f32).

The layer tail and timestep kernels read their weights in v_mfma_f32_16x16x4_f32
fragment order.  The packed copy is cached on the weight tensor itself and rebuilt only
when its storage, shape or version counter changes (an optimizer step, an in-place edit,
load_state_dict), so steady-state forwards launch no packing kernel.  A new packed copy is
published (_lib.publish) before it is cached: a predict on another stream may read it next.
"""
import torch

from . import _lib


def packed(w):
    """Packed copy of a (d_in, d_out) fp32 HIP weight (None -> None)."""
    if w is None:
        return None
    key = (w.data_ptr(), w._version, tuple(w.shape))
    hit = getattr(w, "_regcn_packed", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    d_in, d_out = w.shape
    wc = w.detach().contiguous()
    out = torch.empty(_lib.lib().regcn_packed_weight_floats(d_in), device=w.device, dtype=torch.float32)
    _lib.call("regcn_pack_weight_f32", _lib.fptr(wc, "weight"), d_in, d_out, _lib.fptr(out), _lib.stream())
    w._regcn_packed = (key, out)
    _lib.publish()
    return out


def packed_kp(w):
    """Packed copy of a (d_in, d_out) weight in the k-permuted fragment order of the 64-row
    tail (regcn_pack_weight_kp_f32, csrc/rowtail.hip), cached like `packed`."""
    if w is None:
        return None
    key = (w.data_ptr(), w._version, tuple(w.shape))
    hit = getattr(w, "_regcn_packed_kp", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    d_in, d_out = w.shape
    wc = w.detach().contiguous()
    out = torch.empty(_lib.lib().regcn_packed_weight_kp_floats(d_in), device=w.device, dtype=torch.float32)
    _lib.call("regcn_pack_weight_kp_f32", _lib.fptr(wc, "weight"), d_in, d_out, _lib.fptr(out), _lib.stream())
    w._regcn_packed_kp = (key, out, wc)  # keep wc alive until the packing kernel has run
    _lib.publish()
    return out


def packed_linear(w, n_gates=1):
    """Per-16-column-tile packing of an nn.Linear-layout weight ((n_gates*n_out) x n_in,
    regcn_pack_linear_f32), cached like `packed`."""
    key = (w.data_ptr(), w._version, tuple(w.shape), n_gates)
    hit = getattr(w, "_regcn_packed_lin", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    rows, n_in = w.shape
    n_out = rows // n_gates
    wc = w.detach().contiguous()
    out = torch.empty(_lib.lib().regcn_packed_linear_floats(n_gates, n_out, n_in), device=w.device,
                      dtype=torch.float32)
    _lib.call("regcn_pack_linear_f32", _lib.fptr(wc, "weight"), n_gates, n_out, n_in, _lib.fptr(out), _lib.stream())
    w._regcn_packed_lin = (key, out)
    _lib.publish()
    return out


def packed_linear_cols(w, n_gates, c0, c1):
    """`packed_linear` of the column slice w[:, c0:c1] (e.g. the emb_rel / x_mean halves of
    a GRUCell weight_ih), cached on the weight per slice."""
    key = (w.data_ptr(), w._version, tuple(w.shape), n_gates, c0, c1)
    cache = w.__dict__.setdefault("_regcn_packed_cols", {})
    hit = cache.get((n_gates, c0, c1))
    if hit is not None and hit[0] == key:
        return hit[1]
    rows = w.shape[0]
    n_out, n_in = rows // n_gates, c1 - c0
    wc = w.detach()[:, c0:c1].contiguous()
    out = torch.empty(_lib.lib().regcn_packed_linear_floats(n_gates, n_out, n_in), device=w.device,
                      dtype=torch.float32)
    _lib.call("regcn_pack_linear_f32", _lib.fptr(wc, "weight"), n_gates, n_out, n_in, _lib.fptr(out), _lib.stream())
    cache[(n_gates, c0, c1)] = (key, out, wc)  # keep wc alive until the packing kernel has run
    _lib.publish()
    return out


def packed_t(w):
    """`packed` of the transpose of an nn.Linear weight (out x in): the B operand of
    x @ W^T, cached on the weight itself."""
    key = (w.data_ptr(), w._version, tuple(w.shape))
    hit = getattr(w, "_regcn_packed_t", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    n_out, n_in = w.shape
    wt = w.detach().t().contiguous()
    out = torch.empty(_lib.lib().regcn_packed_weight_floats(n_in), device=w.device, dtype=torch.float32)
    _lib.call("regcn_pack_weight_f32", _lib.fptr(wt, "weight"), n_in, n_out, _lib.fptr(out), _lib.stream())
    w._regcn_packed_t = (key, out, wt)  # keep wt alive until the packing kernel has run
    _lib.publish()
    return out


def packed_k4(w):
    """k4 packing of an nn.Linear weight (out x in, regcn_pack_k4_f32) for the 4-row query
    kernel (csrc/queries.hip), cached on the weight like `packed`."""
    key = (w.data_ptr(), w._version, tuple(w.shape))
    hit = getattr(w, "_regcn_packed_k4", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    n_out, n_in = w.shape
    wc = w.detach().contiguous()
    out = torch.empty(_lib.lib().regcn_packed_k4_floats(n_out, n_in), device=w.device, dtype=torch.float32)
    _lib.call("regcn_pack_k4_f32", _lib.fptr(wc, "weight"), n_out, n_in, _lib.fptr(out), _lib.stream())
    w._regcn_packed_k4 = (key, out, wc)  # keep wc alive until the packing kernel has run
    _lib.publish()
    return out


def bump_versions(params):
    """Fused optimizers (torch.optim.Adam(fused=True)) update parameters in place WITHOUT
    bumping their version counters, which every cache here is keyed on: bump them after the
    step with one multi-tensor in-place x *= 1 (a bitwise identity; detach() shares the
    version counter).  Capturable inside a HIP graph, where it is harmless."""
    ts = [p.detach() for p in params if p is not None]
    if ts:
        with torch.no_grad():
            torch._foreach_mul_(ts, 1.0)


_CACHE_ATTRS = ("_regcn_packed", "_regcn_packed_lin", "_regcn_packed_t", "_regcn_packed_cols", "_regcn_packed_k4",
                "_regcn_packed_kp")


def invalidate(module):
    """Drop every parameter-derived cache of `module`: the packed weight copies above and
    the model's own caches (initial entity state, static radius, curvature).  They are
    keyed on the tensors' version counters, which writes through `.data` do not bump;
    load_state_dict and the replica broadcast call this, and so should any other code
    that edits parameters through `.data`."""
    for t in list(module.parameters()) + list(module.buffers()):
        for a in _CACHE_ATTRS:
            if hasattr(t, a):
                delattr(t, a)
    for m in module.modules():
        for a in ("_init_cache", "_r_static_cache", "_c_cache", "_gru_pre0", "_pristine_cache"):
            m.__dict__.pop(a, None)
