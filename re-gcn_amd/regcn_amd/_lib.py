"""ctypes binding to libregcn_hip.so (the C-ABI declared in include/regcn_hip.h).

The library is built in-tree by `__graft_entry__.build()` (hipcc --offload-arch=gfx950)
and loaded from this directory.  There is no fallback: if the library is missing or a
tensor is not a contiguous fp32/int32 HIP tensor, the call raises.

torch is imported before the library so that libregcn_hip.so binds to the same
libamdhip64 instance (same soname) that torch already loaded: one HIP runtime, one
set of streams.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("REGCN_HIP_LIB") or os.path.join(_HERE, "libregcn_hip.so")  # override: A/B builds
ABI_VERSION = 13

_c_int, _c_i64, _c_f, _c_vp, _c_sz = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t
P = _c_vp

# name -> argtypes (restype int32 unless listed in _RESTYPE)
_SIGS = {
    "regcn_version": [],
    "regcn_last_error_string": [],
    "regcn_set_trace": [P],
    "regcn_log0_f32": [P, _c_i64, _c_int, _c_f, P, P],
    "regcn_exp0_f32": [P, _c_i64, _c_int, _c_f, P, P],
    "regcn_project_f32": [P, _c_i64, _c_int, _c_f, P, P],
    "regcn_apply_radius_f32": [P, P, _c_i64, _c_int, _c_f, P, P],
    "regcn_radius_f32": [P, _c_i64, _c_int, P, P],
    "regcn_sumsq_f32": [P, _c_i64, _c_int, P, P],
    "regcn_mobius_add_f32": [P, P, _c_i64, _c_int, _c_f, P, P],
    "regcn_to_lorentz_f32": [P, _c_i64, _c_int, _c_f, P, P],
    "regcn_to_poincare_f32": [P, _c_i64, _c_int, _c_f, P, P],
    "regcn_prologue_f32": [P, _c_i64, _c_int, _c_f, P, P, P],
    "regcn_ln_roundtrip_f32": [P, _c_i64, _c_int, _c_f, P, P],
    "regcn_init_entities_f32": [P, P, _c_i64, _c_int, _c_f, _c_int, P, P, P, P],
    "regcn_init_entity_rows_f32": [P, P, P, P, _c_i64, _c_int, _c_f, _c_int, P, P, P, P],
    "regcn_union_aggregate_f32": [P, P, P, P, P, P, P, _c_int, P, _c_int, _c_f, _c_int, P, _c_int, P, P],
    "regcn_euclid_aggregate_f32": [P, P, P, P, P, P, _c_int, P, _c_int, _c_int, P, _c_int, P, P],
    "regcn_union_aggregate_src_runs_f32": [P, P, P, P, P, P, P, P, _c_int, P, _c_int, _c_f, _c_int, _c_int, P, _c_int,
                                           P, P],
    "regcn_segment_mean_f32": [P, P, P, P, _c_int, P, _c_int, _c_int, P, _c_int, P, P],
    "regcn_lorentz_aggregate_f32": [P, P, P, P, P, P, _c_int, P, _c_int, _c_int, _c_f, _c_int, P, _c_int, P, P],
    "regcn_packed_weight_floats": [_c_int],
    "regcn_pack_weight_f32": [P, _c_int, _c_int, P, P],
    "regcn_kreduce_workspace_floats": [_c_i64, _c_int, _c_int],
    "regcn_lorentz_centroid_f32": [P, P, _c_i64, _c_int, _c_f, _c_f, P, P, P, P, P],
    "regcn_givens_rotation_f32": [P, P, _c_i64, _c_int, P, P, P, P, P],
    "regcn_tail_f32": [P, P, P, _c_i64, P, P, P, P, _c_i64, _c_int, _c_int, _c_f, P, P, P, P, P, P, P, P],
    "regcn_kreduce_gemm_f32": [P, _c_int, P, _c_int, _c_i64, _c_int, _c_int, P, _c_i64, P, P, P],
    "regcn_layer_tail_f32": [P, P, P, P, P, P, P, P, P, P, _c_int, _c_int, _c_int, _c_int, _c_f, P, P, P, P],
    "regcn_timestep_f32": [P, P, P, P, P, P, P, _c_f, _c_f, _c_int, _c_int, _c_int, _c_int, _c_f, _c_f, P, P, P, P],
    "regcn_timestep_analysis_f32": [P, P, P, P, P, P, P, _c_f, _c_f, _c_int, _c_int, _c_int, _c_int, _c_f, _c_f, P, P,
                                    P, P, P, P],
    "regcn_hyp_score_f32": [P, P, P, P, P, P, _c_int, _c_int, _c_int, _c_f, _c_int, P, P],
    "regcn_hyp_ce_workspace_bytes": [_c_int, _c_int],
    "regcn_hyp_ce_f32": [P, P, P, P, P, P, P, _c_int, _c_int, _c_int, _c_f, _c_int, P, P, P],
    "regcn_rank_f32": [P, _c_int, _c_int, P, P, P, P, P, P],
    "regcn_rank_count_f32": [P, _c_int, _c_int, P, P, P, P, P, P],
    "regcn_hyp_rank_fused_f32": [P, P, P, P, P, P, _c_int, _c_int, _c_int, _c_f, _c_int, P, _c_int, P, _c_int, P,
                                 P],
    "regcn_pack_rows_f32": [P, P, P, ctypes.c_int64, _c_int, P, P],
    "regcn_unpack_rows_f32": [P, P, ctypes.c_int64, _c_int, P, P, P],
    "regcn_gather_rows_f32": [P, P, P, ctypes.c_int64, _c_int, P, P, P],
    "regcn_layer_f32": [P, P],
    "regcn_layer_rowtail_f32": [P, P, P],
    "regcn_layer_rowtail_part_f32": [P, P, _c_int, _c_int, _c_int, P],
    "regcn_packed_weight_kp_floats": [_c_int],
    "regcn_pack_weight_kp_f32": [P, _c_int, _c_int, P, P],
    "regcn_timestep_phase_f32": [P, _c_int, P],
    "regcn_window_plan_i32": [_c_int, P, P, _c_int, P, P, P, P, _c_int, P, P],
    "regcn_cold_chain_f32": [P, P],
    "regcn_zero_step_f32": [P, P],
    "regcn_partial_sum_f32": [P, _c_int, P, _c_int, _c_int, P, _c_int, P],
    "regcn_packed_linear_floats": [_c_int, _c_int, _c_int],
    "regcn_pack_linear_f32": [P, _c_int, _c_int, _c_int, P, P],
    "regcn_relation_gru_f32": [P, P, P, P, P, P, P, P, P, P, P, _c_int, _c_int, P, P],
    "regcn_relation_gru_pre_f32": [P, P, P, P, P, P, _c_int, _c_int, P, P],
    "regcn_relation_gru_x_f32": [P, P, P, P, P, P, P, P, _c_int, _c_int, P, P],
    "regcn_roth_query_f32": [P, P, P, _c_int, _c_int, _c_int, P, P, P, P, P, P, P, P, _c_int, _c_f, P, P],
    "regcn_roth_rel_query_f32": [P, P, _c_int, _c_int, _c_int, P, P, P, P, P, P, _c_int, _c_int, _c_f, P, P, P],
    "regcn_packed_k4_floats": [_c_int, _c_int],
    "regcn_pack_k4_f32": [P, _c_int, _c_int, P, P],
    "regcn_roth_queries_f32": [P, P],
    "regcn_hyp_score_jobs_f32": [P, _c_int, P],
    "regcn_snapshot_workspace_bytes": [_c_i64, _c_int, _c_int],
    "regcn_snapshot_capacity": [_c_int, _c_i64, _c_int, _c_int, _c_int],
    "regcn_snapshot_csr_i32": [P, P],
    "regcn_snapshot_work_i32": [P, P],
    "regcn_transpose_workspace_bytes": [_c_int, _c_int, _c_int],
    "regcn_snapshot_transpose_i32": [P, P],
    "regcn_row_type_order_workspace_bytes": [_c_int, _c_int, _c_int],
    "regcn_snapshot_row_type_order_i32": [_c_int, _c_int, _c_int, P, P, P, P, P, P, _c_sz, P],
    "regcn_row_src_order_workspace_bytes": [_c_int, _c_int],
    "regcn_item_src_order_workspace_bytes": [_c_int, _c_int],
    "regcn_snapshot_item_src_order_i32": [_c_int, _c_int, _c_int, P, P, P, P, P, P, P, _c_sz, P],
    "regcn_snapshot_row_src_order_i32": [_c_int, _c_int, P, P, P, P, _c_sz, P],
    "regcn_snapshot_item_type_order_i32": [_c_int, _c_int, _c_int, _c_int, P, P, P, P, P, P, P, _c_sz, P],
    "regcn_rowmap_bwd_f32": [_c_int, P, P, P, _c_i64, _c_int, _c_f, P, P, P],
    "regcn_union_aggregate_bwd_f32": [P, _c_f, P],
    "regcn_lorentz_sum_raw_f32": [P, P, P, P, P, P, _c_int, _c_int, _c_int, _c_f, P, P, P],
    "regcn_lorentz_aggregate_bwd_f32": [P, _c_int, _c_f, P],
    "regcn_hyp_ce_lse_f32": [P, P, P, P, P, P, _c_int, _c_int, _c_int, _c_f, _c_int, P, P, P, P],
    "regcn_hyp_ce_bwd_f32": [P, P, P, P, P, P, P, P, _c_int, _c_int, _c_int, _c_f, _c_int, P, P, P, P],
}

SCORE_DIST, SCORE_RAW_SCALE = 1, 2
_RESTYPE = {"regcn_last_error_string": ctypes.c_char_p, "regcn_hyp_ce_workspace_bytes": _c_sz,
            "regcn_snapshot_workspace_bytes": _c_sz, "regcn_kreduce_workspace_floats": _c_sz, "regcn_snapshot_capacity": _c_i64,
            "regcn_transpose_workspace_bytes": _c_sz, "regcn_row_type_order_workspace_bytes": _c_sz,
            "regcn_row_src_order_workspace_bytes": _c_sz, "regcn_item_src_order_workspace_bytes": _c_sz,
            "regcn_packed_weight_kp_floats": _c_sz,
            "regcn_packed_weight_floats": _c_sz, "regcn_packed_linear_floats": _c_sz,
            "regcn_packed_k4_floats": _c_sz}

_lib = None

AGG_UNION, AGG_EUCLID, AGG_LORENTZ, AGG_NONE = 0, 2, 3, 4


class LayerDesc(ctypes.Structure):
    """regcn_layer_desc (include/regcn_hip.h); pointer fields take dptr()/None."""
    _fields_ = [
        ("agg_mode", _c_int), ("x", P), ("radius", P), ("rel", P), ("w_rel", P), ("num_bases", _c_int),
        ("gamma", _c_f), ("rowptr", P), ("col_src", P), ("col_type", P), ("norm", P), ("budget", _c_int),
        ("tiles", P), ("n_pos_tiles", _c_int), ("item_ptr", P), ("item_src", P), ("item_tl", P), ("agg", P), ("w_n", P), ("w_loop", P), ("w_evolve", P),
        ("prev_t", P), ("w_skip", P), ("b_skip", P), ("drop_mask", P), ("rows", P), ("n_pos", _c_int),
        ("V", _c_int), ("d", _c_int), ("euclid", _c_int), ("c", _c_f), ("h_out", P), ("x_next", P),
        ("r_next", P), ("fuse_step", _c_int), ("step_x_prev", P), ("step_w_g", P), ("step_b_g", P),
        ("step_r_static", P), ("step_w_r", P), ("step_b_r", P), ("step_eps_r", _c_f), ("step_beta", _c_f),
        ("step_layer_norm", _c_int), ("step_residual", _c_int), ("step_c_radius", _c_f), ("step_h_out", P),
        ("step_x_out", P), ("step_r_out", P), ("trace", P), ("item_src_runs", _c_int),
        ("gate_w", P), ("gate_out", P), ("step_tw", P),
        ("crel_tiles", _c_int), ("crel_item_src", P), ("crel_item_tl", P), ("rel_t", P), ("n_types", _c_int),
        ("send_lo", ctypes.c_int64), ("send_n", _c_int), ("send_ptr", P), ("send_pos", P), ("send_x", P), ("send_r", P),
    ]


class PhaseDesc(ctypes.Structure):
    """regcn_phase_desc (include/regcn_hip.h)."""
    _fields_ = [
        ("agg_mode", _c_int), ("num_bases", _c_int), ("gamma", _c_f), ("c", _c_f), ("rowptr", P), ("col_src", P),
        ("col_type", P), ("norm", P), ("budget", _c_int), ("tiles", P), ("n_pos_tiles", _c_int), ("item_ptr", P),
        ("item_src", P), ("item_tl", P), ("rows", P), ("n_pos", _c_int), ("V", _c_int), ("d", _c_int), ("rel", P),
        ("w_rel", P * 2), ("agg", P * 2), ("w_n", P * 2), ("w_loop", P * 2), ("w_evolve", P * 2), ("w_skip1", P),
        ("b_skip1", P), ("x0", P), ("r0", P), ("s1", P), ("tw", P), ("x1", P), ("r1", P), ("h2", P), ("n2", P),
        ("step_w_g", P), ("step_b_g", P), ("step_r_static", P), ("step_w_r", P), ("step_b_r", P),
        ("step_eps_r", _c_f), ("step_beta", _c_f), ("step_layer_norm", _c_int), ("step_residual", _c_int),
        ("step_c_radius", _c_f), ("step_h_out", P), ("step_x_out", P), ("step_r_out", P),
        ("gru_rel_idx", P), ("gru_rel_start", P), ("gru_rel_count", P), ("gru_x_mean", P), ("gru_emb_rel", P),
        ("gru_h_prev", P), ("gru_w_ih_e", P), ("gru_w_ih_x", P), ("gru_w_hh", P), ("gru_b_ih", P), ("gru_b_hh", P),
        ("gru_R2", _c_int), ("gru_pre", P), ("gru_h_out", P), ("memo_h", P), ("memo_x", P), ("memo_r", P),
        ("n_prev", _c_int), ("prev_rows", P * 16), ("prev_rowptr", P * 16), ("prev_n_pos", _c_int * 16),
        ("skip_zero_rows", _c_int),
    ]


MAX_WINDOW = 16  # REGCN_MAX_WINDOW


class ChainDesc(ctypes.Structure):
    """regcn_chain_desc (include/regcn_hip.h)."""
    _fields_ = [
        ("rows", P), ("n_rows", P), ("T", _c_int), ("d", _c_int), ("grid_bound", _c_int), ("c", _c_f), ("x0", P),
        ("w_evolve0", P), ("w_evolve1", P), ("w_skip1", P), ("b_skip1", P), ("step_w_g", P), ("step_b_g", P),
        ("step_r_static", P), ("step_w_r", P), ("step_b_r", P), ("step_eps_r", _c_f), ("step_beta", _c_f),
        ("step_layer_norm", _c_int), ("step_residual", _c_int), ("step_c_radius", _c_f),
        ("h_out", P * MAX_WINDOW), ("x_out", P * MAX_WINDOW), ("r_out", P * MAX_WINDOW),
    ]


# regcn_snapshot_desc (include/regcn_hip.h): stats slots and capacity ids
SNAP = dict(MAX_DEG=0, N_POS=1, INVALID=2, N_PAIRS=3, REL_MAX=4, N_HEAVY=5, N_TILES=6, N_ITEMS=7, WALK_TILES=8,
            A_STAR=9, CHUNKS=10, HEAVY_CHUNKS=13, REL_CHUNKS=16, NSTATS=20)
CAP = dict(TILES=0, ITEMS=1, CHUNKS=2, FIXUPS=3, HEAVY_CHUNKS=4, HEAVY_FIXUPS=5, REL_CHUNKS=6, REL_FIXUPS=7,
           REL_IDX=8)


class RothQueriesDesc(ctypes.Structure):
    """regcn_roth_queries_desc (include/regcn_hip.h)."""
    _fields_ = [("ent", P), ("rel", P), ("trip", P), ("n_test", _c_int), ("B", _c_int), ("num_rels", _c_int),
                ("d", _c_int), ("c", _c_f), ("w1", P), ("b1", P), ("w2", P), ("b2", P), ("w_rot", P), ("b_rot", P),
                ("w_trans", P), ("b_trans", P), ("q_ent", P), ("rw1", P), ("rb1", P), ("rw2", P), ("rb2", P),
                ("global_rot", P), ("q_rel", P), ("n_cand", _c_int), ("cand", P), ("all_triples", P)]


class ScoreJob(ctypes.Structure):
    """regcn_score_job (include/regcn_hip.h)."""
    _fields_ = [("q", P), ("cand", P), ("bias", P), ("scale", P), ("margin", P), ("B", _c_int), ("N", _c_int),
                ("d", _c_int), ("c", _c_f), ("flags", _c_int), ("out", P)]


class SnapshotDesc(ctypes.Structure):
    _fields_ = [
        ("triples", P), ("T", _c_i64), ("V", _c_int), ("R", _c_int), ("budget", _c_int), ("pack_items", _c_int),
        ("chunk_edges", _c_int), ("workspace", P), ("ws_bytes", _c_sz), ("stats", P),
        ("in_deg", P), ("rowptr", P), ("col_src", P), ("col_type", P), ("norm", P), ("edge_type", P),
        ("edge_norm", P), ("rel_ent_count", P), ("rel_idx", P), ("rel_start", P), ("rel_count", P),
        ("rows", P), ("tiles", P), ("item_ptr", P), ("item_src", P), ("item_tl", P), ("chunks", P), ("fixups", P),
        ("heavy_chunks", P), ("heavy_fixups", P), ("rel_chunks", P), ("rel_fixups", P),
    ]


class TransposeDesc(ctypes.Structure):
    _fields_ = [("V", _c_int), ("E", _c_int), ("R2", _c_int), ("rowptr", P), ("col_src", P), ("col_type", P),
                ("workspace", P), ("ws_bytes", _c_sz), ("csr_dst", P), ("sptr", P), ("sp", P), ("tptr", P), ("tp", P)]


class EdgeBwdDesc(ctypes.Structure):
    _fields_ = [("V", _c_int), ("E", _c_int), ("R2", _c_int), ("d", _c_int), ("x", P), ("radius", P), ("rel", P),
                ("W", P), ("norm", P), ("rowptr", P), ("col_src", P), ("col_type", P), ("csr_dst", P), ("sptr", P),
                ("sp", P), ("tptr", P), ("tp", P), ("G", P), ("G0", P), ("dx", P), ("drel", P), ("dradius", P),
                ("dW", P), ("edge_scratch", P)]


def call_desc(name, desc):
    check(getattr(lib(), name)(ctypes.byref(desc), stream()), name)


class HipLibraryError(RuntimeError):
    pass


def lib():
    """Load (once) and return the ctypes handle; raise if the HIP library is unavailable."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HipLibraryError(
                "libregcn_hip.so not found at %s; build it with `python -c \"import __graft_entry__ as g; "
                "g.build()\"`" % LIB_PATH)
        h = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, _c_int)
        v = h.regcn_version()
        if v != ABI_VERSION:
            raise HipLibraryError("libregcn_hip.so ABI %d != expected %d" % (v, ABI_VERSION))
        _lib = h
    return _lib


def exported_symbols():
    return list(_SIGS)


# measurement (bench.py): when a list, every library call appends (name, HIP event recorded
# on the current stream right after the call's launches); consecutive events bracket the
# device time of each call on an in-order stream
EVENT_TRACE = None


def trace_mark(name):
    """Record a named HIP event on the current stream into EVENT_TRACE (if tracing)."""
    if EVENT_TRACE is not None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        EVENT_TRACE.append((name, ev))


def check(rc, name):
    if rc != 0:
        msg = lib().regcn_last_error_string().decode(errors="replace")
        raise RuntimeError("%s failed (rc=%d): %s" % (name, rc, msg))
    if EVENT_TRACE is not None:
        trace_mark(name)


def call(name, *args):
    check(getattr(lib(), name)(*args), name)


def call_layer(desc):
    check(lib().regcn_layer_f32(ctypes.byref(desc), stream()),
          "regcn_layer_f32(step)" if desc.fuse_step else "regcn_layer_f32")


def publish():
    """Make device data just written on the current stream safe to read from any stream.
    Lazily built caches (packed weights, a snapshot's edge orders, parameter-only states) are
    read by whichever stream asks next -- another lane's predict may run on another stream --
    so the builder waits for its kernels once.  Inside a HIP-graph capture the graph keeps its
    own order and nothing is done."""
    if not torch.cuda.is_current_stream_capturing():
        torch.cuda.current_stream().synchronize()


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def addr(t, dtype=torch.float32, what="tensor"):
    """Device address (int) of a contiguous HIP tensor (None -> None)."""
    if t is None:
        return None
    if not isinstance(t, torch.Tensor):
        raise TypeError("%s must be a torch.Tensor" % what)
    if not t.is_cuda:
        raise ValueError("%s must live on a HIP device (got %s); the HIP path has no CPU fallback" % (what, t.device))
    if t.dtype != dtype:
        raise TypeError("%s must be %s (got %s)" % (what, dtype, t.dtype))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % what)
    return t.data_ptr()


def dptr(t, dtype=torch.float32, what="tensor"):
    """Device pointer of a contiguous HIP tensor (None -> NULL)."""
    a = addr(t, dtype, what)
    return None if a is None else ctypes.c_void_p(a)


def fptr(t, what="tensor"):
    return dptr(t, torch.float32, what)


def iptr(t, what="index tensor"):
    return dptr(t, torch.int32, what)
