// extern "C" entry points of libregcn_hip.so (declared in include/regcn_hip.h).
#include <stdarg.h>
#include <stdio.h>

#include "regcn_internal.h"

namespace regcn {

static thread_local char g_err[512] = "";
int64_t* g_trace = nullptr;

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error((int)e, "%s: %s", what, hipGetErrorString(e));
  return 0;
}

}  // namespace regcn

using namespace regcn;

#define ST(s) ((hipStream_t)(s))

extern "C" {

int regcn_version(void) { return REGCN_ABI_VERSION; }
int regcn_set_trace(int64_t* buf) {
  g_trace = buf;
  return 0;
}
const char* regcn_last_error_string(void) { return g_err; }

int regcn_log0_f32(const float* x, int64_t rows, int32_t d, float c, float* out, void* s) {
  return rowmap(0, x, nullptr, nullptr, rows, d, c, out, nullptr, nullptr, ST(s));
}
int regcn_exp0_f32(const float* v, int64_t rows, int32_t d, float c, float* out, void* s) {
  return rowmap(1, v, nullptr, nullptr, rows, d, c, out, nullptr, nullptr, ST(s));
}
int regcn_project_f32(const float* x, int64_t rows, int32_t d, float c, float* out, void* s) {
  return rowmap(2, x, nullptr, nullptr, rows, d, c, out, nullptr, nullptr, ST(s));
}
int regcn_apply_radius_f32(const float* x, const float* radius, int64_t rows, int32_t d, float c, float* out,
                           void* s) {
  return rowmap(3, x, nullptr, radius, rows, d, c, out, nullptr, nullptr, ST(s));
}
int regcn_radius_f32(const float* x, int64_t rows, int32_t d, float* out, void* s) {
  return rowmap(4, x, nullptr, nullptr, rows, d, 0.01f, out, nullptr, nullptr, ST(s));
}
int regcn_sumsq_f32(const float* x, int64_t rows, int32_t d, float* out, void* s) {
  return rowmap(9, x, nullptr, nullptr, rows, d, 0.01f, out, nullptr, nullptr, ST(s));
}
int regcn_mobius_add_f32(const float* x, const float* y, int64_t rows, int32_t d, float c, float* out, void* s) {
  return rowmap(5, x, y, nullptr, rows, d, c, out, nullptr, nullptr, ST(s));
}
int regcn_to_lorentz_f32(const float* x, int64_t rows, int32_t d, float c, float* out, void* s) {
  return rowmap(6, x, nullptr, nullptr, rows, d, c, out, nullptr, nullptr, ST(s));
}
int regcn_to_poincare_f32(const float* y, int64_t rows, int32_t d, float c, float* out, void* s) {
  return rowmap(7, y, nullptr, nullptr, rows, d, c, out, nullptr, nullptr, ST(s));
}
int regcn_prologue_f32(const float* h, int64_t rows, int32_t d, float c, float* x_out, float* r_out, void* s) {
  return rowmap(8, h, nullptr, nullptr, rows, d, c, x_out, r_out, nullptr, ST(s));
}
int regcn_ln_roundtrip_f32(const float* x, int64_t rows, int32_t d, float c, float* out, void* s) {
  return rowmap(10, x, nullptr, nullptr, rows, d, c, out, nullptr, nullptr, ST(s));
}
int regcn_init_entities_f32(const float* dyn, const float* r_static, int64_t rows, int32_t d, float c,
                            int32_t layer_norm, float* h_out, float* x_out, float* r_out, void* s) {
  return rowmap(layer_norm ? 12 : 11, dyn, nullptr, r_static, rows, d, c, h_out, x_out, r_out, ST(s));
}
int regcn_init_entity_rows_f32(const float* dyn, const float* r_static, const int32_t* src, const int32_t* dst,
                               int64_t n, int32_t d, float c, int32_t layer_norm, float* h_out, float* x_out,
                               float* r_out, void* s) {
  return init_rows(dyn, r_static, src, dst, n, d, c, layer_norm, h_out, x_out, r_out, ST(s));
}

int regcn_union_aggregate_f32(const float* x, const float* radius, const float* rel, const int32_t* col_src,
                              const int32_t* col_type, const float* norm, const int32_t* chunks, int32_t n_chunks,
                              const int32_t* fixups, int32_t n_fix, float gamma, int32_t d, float* partial,
                              int32_t partial_stride, float* out, void* s) {
  return gather_sum(0, x, radius, rel, col_src, col_type, norm, chunks, n_chunks, fixups, n_fix, gamma, d, partial,
                    partial_stride, out, ST(s));
}
int regcn_union_aggregate_src_runs_f32(const float* x, const float* radius, const float* rel, const int32_t* col_src,
                                       const int32_t* col_type, const int32_t* col_src_by_src, const float* norm,
                                       const int32_t* chunks, int32_t n_chunks, const int32_t* fixups, int32_t n_fix,
                                       float gamma, int32_t euclid, int32_t d, float* partial, int32_t partial_stride,
                                       float* out, void* s) {
  if (!col_src_by_src && n_chunks > 0) return set_error(REGCN_EINVAL, "null source-order column");
  return gather_sum(euclid ? 2 : 0, x, radius, rel, col_src, col_type, norm, chunks, n_chunks, fixups, n_fix, gamma, d,
                    partial, partial_stride, out, ST(s), col_src_by_src);
}
int regcn_euclid_aggregate_f32(const float* h, const float* rel, const int32_t* col_src, const int32_t* col_type,
                               const float* norm, const int32_t* chunks, int32_t n_chunks, const int32_t* fixups,
                               int32_t n_fix, int32_t d, float* partial, int32_t partial_stride, float* out,
                               void* s) {
  return gather_sum(2, h, nullptr, rel, col_src, col_type, norm, chunks, n_chunks, fixups, n_fix, 0.f, d, partial,
                    partial_stride, out, ST(s));
}
int regcn_segment_mean_f32(const float* x, const int32_t* idx, const float* count, const int32_t* chunks,
                           int32_t n_chunks, const int32_t* fixups, int32_t n_fix, int32_t d, float* partial,
                           int32_t partial_stride, float* out, void* s) {
  return gather_sum(1, x, nullptr, nullptr, idx, nullptr, count, chunks, n_chunks, fixups, n_fix, 0.f, d, partial,
                    partial_stride, out, ST(s));
}
int regcn_lorentz_aggregate_f32(const float* x, const float* rel, const float* weight, const int32_t* col_src,
                                const int32_t* col_type, const int32_t* chunks, int32_t n_chunks,
                                const int32_t* fixups, int32_t n_fix, int32_t num_bases, float c, int32_t d,
                                float* partial, int32_t partial_stride, float* out, void* s) {
  return lorentz_sum(x, rel, weight, col_src, col_type, chunks, n_chunks, fixups, n_fix, num_bases, c, d, partial,
                     partial_stride, out, ST(s));
}

int regcn_partial_sum_f32(float* partial, int32_t partial_stride, const int32_t* fixups, int32_t n_fix,
                          int32_t width, float* out, int32_t out_stride, void* s) {
  return partial_sum(partial, partial_stride, fixups, n_fix, width, out, out_stride, ST(s));
}

size_t regcn_packed_weight_floats(int32_t d_in) { return packed_weight_floats(d_in); }

int regcn_pack_weight_f32(const float* w, int32_t d_in, int32_t d_out, float* packed, void* s) {
  return pack_weight(w, d_in, d_out, packed, ST(s));
}

size_t regcn_kreduce_workspace_floats(int64_t K, int32_t M, int32_t N) { return kreduce_workspace_floats(K, M, N); }

int regcn_kreduce_gemm_f32(const float* a, int32_t a_kmajor, const float* b, int32_t b_kmajor, int64_t K, int32_t M,
                           int32_t N, const float* c0, int64_t c0_ld, float* out, float* workspace, void* s) {
  return kreduce_gemm(a, a_kmajor, b, b_kmajor, K, M, N, c0, c0_ld, out, workspace, ST(s));
}

int regcn_tail_f32(const float* agg, const float* lx, const float* ex, int64_t loop_ld, const uint8_t* pos,
                   const float* z, const float* bias, const float* p, int64_t V, int32_t d, int32_t flags, float slope,
                   const float* grad_out, float* out, float* d_agg, float* d_lx, float* d_ex, float* d_z, float* d_p,
                   void* s) {
  TailArgs t{agg, lx, ex, z, bias, p, grad_out, pos, out, d_agg, d_lx, d_ex, d_z, d_p, V, loop_ld, d, flags, slope};
  return tail(t, grad_out != nullptr, ST(s));
}

int regcn_lorentz_centroid_f32(const float* S0, const float* Sv, int64_t V, int32_t d, float c, float sqrt_c,
                               const float* grad_y, float* y, float* d_S0, float* d_Sv, void* s) {
  return centroid(S0, Sv, V, d, c, sqrt_c, grad_y, y, d_S0, d_Sv, ST(s));
}

int regcn_givens_rotation_f32(const float* x, const float* angles, int64_t n_pairs, int32_t reflect,
                              const float* grad_out, float* out, float* d_x, float* d_angles, void* s) {
  return givens(x, angles, n_pairs, reflect, grad_out, out, d_x, d_angles, ST(s));
}

int regcn_layer_tail_f32(const float* agg, const float* w_n, const float* x, const float* w_loop,
                         const float* w_evolve, const float* prev_t, const float* w_skip, const float* b_skip,
                         const float* drop_mask, const int32_t* rows, int32_t n_pos, int32_t V, int32_t d,
                         int32_t euclid, float c, float* h_out, float* x_next, float* r_next, void* s) {
  LayerArgs a{};
  a.agg_mode = 4;  // AGG_NONE
  a.agg = agg;
  a.w_n = w_n;
  a.x = x;
  a.w_loop = w_loop;
  a.w_evolve = w_evolve;
  a.prev_t = prev_t;
  a.w_skip = w_skip;
  a.b_skip = b_skip;
  a.drop_mask = drop_mask;
  a.rows = rows;
  a.n_pos = agg ? n_pos : 0;  // no neighbour term: every row takes the pos/zero weight split below
  a.V = V;
  a.d = d;
  a.euclid = euclid;
  a.k = make_curv(c);
  a.h_out = h_out;
  a.x_next = x_next;
  a.r_next = r_next;
  if (!agg && n_pos > 0) {
    // no neighbour term, but rows still choose W_loop (in-degree > 0) or W_evolve: two
    // launches over the two row ranges, each as "zero in-degree" tiles
    LayerArgs z = a;
    z.n_pos = 0;
    z.rows = rows;
    z.V = n_pos;
    z.w_evolve = w_loop;
    int rc = layer(z, ST(s));
    if (rc) return rc;
    z.rows = rows + n_pos;
    z.V = V - n_pos;
    z.w_evolve = w_evolve;
    return layer(z, ST(s));
  }
  return layer(a, ST(s));
}

int regcn_window_plan_i32(int32_t T, const int32_t* const* pos_rows, const int32_t* n_pos, int32_t V, int32_t* flags,
                          int32_t* c_rows, int32_t* u_rows, int32_t* z_rows, int32_t z_stride, int32_t* counts,
                          void* s) {
  if (T < 1 || T > REGCN_MAX_WINDOW || !pos_rows || !n_pos) return set_error(REGCN_EINVAL, "bad window");
  PlanArgs a{};
  a.T = T;
  a.V = V;
  for (int t = 0; t < T; ++t) {
    a.pos_rows[t] = pos_rows[t];
    a.n_pos[t] = n_pos[t];
  }
  a.flags = flags;
  a.c_rows = c_rows;
  a.u_rows = u_rows;
  a.z_rows = z_rows;
  a.z_stride = z_stride;
  a.counts = counts;
  return window_plan(a, ST(s));
}

// regcn_cold_chain_f32 / regcn_zero_step_f32 share the descriptor
static int chain_args(const regcn_chain_desc* g, ChainArgs& a) {
  if (!g) return set_error(REGCN_EINVAL, "null descriptor");
  a.rows = g->rows;
  a.n_rows = g->n_rows;
  a.T = g->T;
  a.d = g->d;
  a.x0 = g->x0;
  a.w_evolve0 = g->w_evolve0;
  a.w_evolve1 = g->w_evolve1;
  a.w_skip1 = g->w_skip1;
  a.b_skip1 = g->b_skip1;
  a.k = make_curv(g->c);
  StepArgs& t = a.step;
  t.x_prev = g->x0;
  t.w_g = g->step_w_g;
  t.b_g = g->step_b_g;
  t.r_static = g->step_r_static;
  t.w_r = g->step_w_r;
  t.b_r = g->step_b_r;
  t.eps_r = g->step_eps_r;
  t.beta = g->step_beta;
  t.layer_norm = g->step_layer_norm;
  t.residual = g->step_residual;
  t.d = g->d;
  t.k = a.k;
  t.k_rad = make_curv(g->step_c_radius);
  for (int i = 0; i < REGCN_MAX_WINDOW; ++i) {
    a.h_out[i] = g->h_out[i];
    a.x_out[i] = g->x_out[i];
    a.r_out[i] = g->r_out[i];
  }
  return 0;
}

int regcn_cold_chain_f32(const regcn_chain_desc* g, void* s) {
  ChainArgs a{};
  if (int rc = chain_args(g, a)) return rc;
  return cold_chain(a, g->grid_bound, ST(s));
}

int regcn_zero_step_f32(const regcn_chain_desc* g, void* s) {
  ChainArgs a{};
  if (int rc = chain_args(g, a)) return rc;
  return zero_step(a, g->grid_bound, ST(s));
}

int regcn_timestep_phase_f32(const regcn_phase_desc* g, int32_t phase, void* s) {
  if (!g) return set_error(REGCN_EINVAL, "null descriptor");
  PhaseArgs a{};
  const Curv k = make_curv(g->c);
  for (int i = 0; i < 2; ++i) {
    LayerArgs& l = a.L[i];
    l.agg_mode = g->agg_mode;
    l.nb = g->num_bases;
    l.gamma = g->gamma;
    l.rowptr = g->rowptr;
    l.col_src = g->col_src;
    l.col_type = g->col_type;
    l.norm = g->norm;
    l.budget = g->budget;
    l.tiles = g->tiles;
    l.n_pos_tiles = g->n_pos_tiles;
    l.item_ptr = g->item_ptr;
    l.item_src = g->item_src;
    l.item_tl = g->item_tl;
    l.rows = g->rows;
    l.n_pos = g->n_pos;
    l.V = g->V;
    l.d = g->d;
    l.k = k;
    l.rel = g->rel;
    l.w_rel = g->w_rel[i];
    l.agg = g->agg[i];
    l.w_n = g->w_n[i];
    l.w_loop = g->w_loop[i];
    l.w_evolve = g->w_evolve[i];
  }
  a.L[0].x = g->x0;
  a.L[0].radius = g->r0;
  a.L[1].x = g->x1;
  a.L[1].radius = g->r1;
  if (g->w_skip1) {
    a.L[1].prev_t = g->x0;
    a.L[1].w_skip = g->w_skip1;
    a.L[1].b_skip = g->b_skip1;
  }
  StepArgs& t = a.step;
  t.x_prev = g->x0;
  t.w_g = g->step_w_g;
  t.b_g = g->step_b_g;
  t.r_static = g->step_r_static;
  t.w_r = g->step_w_r;
  t.b_r = g->step_b_r;
  t.eps_r = g->step_eps_r;
  t.beta = g->step_beta;
  t.layer_norm = g->step_layer_norm;
  t.residual = g->step_residual;
  t.V = g->V;
  t.d = g->d;
  t.k = k;
  t.k_rad = make_curv(g->step_c_radius);
  t.h_out = g->step_h_out;
  t.x_out = g->step_x_out;
  t.r_out = g->step_r_out;
  if (t.residual && (!t.w_r || !t.b_r)) return set_error(REGCN_EINVAL, "residual radius needs w_r and b_r");
  if (!t.r_static || !t.b_g) return set_error(REGCN_EINVAL, "null timestep pointer");
  RelGru2Args& r = a.gru;
  r.x = g->x0;
  r.rel_idx = g->gru_rel_idx;
  r.rel_start = g->gru_rel_start;
  r.rel_count = g->gru_rel_count;
  r.x_mean = g->gru_x_mean;
  r.emb_rel = g->gru_emb_rel;
  r.h_prev = g->gru_h_prev;
  r.w_ih_e = g->gru_w_ih_e;
  r.w_ih_x = g->gru_w_ih_x;
  r.w_hh = g->gru_w_hh;
  r.b_ih = g->gru_b_ih;
  r.b_hh = g->gru_b_hh;
  r.R2 = g->gru_R2;
  r.d = g->d;
  r.pre = g->gru_pre;
  r.h_out = g->gru_h_out;
  a.memo_h = g->memo_h;
  a.memo_x = g->memo_x;
  a.memo_r = g->memo_r;
  a.n_prev = a.memo_h ? g->n_prev : 0;
  if (a.memo_h) {
    if (!a.memo_x || !a.memo_r) return set_error(REGCN_EINVAL, "memo mode needs memo_h, memo_x, memo_r");
    if (a.n_prev < 0 || a.n_prev > REGCN_MAX_WINDOW) return set_error(REGCN_EINVAL, "n_prev out of range");
    for (int i = 0; i < a.n_prev; ++i) {
      a.prev_rows[i] = g->prev_rows[i];
      a.prev_rowptr[i] = g->prev_rowptr[i];
      a.prev_n_pos[i] = g->prev_n_pos[i];
      if (a.prev_n_pos[i] < 0 || (a.prev_n_pos[i] && (!a.prev_rows[i] || !a.prev_rowptr[i])))
        return set_error(REGCN_EINVAL, "earlier snapshot %d: null rows / rowptr", i);
    }
  }
  a.skip_zero_rows = a.memo_h ? 0 : g->skip_zero_rows;
  a.d = g->d;
  a.s1 = g->s1;
  a.tw = g->tw;
  a.x1 = g->x1;
  a.r1 = g->r1;
  a.h2 = g->h2;
  a.n2 = g->n2;
  return timestep_phase(a, phase, ST(s));
}

static int layer_args(const regcn_layer_desc* g, LayerArgs& a);

int regcn_layer_f32(const regcn_layer_desc* g, void* s) {
  if (!g) return set_error(REGCN_EINVAL, "null descriptor");
  LayerArgs a{};
  const int rc = layer_args(g, a);
  if (rc == -1) return set_error(REGCN_EINVAL, "gate_w / gate_out / step_tw are regcn_layer_rowtail_f32 fields");
  return rc ? rc : layer(a, ST(s));
}

int regcn_layer_rowtail_f32(const regcn_layer_desc* g, float* agg, void* s) {
  if (!g) return set_error(REGCN_EINVAL, "null descriptor");
  LayerArgs a{};
  const int rc = layer_args(g, a);
  return (rc && rc != -1) ? rc : layer_rowtail(a, agg, ST(s));
}

int regcn_layer_rowtail_part_f32(const regcn_layer_desc* g, float* agg, int32_t which, int32_t lo, int32_t hi,
                                 void* s) {
  if (!g) return set_error(REGCN_EINVAL, "null descriptor");
  LayerArgs a{};
  const int rc = layer_args(g, a);
  return (rc && rc != -1) ? rc : layer_rowtail_part(a, agg, which, lo, hi, ST(s));
}

size_t regcn_packed_weight_kp_floats(int32_t d_in) { return packed_weight_kp_floats(d_in); }

int regcn_pack_weight_kp_f32(const float* w, int32_t d_in, int32_t d_out, float* packed, void* s) {
  return pack_weight_kp(w, d_in, d_out, packed, ST(s));
}

static int layer_args(const regcn_layer_desc* g, LayerArgs& a) {
  a.agg_mode = g->agg_mode;
  a.x = g->x;
  a.radius = g->radius;
  a.rel = g->rel;
  a.w_rel = g->w_rel;
  a.nb = g->num_bases;
  a.gamma = g->gamma;
  a.rowptr = g->rowptr;
  a.col_src = g->col_src;
  a.col_type = g->col_type;
  a.norm = g->norm;
  a.budget = g->budget;
  a.tiles = g->tiles;
  a.n_pos_tiles = g->n_pos_tiles;
  a.item_ptr = g->item_ptr;
  a.item_src = g->item_src;
  a.item_tl = g->item_tl;
  a.agg = g->agg;
  a.w_n = g->w_n;
  a.w_loop = g->w_loop;
  a.w_evolve = g->w_evolve;
  a.prev_t = g->prev_t;
  a.w_skip = g->w_skip;
  a.b_skip = g->b_skip;
  a.drop_mask = g->drop_mask;
  a.rows = g->rows;
  a.n_pos = g->n_pos;
  a.V = g->V;
  a.d = g->d;
  a.euclid = g->euclid;
  a.k = make_curv(g->c);
  a.h_out = g->h_out;
  a.x_next = g->x_next;
  a.r_next = g->r_next;
  a.fuse_step = g->fuse_step;
  a.item_src_runs = g->item_src_runs;
  a.crel_tiles = g->crel_tiles;
  a.crel_item_src = g->crel_item_src;
  a.crel_item_tl = g->crel_item_tl;
  a.rel_t = g->rel_t;
  a.n_types = g->n_types;
  a.send_lo = g->send_lo;
  a.send_n = g->send_n;
  a.send_ptr = g->send_ptr;
  a.send_pos = g->send_pos;
  a.send_x = g->send_x;
  a.send_r = g->send_r;
  if (a.send_x && (!a.send_ptr || !a.send_pos || !a.send_r || a.send_n < 0 || a.send_lo < 0))
    return set_error(REGCN_EINVAL, "send block needs send_ptr, send_pos, send_r and send_n >= 0");
  if (a.item_src_runs && a.agg_mode != REGCN_AGG_UNION && a.agg_mode != REGCN_AGG_EUCLID)
    return set_error(REGCN_EINVAL, "item_src_runs applies to the union / euclid gathers only");
  if (g->fuse_step) {
    StepArgs& t = a.step;
    t.hc = nullptr;
    t.x_prev = g->step_x_prev;
    t.w_g = g->step_w_g;
    t.b_g = g->step_b_g;
    t.r_static = g->step_r_static;
    t.w_r = g->step_w_r;
    t.b_r = g->step_b_r;
    t.eps_r = g->step_eps_r;
    t.beta = g->step_beta;
    t.layer_norm = g->step_layer_norm;
    t.residual = g->step_residual;
    t.V = g->V;
    t.d = g->d;
    t.k = a.k;
    t.k_rad = make_curv(g->step_c_radius);
    t.h_out = g->step_h_out;
    t.x_out = g->step_x_out;
    t.r_out = g->step_r_out;
    t.tw = g->step_tw;
  }
  a.w_gate = g->gate_w;
  a.gate_out = g->gate_out;
  a.trace = g->trace;
  if (g->gate_w || g->gate_out || g->step_tw)
    return -1;  // marker: only regcn_layer_rowtail_f32 reads these (checked there)
  return 0;
}

int regcn_timestep_f32(const float* hc, const float* x_prev, const float* w_g, const float* b_g,
                       const float* r_static, const float* w_r, const float* b_r, float eps_r, float beta,
                       int32_t layer_norm, int32_t residual, int32_t V, int32_t d, float c, float c_radius,
                       float* h_out, float* x_out, float* r_out, void* s) {
  if (residual && !b_r) return set_error(REGCN_EINVAL, "residual radius needs b_r");
  StepArgs a{hc, x_prev, w_g, b_g, r_static, w_r, b_r, eps_r, beta, layer_norm, residual, V, d,
             make_curv(c), make_curv(c_radius), h_out, x_out, r_out};
  return timestep(a, ST(s));
}

int regcn_timestep_analysis_f32(const float* hc, const float* x_prev, const float* w_g, const float* b_g,
                                const float* r_static, const float* w_r, const float* b_r, float eps_r, float beta,
                                int32_t layer_norm, int32_t residual, int32_t V, int32_t d, float c, float c_radius,
                                float* h_out, float* x_out, float* r_out, float* gate_out, float* stat_out, void* s) {
  if (residual && !b_r) return set_error(REGCN_EINVAL, "residual radius needs b_r");
  StepArgs a{hc, x_prev, w_g, b_g, r_static, w_r, b_r, eps_r, beta, layer_norm, residual, V, d,
             make_curv(c), make_curv(c_radius), h_out, x_out, r_out, gate_out, stat_out};
  return timestep(a, ST(s), true);
}

size_t regcn_packed_linear_floats(int32_t n_gates, int32_t n_out, int32_t n_in) {
  return packed_linear_floats(n_gates, n_out, n_in);
}

int regcn_pack_linear_f32(const float* w, int32_t n_gates, int32_t n_out, int32_t n_in, float* packed, void* s) {
  return pack_linear(w, n_gates, n_out, n_in, packed, ST(s));
}

int regcn_relation_gru_f32(const float* x, const int32_t* rel_idx, const int32_t* rel_start, const float* rel_count,
                           const float* x_mean, const float* emb_rel, const float* h_prev, const float* w_ih,
                           const float* w_hh, const float* b_ih, const float* b_hh, int32_t R2, int32_t d,
                           float* h_out, void* s) {
  RelGruArgs a{x, rel_idx, rel_start, rel_count, x_mean, emb_rel, h_prev, w_ih, w_hh, b_ih, b_hh, R2, d, h_out};
  return rel_gru(a, ST(s));
}

int regcn_relation_gru_pre_f32(const float* emb_rel, const float* h_prev, const float* w_ih_e, const float* w_hh,
                               const float* b_ih, const float* b_hh, int32_t R2, int32_t d, float* pre, void* s) {
  RelGru2Args a{};
  a.emb_rel = emb_rel;
  a.h_prev = h_prev;
  a.w_ih_e = w_ih_e;
  a.w_hh = w_hh;
  a.b_ih = b_ih;
  a.b_hh = b_hh;
  a.R2 = R2;
  a.d = d;
  a.pre = pre;
  return rel_gru_pre(a, ST(s));
}

int regcn_relation_gru_x_f32(const float* x, const int32_t* rel_idx, const int32_t* rel_start,
                             const float* rel_count, const float* x_mean, const float* h_prev, const float* w_ih_x,
                             const float* pre, int32_t R2, int32_t d, float* h_out, void* s) {
  RelGru2Args a{};
  a.x = x;
  a.rel_idx = rel_idx;
  a.rel_start = rel_start;
  a.rel_count = rel_count;
  a.x_mean = x_mean;
  a.h_prev = h_prev;
  a.w_ih_x = w_ih_x;
  a.pre = const_cast<float*>(pre);
  a.R2 = R2;
  a.d = d;
  a.h_out = h_out;
  return rel_gru_x(a, ST(s));
}

int regcn_roth_query_f32(const float* ent, const float* rel, const int64_t* trip, int32_t n_test, int32_t B,
                         int32_t num_rels, const float* w1, const float* b1, const float* w2, const float* b2,
                         const float* w_rot, const float* b_rot, const float* w_trans, const float* b_trans, int32_t d,
                         float c, float* q_out, void* s) {
  QueryArgs a{};
  a.ent = ent;
  a.rel = rel;
  a.trip = trip;
  a.n_test = n_test;
  a.B = B;
  a.num_rels = num_rels;
  a.w1 = w1;
  a.b1 = b1;
  a.w2 = w2;
  a.b2 = b2;
  a.wrot = w_rot;
  a.brot = b_rot;
  a.wtr = w_trans;
  a.btr = b_trans;
  a.d = d;
  a.k = make_curv(c);
  a.q_out = q_out;
  return query(a, 0, ST(s));
}

int regcn_roth_rel_query_f32(const float* ent, const int64_t* trip, int32_t n_test, int32_t B, int32_t num_rels,
                             const float* w1, const float* b1, const float* w2, const float* b2,
                             const float* global_rot, const float* rel, int32_t n_cand, int32_t d, float c,
                             float* q_out, float* cand_out, void* s) {
  QueryArgs a{};
  a.ent = ent;
  a.rel = rel;
  a.trip = trip;
  a.n_test = n_test;
  a.B = B;
  a.num_rels = num_rels;
  a.w1 = w1;
  a.b1 = b1;
  a.w2 = w2;
  a.b2 = b2;
  a.global_rot = global_rot;
  a.n_cand = n_cand;
  a.d = d;
  a.k = make_curv(c);
  a.q_out = q_out;
  a.cand_out = cand_out;
  return query(a, 1, ST(s));
}

static ScoreArgs score_args(const float* q, const float* cand, const float* bias, const float* c_rel, const float* scale, const float* margin,
                            int32_t B, int32_t N, int32_t d, float c, int32_t use_dist) {
  ScoreArgs a{};
  Curv k = make_curv(c);
  a.q = q; a.e = cand; a.bias = bias; a.c_r = c_rel;
  a.B = B; a.N = N; a.d = d; a.use_dist = use_dist & 1; a.scale_raw = (use_dist >> 1) & 1;
  a.c = k.c; a.sqrt_c = k.sqrt_c; a.mx = k.mx;
  a.dist_mx = (float)(1.0 / (sqrt((double)c) + 1e-6) - 1e-6);
  a.scale_p = scale; a.margin_p = margin;
  return a;
}

int regcn_hyp_score_f32(const float* q, const float* cand, const float* bias, const float* c_rel, const float* scale, const float* margin, int32_t B,
                        int32_t N, int32_t d, float c, int32_t use_dist, float* out, void* s) {
  if (c_rel && !(use_dist & 1)) return set_error(REGCN_EINVAL, "per-query curvature requires use_dist");
  ScoreArgs a = score_args(q, cand, bias, c_rel, scale, margin, B, N, d, c, use_dist);
  a.out = out;
  return score(a, 0, nullptr, ST(s));
}

size_t regcn_packed_k4_floats(int32_t n_out, int32_t n_in) { return packed_k4_floats(n_out, n_in); }
int regcn_pack_k4_f32(const float* W, int32_t n_out, int32_t n_in, float* out, void* s) {
  return pack_k4(W, n_out, n_in, out, ST(s));
}
int regcn_roth_queries_f32(const regcn_roth_queries_desc* desc, void* s) {
  if (!desc) return set_error(REGCN_EINVAL, "null desc");
  return roth_queries(*desc, ST(s));
}

int regcn_hyp_score_jobs_f32(const regcn_score_job* jobs, int32_t n_jobs, void* s) {
  if (!jobs || n_jobs < 1 || n_jobs > 2) return set_error(REGCN_EINVAL, "1 or 2 score jobs");
  ScoreArgs a[2];
  for (int i = 0; i < 2; ++i) {
    const regcn_score_job& j = jobs[i < n_jobs ? i : 0];
    if (j.flags & REGCN_SCORE_DIST) return set_error(REGCN_ENOTSUP, "score jobs compute the proxy score only");
    a[i] = score_args(j.q, j.cand, j.bias, nullptr, j.scale, j.margin, j.B, i < n_jobs ? j.N : 0, j.d, j.c, j.flags);
    a[i].out = j.out;
  }
  return score_jobs(a[0], a[1], ST(s));
}

size_t regcn_hyp_ce_workspace_bytes(int32_t B, int32_t N) {
  return ((size_t)B * ce_partial_slots(N) * 2 + (size_t)B) * sizeof(float);
}

int regcn_hyp_ce_f32(const float* q, const float* cand, const float* bias, const float* c_rel, const float* scale, const float* margin,
                     const int32_t* target, int32_t B, int32_t N, int32_t d, float c, int32_t use_dist,
                     void* workspace, float* loss_per_query, void* s) {
  if (c_rel && !(use_dist & 1)) return set_error(REGCN_EINVAL, "per-query curvature requires use_dist");
  if (!workspace) return set_error(REGCN_EINVAL, "null workspace");
  ScoreArgs a = score_args(q, cand, bias, c_rel, scale, margin, B, N, d, c, use_dist);
  const size_t nblk = ce_partial_slots(N);
  a.target = target;
  a.part = (float*)workspace;
  a.tgt_logit = a.part + (size_t)B * nblk * 2;
  return score(a, 1, loss_per_query, ST(s));
}

int regcn_rank_f32(const float* score_m, int32_t B, int32_t N, const int32_t* target, const int32_t* filt_ptr,
                   const int32_t* filt_idx, int32_t* rank_raw, int32_t* rank_filt, void* s) {
  return rank(score_m, B, N, target, nullptr, filt_ptr, filt_idx, 1, rank_raw, rank_filt, ST(s));
}
int regcn_rank_count_f32(const float* score_m, int32_t B, int32_t N, const float* threshold, const int32_t* filt_ptr,
                         const int32_t* filt_idx, int32_t* count_raw, int32_t* count_filt, void* s) {
  if (!threshold) return set_error(REGCN_EINVAL, "null threshold");
  return rank(score_m, B, N, nullptr, threshold, filt_ptr, filt_idx, 0, count_raw, count_filt, ST(s));
}

int regcn_hyp_rank_fused_f32(const float* q, const float* cand, const float* bias, const float* scale,
                             const float* margin, const float* threshold, int32_t B, int32_t N, int32_t d, float c,
                             int32_t flags, const int32_t* ranges, int32_t n_ranges, void* workspace,
                             int32_t accumulate, int32_t* counts, void* s) {
  if (flags & ~REGCN_SCORE_RAW_SCALE) return set_error(REGCN_ENOTSUP, "fused rank count: proxy score flags only");
  if (!workspace && B > 0) return set_error(REGCN_EINVAL, "null workspace");
  if (n_ranges < 0 || n_ranges > SCORE_MAX_RANGES || (n_ranges > 0 && !ranges))
    return set_error(REGCN_EINVAL, "fused rank count takes 0..%d candidate ranges", SCORE_MAX_RANGES);
  ScoreArgs a = score_args(q, cand, bias, nullptr, scale, margin, B, N, d, c, flags);
  int tiles = 0, k = 0;
  for (int r = 0; r < n_ranges; ++r) {  // host array {start, end} per range; empty ranges dropped
    const int lo = ranges[2 * r], hi = ranges[2 * r + 1];
    if (lo < 0 || hi < lo || hi > N) return set_error(REGCN_EINVAL, "candidate range [%d, %d) outside [0, %d)", lo, hi, N);
    if (hi == lo) continue;
    a.rng_start[k] = lo;
    a.rng_len[k] = hi - lo;
    a.rng_tile[k] = tiles;
    tiles += (hi - lo + 63) / 64;
    ++k;
  }
  a.n_rng = n_ranges ? k : 0;
  a.rng_tile[a.n_rng] = tiles;
  a.rng_total = tiles;
  if (n_ranges && !k) a.N = 0;  // every range empty
  a.thr = threshold;
  a.part = (float*)workspace;
  return rank_fused(a, accumulate, counts, ST(s));
}

int regcn_pack_rows_f32(const float* x, const float* radius, const int64_t* ids, int64_t n, int32_t d, float* out,
                        void* s) {
  return exchange_rows(1, const_cast<float*>(x), const_cast<float*>(radius), ids, n, d, out, ST(s));
}
int regcn_gather_rows_f32(const float* x, const float* radius, const int64_t* ids, int64_t n, int32_t d, float* x_out,
                          float* r_out, void* s) {
  return gather_rows(x, radius, ids, n, d, x_out, r_out, ST(s));
}
int regcn_unpack_rows_f32(const float* in, const int64_t* ids, int64_t n, int32_t d, float* x, float* radius, void* s) {
  return exchange_rows(0, x, radius, ids, n, d, const_cast<float*>(in), ST(s));
}

size_t regcn_snapshot_workspace_bytes(int64_t T, int32_t V, int32_t R) { return snapshot_ws_bytes(T, V, R); }
int64_t regcn_snapshot_capacity(int32_t what, int64_t T, int32_t V, int32_t R, int32_t chunk_edges) {
  return snapshot_capacity(what, T, V, R, chunk_edges);
}
int regcn_snapshot_csr_i32(const regcn_snapshot_desc* desc, void* s) { return snapshot_csr(desc, ST(s)); }
int regcn_snapshot_work_i32(const regcn_snapshot_desc* desc, void* s) { return snapshot_work(desc, ST(s)); }

int regcn_hyp_ce_lse_f32(const float* q, const float* cand, const float* bias, const float* scale,
                         const float* margin, const int32_t* target, int32_t B, int32_t N, int32_t d, float c,
                         int32_t flags, void* workspace, float* loss_per_query, float* lse, void* s) {
  if (!workspace) return set_error(REGCN_EINVAL, "null workspace");
  ScoreArgs a = score_args(q, cand, bias, nullptr, scale, margin, B, N, d, c, flags);
  const size_t nblk = ce_partial_slots(N);
  a.target = target;
  a.part = (float*)workspace;
  a.tgt_logit = a.part + (size_t)B * nblk * 2;
  a.lse_out = lse;
  return score(a, 1, loss_per_query, ST(s));
}
int regcn_hyp_ce_bwd_f32(const float* q, const float* cand, const float* bias, const float* scale,
                         const float* margin, const int32_t* target, const float* lse, const float* grad_loss,
                         int32_t B, int32_t N, int32_t d, float c, int32_t flags, float* coef, float* rsum,
                         float* csum, void* s) {
  ScoreArgs a = score_args(q, cand, bias, nullptr, scale, margin, B, N, d, c, flags);
  a.target = target;
  a.lse = lse;
  a.gl = grad_loss;
  a.coef = coef;
  a.rsum = rsum;
  a.csum = csum;
  return score_ce_bwd(a, ST(s));
}
int regcn_rowmap_bwd_f32(int32_t op, const float* x, const float* y, const float* g, int64_t rows, int32_t d,
                         float c, float* dx, float* dy, void* s) {
  return rowmap_bwd(op, x, y, g, rows, d, c, dx, dy, ST(s));
}
int regcn_union_aggregate_bwd_f32(const regcn_edge_bwd_desc* desc, float gamma, void* s) {
  if (!desc) return set_error(REGCN_EINVAL, "null descriptor");
  return union_bwd(desc, gamma, ST(s));
}
int regcn_lorentz_sum_raw_f32(const float* x, const float* rel, const float* weight, const int32_t* rowptr,
                              const int32_t* col_src, const int32_t* col_type, int32_t V, int32_t d, int32_t num_bases,
                              float c, float* S0, float* Sv, void* s) {
  return lorentz_raw(x, rel, weight, rowptr, col_src, col_type, V, d, num_bases, c, S0, Sv, ST(s));
}
int regcn_lorentz_aggregate_bwd_f32(const regcn_edge_bwd_desc* desc, int32_t num_bases, float c, void* s) {
  if (!desc) return set_error(REGCN_EINVAL, "null descriptor");
  return lorentz_bwd(desc, num_bases, c, ST(s));
}
size_t regcn_transpose_workspace_bytes(int32_t E, int32_t V, int32_t R2) { return transpose_ws_bytes(E, V, R2); }
int regcn_snapshot_transpose_i32(const regcn_transpose_desc* desc, void* s) { return snapshot_transpose(desc, ST(s)); }
size_t regcn_item_src_order_workspace_bytes(int32_t n_items, int32_t V) { return item_src_ws_bytes(n_items, V); }
int regcn_snapshot_item_src_order_i32(int32_t V, int32_t n_tiles, int32_t n_items, const int32_t* tiles,
                                      const int32_t* item_ptr, const int32_t* item_src, const int32_t* item_tl,
                                      int32_t* out_src, int32_t* out_tl, void* workspace, size_t ws_bytes, void* s) {
  return item_src_order(V, n_tiles, n_items, tiles, item_ptr, item_src, item_tl, out_src, out_tl, workspace, ws_bytes,
                        ST(s));
}
int regcn_snapshot_item_type_order_i32(int32_t V, int32_t R2, int32_t n_tiles, int32_t n_items, const int32_t* tiles,
                                       const int32_t* item_ptr, const int32_t* item_src, const int32_t* item_tl,
                                       int32_t* out_src, int32_t* out_tl, void* workspace, size_t ws_bytes, void* s) {
  return item_type_order(V, R2, n_tiles, n_items, tiles, item_ptr, item_src, item_tl, out_src, out_tl, workspace,
                         ws_bytes, ST(s));
}
size_t regcn_row_src_order_workspace_bytes(int32_t E, int32_t V) { return row_src_ws_bytes(E, V); }
int regcn_snapshot_row_src_order_i32(int32_t V, int32_t E, const int32_t* rowptr, const int32_t* col_src, int32_t* out_src,
                                     void* workspace, size_t ws_bytes, void* s) {
  return row_src_order(V, E, rowptr, col_src, out_src, workspace, ws_bytes, ST(s));
}
size_t regcn_row_type_order_workspace_bytes(int32_t E, int32_t V, int32_t R2) { return row_type_ws_bytes(E, V, R2); }
int regcn_snapshot_row_type_order_i32(int32_t V, int32_t E, int32_t R2, const int32_t* rowptr, const int32_t* col_src,
                                      const int32_t* col_type, int32_t* out_src, int32_t* out_type, void* workspace,
                                      size_t ws_bytes, void* s) {
  return row_type_order(V, E, R2, rowptr, col_src, col_type, out_src, out_type, workspace, ws_bytes, ST(s));
}

}  // extern "C"
