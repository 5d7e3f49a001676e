// Host-side internals shared by the kernel translation units (not part of the C-ABI).
#pragma once
#include <algorithm>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/regcn_hip.h"
#include "common.h"

namespace regcn {

extern int64_t* g_trace;  // regcn_set_trace (profiling)

int set_error(int code, const char* fmt, ...);
int check_launch(const char* what);

inline Curv make_curv(double c) {
  Curv k;
  double sc = sqrt(c);
  k.c = (float)c;
  k.sqrt_c = (float)sc;
  k.mx = (float)(1.0 / sc - 1e-6 - 1e-6);
  k.rmax = (float)(1.0 / sc - 1e-6);
  k.atanh_mx = (float)(1.0 - 1e-6);
  return k;
}

// rowwise.hip
int rowmap(int op, const float* a, const float* b, const float* vec, int64_t rows, int d, float c,
           float* out, float* out2, float* out3, hipStream_t st);
int init_rows(const float* dyn, const float* r_static, const int32_t* src, const int32_t* dst, int64_t n, int d,
              float c, int layer_norm, float* h, float* x, float* r, hipStream_t st);

// aggregate.hip
int gather_sum(int mode, const float* x, const float* radius, const float* rel, const int* col_src,
               const int* col_type, const float* rowscale, const void* chunks, int n_chunks,
               const void* fixups, int n_fix, float gamma, int d, float* partial, int pstride, float* out,
               hipStream_t st, const int* col_src_s = nullptr);
int partial_sum(float* partial, int pstride, const void* fixups, int n_fix, int width, float* out, int ostride,
                hipStream_t st);
int lorentz_sum(const float* x, const float* rel, const float* W, const int* col_src, const int* col_type,
                const void* chunks, int n_chunks, const void* fixups, int n_fix, int nb, float c, int d,
                float* partial, int pstride, float* out, hipStream_t st);

// backward.hip
int rowmap_bwd(int op, const float* x, const float* y, const float* g, int64_t rows, int d, float c, float* dx,
               float* dy, hipStream_t st);
int union_bwd(const regcn_edge_bwd_desc* a, float gamma, hipStream_t st);
int lorentz_raw(const float* x, const float* rel, const float* W, const int* rowptr, const int* col_src,
                const int* col_type, int V, int d, int nb, float c, float* S0, float* Sv, hipStream_t st);
int lorentz_bwd(const regcn_edge_bwd_desc* a, int nb, float c, hipStream_t st);

// graphbuild.hip
int snapshot_transpose(const regcn_transpose_desc* d, hipStream_t st);
size_t transpose_ws_bytes(int E, int V, int R2);
size_t row_type_ws_bytes(int E, int V, int R2);
int row_type_order(int V, int E, int R2, const int* rowptr, const int* col_src, const int* col_type, int* out_src,
                   int* out_type, void* ws, size_t ws_bytes, hipStream_t st);
size_t item_src_ws_bytes(int n_items, int V);
int item_src_order(int V, int n_tiles, int n_items, const int* tiles, const int* item_ptr, const int* item_src,
                   const int* item_tl, int* out_src, int* out_tl, void* ws, size_t ws_bytes, hipStream_t st);
int item_type_order(int V, int R2, int n_tiles, int n_items, const int* tiles, const int* item_ptr,
                    const int* item_src, const int* item_tl, int* out_src, int* out_tl, void* workspace,
                    size_t ws_bytes, hipStream_t st);
size_t row_src_ws_bytes(int E, int V);
int row_src_order(int V, int E, const int* rowptr, const int* col_src, int* out_src, void* ws, size_t ws_bytes,
                  hipStream_t st);
int snapshot_csr(const regcn_snapshot_desc* d, hipStream_t st);
int snapshot_work(const regcn_snapshot_desc* d, hipStream_t st);
size_t snapshot_ws_bytes(int64_t T, int V, int R);
int64_t snapshot_capacity(int what, int64_t T, int V, int R, int C);

// ---- argument blocks of the fused kernels (layer.hip, score.hip) ----
struct StepArgs {
  const float* hc;
  const float* x_prev;
  const float* w_g;
  const float* b_g;
  const float* r_static;
  const float* w_r;
  const float* b_r;   // device scalar
  float eps_r, beta;
  int layer_norm, residual, V, d;
  Curv k;       // model curvature (tensor c)
  Curv k_rad;   // TemporalRadiusEvolution's constructor-time c (hyperbolic_ops.py:385, :406)
  float* h_out;
  float* x_out;
  float* r_out;
  float* gate_out;  // --run-analysis (k_timestep<true>): V x d time gate
  float* stat_out;  // 3 x V: clipped radius delta, dynamic radius, base radius (residual only)
  const float* tw;  // rowtail: precomputed gate pre-activation rows clamp(x_prev) @ W_g, or null
};

// One message-passing layer: inline CSR gather + self-loop/neighbour GEMMs + epilogue,
// optionally followed by the timestep (layer.hip).  Weights are prepacked.
struct LayerArgs {
  int agg_mode;             // AGG_UNION / AGG_EUCLID / AGG_LORENTZ (inline gather) or AGG_NONE
  const float* x;           // V x d layer input (tangent rows; raw rows for euclid)
  const float* radius;      // V, union message weights
  const float* rel;         // R2 x d relation rows
  const float* w_rel;       // R2 x nb*s*s Lorentz block weights
  int nb;
  float gamma;
  const int* rowptr;        // V + 1, destination-sorted CSR
  const int* col_src;
  const int* col_type;
  const float* norm;        // V, union / euclid row scale
  int budget;               // rows with in-degree > budget read `agg` (pre-aggregated)
  const int* tiles;         // n_pos_tiles x {start, count} over rows[0, n_pos); null: 16-row tiles
  int n_pos_tiles;
  const int* item_ptr;      // n_pos_tiles + 1: each tile's in-edge items
  const int* item_src;      // source entity of each item
  const int* item_tl;       // relation type << 4 | tile-local destination row
  const float* agg;         // V x d pre-aggregated rows (heavy rows; every pos row for AGG_NONE)
  const float* w_n;
  const float* w_loop;
  const float* w_evolve;
  const float* prev_t;
  const float* w_skip;
  const float* b_skip;
  const float* drop_mask;
  const int* rows;          // V: rows with in-degree > 0 first (n_pos), then the rest
  int n_pos, V, d, euclid;
  Curv k;
  float* h_out;
  float* x_next;
  float* r_next;
  int fuse_step;            // run the timestep on the layer output (step.hc unused)
  StepArgs step;
  int64_t* trace;           // debug: 8 phase timestamps per workgroup, or null
  int item_src_runs;        // union / euclid items in (row, source) order: one x row per source run
  const float* w_gate;      // rowtail, a cell's first layer: W_g (kp-packed) ...
  float* gate_out;          // ... and the V x d rows clamp(x) @ W_g it writes for the timestep
  // rowtail gather, union / euclid: tiles [0, crel_tiles) sum their relation weights per (row,
  // type) and apply the relation rows as one MFMA product per tile (rowtail.hip k_gather_crel)
  int crel_tiles;
  const int* crel_item_src;  // those tiles' items in (row, type) order
  const int* crel_item_tl;
  const float* rel_t;        // ceil(d / 16) 16 x crel_kpad(n_types): rel transposed, zero padded
  int n_types;               // R2 <= 512
  // rowtail tail: the halo exchange's send block written alongside x_next / step.x_out (row id
  // i -> slots send_pos[send_ptr[i - send_lo] ..]), send_x null when off
  int64_t send_lo;
  int send_n;
  const int* send_ptr;
  const int* send_pos;
  float* send_x;
  float* send_r;
};

struct ScoreArgs {
  const float* q;
  const float* e;
  const float* bias;     // [N] or null
  const float* c_r;      // [B] or null (per-query curvature, true-distance mode only)
  const int* target;     // [B] (CE mode)
  int B, N, d;
  int use_dist;
  float c, sqrt_c, mx, dist_mx;
  const float* scale_p;  // device scalar or null (1.0): softplus(raw) + 1e-6, hyperbolic_decoder.py:717
  const float* margin_p; // device scalar or null (0.0)
  int scale_raw;         // scale_p holds the raw parameter: softplus(raw) + 1e-6 in-kernel
  float scale, margin;   // filled in-kernel from the pointers
  float* out;            // [B, N] score (SCORE mode)
  float* part;           // [B, nblk, 2] (CE mode): running max, sum exp
  float* tgt_logit;      // [B] (CE mode)
  int64_t* trace;        // profiling stamps (g_trace at launch), or null
  float* lse_out;        // [B] (CE mode, optional): log-sum-exp per query
  // CE backward (MODE 2): G[b,n] = gl[b] (softmax - onehot), coefficients of dS/d(xy, x2, y2)
  const float* lse;      // [B]
  const float* gl;       // [B] upstream gradient of each query's loss
  float* coef;           // [B, N]: G dS/dxy
  float* rsum;           // [B, nblk]: per candidate block, sum_n G dS/dx2
  float* csum;           // [ngroups16, N, 3]: per 16-query group, sum_b (G dS/dy2, G, G (margin - n^2))
  // fused rank count (MODE 3): per query #{n : S[b,n] > thr[b]}, partial counts in `part`
  const float* thr;      // [B]
  // candidate row ranges (n_rng > 0): the candidates are rows [rng_start[r], rng_start[r] +
  // rng_len[r]) of e, tiled range by range (range r's tiles [rng_tile[r], rng_tile[r + 1])),
  // so one launch covers a rank's owner ranges; n_rng == 0: rows [0, N)
  int n_rng, rng_total;  // rng_total = rng_tile[n_rng] (device code indexes the arrays statically only)
  int bal;               // MODE 0, > 0: balanced grid, query tile blk % nbq takes candidate tiles
                         // blk / nbq + bal i (set by the launcher for small candidate sets)
  int rng_start[8], rng_len[8], rng_tile[9];
};

constexpr int SCORE_MAX_RANGES = 8;

// Relation GRU of one timestep (relgru.hip).
struct RelGruArgs {
  const float* x;          // V x d entity tangent rows (x_mean source)
  const int* rel_idx;      // r_to_e entity ids
  const int* rel_start;    // R2 span starts into rel_idx
  const float* rel_count;  // R2 span lengths (0: relation absent)
  const float* x_mean;     // R2 x d precomputed means, or null (gather in-kernel)
  const float* emb_rel;    // R2 x d
  const float* h_prev;     // R2 x d GRU state
  const float* w_ih;       // packed (pack_linear, 3 gates, d x 2d)
  const float* w_hh;       // packed (3 gates, d x d)
  const float* b_ih;
  const float* b_hh;
  int R2, d;
  float* h_out;
  int64_t* trace;  // profiling stamps (g_trace at launch), or null
};

// Two-phase relation GRU (relgru.hip k_gru_pre / k_gru_x).
struct RelGru2Args {
  const float* x;          // V x d entity tangent rows (x_mean source)
  const int* rel_idx;
  const int* rel_start;
  const float* rel_count;
  const float* x_mean;     // R2 x d precomputed means, or null (gathered in-kernel)
  const float* emb_rel;    // R2 x d
  const float* h_prev;     // R2 x d GRU state
  const float* w_ih_e;     // packed (3 gates, d x d): W_ih[:, :d]
  const float* w_ih_x;     // packed (3 gates, d x d): W_ih[:, d:]
  const float* w_hh;       // packed (3 gates, d x d)
  const float* b_ih;
  const float* b_hh;
  int R2, d;
  float* pre;              // R2 x 4 x d gate partials (k_gru_pre out, k_gru_x in)
  float* h_out;
};
int rel_gru_pre(const RelGru2Args& a, hipStream_t st);
int rel_gru_x(const RelGru2Args& a, hipStream_t st);

// History-window plan and the cold-row chain (window.hip).
struct PlanArgs {
  int T, V;
  const int* pos_rows[REGCN_MAX_WINDOW];  // rows[:n_pos] of each snapshot
  int n_pos[REGCN_MAX_WINDOW];
  int* flags;    // V scratch
  int* c_rows;   // V: rows without in-edges in every snapshot
  int* u_rows;   // V: the others
  int* z_rows;   // T x z_stride: U rows without in-edges at t
  int z_stride;
  int* counts;   // 2 + T: |C|, |U|, |Z_t|
};
int window_plan(const PlanArgs& a, hipStream_t st);

struct ChainArgs {
  const int* rows;     // C rows
  const int* n_rows;   // device count
  int T, d;
  const float* x0;     // log0(h_init) rows
  const float* w_evolve0;
  const float* w_evolve1;
  const float* w_skip1;
  const float* b_skip1;
  Curv k;
  StepArgs step;       // per-timestep outputs below
  float* h_out[REGCN_MAX_WINDOW];
  float* x_out[REGCN_MAX_WINDOW];
  float* r_out[REGCN_MAX_WINDOW];
};
int cold_chain(const ChainArgs& a, int grid_bound, hipStream_t st);
int zero_step(const ChainArgs& a, int n_rows, hipStream_t st);

// One timestep of a 2-layer cell in three phase launches (timestep.hip).
struct PhaseArgs {
  LayerArgs L[2];     // layer 0 / 1: snapshot lists, inputs (x, radius, rel, prev_t), weights
  StepArgs step;      // x_prev = x0 (the timestep input), outputs h/x/r
  RelGru2Args gru;    // phase A: x-half of this timestep's GRU; phase B: pre-half of the next
  int d;
  float* s1;          // V x d: x0 @ W_loop[0] (in-edge rows)
  float* tw;          // V x d: clamp(x0) @ W_g (in-edge rows)
  float* x1;          // V x d: layer-0 output tangent rows
  float* r1;          // V: |layer-0 output|
  float* h2;          // V x d: layer-1 output of rows without in-edges (Poincare)
  float* n2;          // V: its |.|^2 as the epilogue carries it
  // memo mode (memo_h != NULL, regcn_phase_desc): pristine rows copy memo_* in phase A; the
  // rows without in-edges that run come from the earlier snapshots' in-edge rows
  const float* memo_h;
  const float* memo_x;
  const float* memo_r;
  int n_prev;
  const int* prev_rows[REGCN_MAX_WINDOW];
  const int* prev_rowptr[REGCN_MAX_WINDOW];
  int prev_n_pos[REGCN_MAX_WINDOW];
  int skip_zero_rows;  // plain mode: the rows without in-edges run in k_zero_step instead
  int n_pos_rt, n_zero_rt, n_gru, gru_rt, n_copy;  // block counts (set by the launcher)
  int64_t* trace;     // profiling (regcn_set_trace): {start, end} s_memrealtime per workgroup
};
int timestep_phase(PhaseArgs a, int phase, hipStream_t st);

// RotH decoder queries (query.hip).  Linear weights are packed transposed (x @ W^T).
struct QueryArgs {
  const float* ent;         // V x d final entity embedding
  const float* rel;         // R2 x d relation embedding (RotH: query rows; RotHRel: candidates)
  const int64_t* trip;      // n_test x 3 test triples (s, r, o)
  int n_test, B, num_rels;  // B <= 2 n_test queries: forward then inverse
  const float* w1;          // reshape_fc1 / fc2
  const float* b1;
  const float* w2;
  const float* b2;
  const float* wrot;        // RotH rot_proj (d -> d/2)
  const float* brot;
  const float* wtr;         // RotH trans_proj
  const float* btr;
  const float* global_rot;  // RotHRel (d/2)
  int n_cand;               // RotHRel: rows of exp0(rel) written to cand_out
  int d;
  Curv k;
  float* q_out;             // B x d
  float* cand_out;
};
int query(const QueryArgs& a, int mode, hipStream_t st);
// queries.hip: a predict's RotH + RotHRel queries, candidates and all_triples in one launch
size_t packed_k4_floats(int n_out, int n_in);
int pack_k4(const float* W, int n_out, int n_in, float* out, hipStream_t st);
int roth_queries(const regcn_roth_queries_desc& a, hipStream_t st);

size_t packed_linear_floats(int n_gates, int n_out, int n_in);
int pack_linear(const float* W, int n_gates, int n_out, int n_in, float* Wp, hipStream_t st);
int rel_gru(const RelGruArgs& a, hipStream_t st);

size_t packed_weight_floats(int d_in);
int pack_weight(const float* W, int d_in, int d_out, float* Wp, hipStream_t st);
size_t kreduce_workspace_floats(int64_t K, int M, int N);
struct TailArgs {
  const float *agg, *lx, *ex, *z, *bias, *p, *gy;
  const uint8_t* pos;
  float *out, *dagg, *dlx, *dex, *dz, *dp;
  int64_t V, loop_ld;
  int d, flags;
  float slope;
};
int tail(const TailArgs& t, int backward, hipStream_t st);
int givens(const float* x, const float* ang, int64_t n_pairs, int reflect, const float* gy, float* out, float* dx, float* dang,
           hipStream_t st);
int centroid(const float* S0, const float* Sv, int64_t V, int d, float c, float sqc, const float* gy, float* y,
             float* dS0, float* dSv, hipStream_t st);
int kreduce_gemm(const float* A, int a_kmajor, const float* B, int b_kmajor, int64_t K, int M, int N, const float* C0,
                 int64_t c0_ld, float* out, float* ws, hipStream_t st);
int layer(const LayerArgs& a, hipStream_t st);
// rowtail.hip: large snapshots' layer as an agg gather + a 64-row MFMA tail (k-permuted packing)
size_t packed_weight_kp_floats(int d_in);
int pack_weight_kp(const float* W, int d_in, int d_out, float* Wp, hipStream_t st);
int layer_rowtail(const LayerArgs& a, float* agg, hipStream_t st);
int layer_rowtail_part(const LayerArgs& a, float* agg, int which, int lo, int hi, hipStream_t st);
int timestep(const StepArgs& a, hipStream_t st, bool analysis = false);
int score(ScoreArgs& a, int mode, float* loss, hipStream_t st);
int score_jobs(ScoreArgs& a0, ScoreArgs& a1, hipStream_t st);
// CE partial (max, sum exp) slots per query: one per candidate tile (generic kernel) or one per
// workgroup of the query's tile (persistent fp32 kernel, <= 8 x 32).
inline size_t ce_partial_slots(int N) { return std::max<size_t>(((size_t)N + 63) / 64, 256); }
int score_ce_bwd(ScoreArgs& a, hipStream_t st);
int exchange_rows(int pack, float* x, float* r, const int64_t* idx, int64_t n, int d, float* buf, hipStream_t st);
int gather_rows(const float* x, const float* r, const int64_t* idx, int64_t n, int d, float* x_out, float* r_out,
                hipStream_t st);
int rank_fused(ScoreArgs& a, int accumulate, int* counts, hipStream_t st);
int rank(const float* S, int B, int N, const int* target, const float* ts, const int* filt_ptr, const int* filt_idx,
         int add, int* rank_raw, int* rank_filt, hipStream_t st);

}  // namespace regcn
