/*
 * regcn_hip.h — C-ABI of libregcn_hip.so, the MI355X (gfx950) hot path of RE-GCN.
 *
 * This is the drop-in boundary for the per-timestep relational message passing
 * + hyperbolic scoring loop of sgxxyyds/RE-GCN (BASELINE.json north_star).  Each
 * entry point names the reference interface it replaces (file:line under the
 * reference tree).  A host binding (ctypes in re-gcn_amd/regcn_amd/_lib.py; see
 * INTEGRATION.md for the stub a reference maintainer would add) calls these
 * with device pointers from the caller's allocator.
 *
 * Conventions
 *  - Plain pointers and sizes only; every pointer is device memory, fp32 data,
 *    int32 indices, rows contiguous and row-major.
 *  - `stream` is a hipStream_t (passed as void*); all work is enqueued
 *    asynchronously on it.  No call allocates, frees or synchronises, so every
 *    call may be captured into a hipGraph.
 *  - Return value: 0 on success; a positive hipError_t if a launch failed;
 *    a negative REGCN_E* code for an argument error.  The thread-local
 *    regcn_last_error_string() describes the most recent failure.
 *  - Curvature `c` is the ball curvature (Poincaré ball c|x|^2 < 1).
 */
#ifndef REGCN_HIP_H
#define REGCN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define REGCN_ABI_VERSION 13
#define REGCN_EINVAL (-1)
#define REGCN_ENOTSUP (-2)

/* Snapshot work lists built by the host (re-gcn_amd/regcn_amd/graph.py):
 * chunks: int32[n_chunks][4] = {row, edge_begin, edge_end, slot}; slot < 0 means
 *         the row is finished by that chunk, slot >= 0 names its partial row.
 * fixups: int32[n_fix][4]    = {row, slot_begin, slot_end, out}: out = 0 finishes `row`
 *         from the slots' sum; out = k > 0 is a first-level group whose raw sum goes to
 *         partial slot k - 1 (summed before any out = 0 entry; the host cuts rows with more
 *         than 64 slots into such groups).  `partial` is written by the groups. */

int regcn_version(void);
const char* regcn_last_error_string(void);
/* Profiling hook (not needed in production): while `buf` is non-NULL, the relation GRU,
 * query and score launches write per-workgroup phase timestamps (s_memrealtime, 100 MHz;
 * 16 int64 slots per workgroup, indexed by the flattened workgroup id) into it. */
int regcn_set_trace(int64_t* buf);

/* ---- a3: Poincaré / Lorentz row maps (hyperbolic_src/hyperbolic_ops.py) ------------ */
/* HyperbolicOps.log_map_zero, hyperbolic_ops.py:97-116 */
int regcn_log0_f32(const float* x, int64_t rows, int32_t d, float c, float* out, void* stream);
/* HyperbolicOps.exp_map_zero (+ project_to_ball), hyperbolic_ops.py:76-95 */
int regcn_exp0_f32(const float* v, int64_t rows, int32_t d, float c, float* out, void* stream);
/* HyperbolicOps.project_to_ball, hyperbolic_ops.py:55-74 */
int regcn_project_f32(const float* x, int64_t rows, int32_t d, float c, float* out, void* stream);
/* HyperbolicOps.apply_radius, hyperbolic_ops.py:208-233 (radius: one value per row) */
int regcn_apply_radius_f32(const float* x, const float* radius, int64_t rows, int32_t d, float c, float* out,
                           void* stream);
/* HyperbolicOps.get_radius, hyperbolic_ops.py:193-206 */
int regcn_radius_f32(const float* x, int64_t rows, int32_t d, float* out, void* stream);
/* row |x|^2 (scorer operand norms) */
int regcn_sumsq_f32(const float* x, int64_t rows, int32_t d, float* out, void* stream);
/* HyperbolicOps.mobius_add, hyperbolic_ops.py:118-143 */
int regcn_mobius_add_f32(const float* x, const float* y, int64_t rows, int32_t d, float c, float* out,
                         void* stream);
/* LorentzOps.to_lorentz, hyperbolic_ops.py:476-499 (out: rows x (d+1)) */
int regcn_to_lorentz_f32(const float* x, int64_t rows, int32_t d, float c, float* out, void* stream);
/* LorentzOps.to_poincare, hyperbolic_ops.py:501-518 (y: rows x (d+1)) */
int regcn_to_poincare_f32(const float* y, int64_t rows, int32_t d, float c, float* out, void* stream);
/* Fused layer prologue: x = log0(h), r = get_radius(h)
 * (hyperbolic_layers.py:268-270, hyperbolic_model.py:802) */
int regcn_prologue_f32(const float* h, int64_t rows, int32_t d, float c, float* x_out, float* r_out,
                       void* stream);
/* exp0(normalize(log0(x))): layer-norm round trip, hyperbolic_model.py:832-835, :926-929 */
int regcn_ln_roundtrip_f32(const float* x, int64_t rows, int32_t d, float c, float* out, void* stream);
/* Initial entity state, hyperbolic_model.py:779-782: h = apply_radius(exp0([normalize]dyn), r_static);
 * also emits x = log0(h) and r = |h| for the first timestep (x_out/r_out may be NULL; h_out may be
 * NULL when x_out is not: the fused timestep reads x and |h| only). */
int regcn_init_entities_f32(const float* dyn, const float* r_static, int64_t rows, int32_t d, float c,
                            int32_t layer_norm, float* h_out, float* x_out, float* r_out, void* stream);
/* The same map over a row list (owner partition: a rank's own rows and the halo rows its first
 * layer reads, parallel.ShardedGraph.initial_rows): row src[i] of dyn / r_static -> row dst[i]
 * of h_out, x_out, r_out (row i when dst is NULL); h_out may be NULL (halo rows need x and |h|
 * only).  Replaces the same hyperbolic_model.py:779-782 state as regcn_init_entities_f32,
 * computed only where the rank reads it. */
int regcn_init_entity_rows_f32(const float* dyn, const float* r_static, const int32_t* src, const int32_t* dst,
                               int64_t n, int32_t d, float c, int32_t layer_norm, float* h_out, float* x_out,
                               float* r_out, void* stream);

/* ---- a2/a4/a5/a6: CSR gather + segment reduce --------------------------------------- */
/* Union aggregation (HyperbolicUnionRGCNLayer msg/reduce/apply, hyperbolic_layers.py:222-240,
 * :290; DGL update_all + fn.sum): out[v] = norm[v] * sum_e w_e (x[src_e] + rel[type_e]),
 * w_e = exp(-gamma |radius[src_e] - radius[v]|).  The W_n product is applied afterwards
 * by regcn_layer_tail_f32 (linearity).  Rows absent from the chunk list are not written. */
int regcn_union_aggregate_f32(const float* x, const float* radius, const float* rel, const int32_t* col_src,
                              const int32_t* col_type, const float* norm, const int32_t* chunks, int32_t n_chunks,
                              const int32_t* fixups, int32_t n_fix, float gamma, int32_t d, float* partial,
                              int32_t partial_stride, float* out, void* stream);
/* The union (euclid = 0) or Euclidean (euclid = 1: w_e = 1, x = raw h, radius unused)
 * aggregation over the same chunks with the source half summed over source runs:
 * col_src / col_type in row/type order (regcn_snapshot_row_type_order_i32) carry the
 * relation half, col_src_by_src (regcn_snapshot_row_src_order_i32) the source half, where
 * a row's k in-edges from one source cost one gathered row, k * w_e * x[src] (w_e depends
 * on the source and the row only).  Same sums as regcn_union_aggregate_f32 within fp32
 * rounding (the DGL message sum of hyperbolic_layers.py:222-240 / rgcn/layers.py:257-279
 * regrouped by linearity). */
int regcn_union_aggregate_src_runs_f32(const float* x, const float* radius, const float* rel,
                                       const int32_t* col_src, const int32_t* col_type,
                                       const int32_t* col_src_by_src, const float* norm, const int32_t* chunks,
                                       int32_t n_chunks, const int32_t* fixups, int32_t n_fix, float gamma,
                                       int32_t euclid, int32_t d, float* partial, int32_t partial_stride,
                                       float* out, void* stream);
/* Euclidean UnionRGCNLayer aggregation (rgcn/layers.py:257-279): w_e = 1, x = raw h. */
int regcn_euclid_aggregate_f32(const float* h, const float* rel, const int32_t* col_src, const int32_t* col_type,
                               const float* norm, const int32_t* chunks, int32_t n_chunks, const int32_t* fixups,
                               int32_t n_fix, int32_t d, float* partial, int32_t partial_stride, float* out,
                               void* stream);
/* Relation-context mean (hyperbolic_model.py:802-812, src/rrgcn.py:161-166):
 * out[r] = mean of x[idx[e]] over r's span; count[r] = span length. */
int regcn_segment_mean_f32(const float* x, const int32_t* idx, const float* count, const int32_t* chunks,
                           int32_t n_chunks, const int32_t* fixups, int32_t n_fix, int32_t d, float* partial,
                           int32_t partial_stride, float* out, void* stream);
/* Lorentz aggregation (LorentzRGCNLayer msg/reduce, hyperbolic_layers.py:589-625, :665-671):
 * per edge m = blockdiag(W[type]) x_src + rel[type], L = to_lorentz(exp0(m)); per row the
 * Lorentz centroid -> to_poincare -> log0 (tangent output).  weight: [R2][nb*s*s], s = d/nb.
 * partial_stride >= d + 1. */
int regcn_lorentz_aggregate_f32(const float* x, const float* rel, const float* weight, const int32_t* col_src,
                                const int32_t* col_type, const int32_t* chunks, int32_t n_chunks,
                                const int32_t* fixups, int32_t n_fix, int32_t num_bases, float c, int32_t d,
                                float* partial, int32_t partial_stride, float* out, void* stream);

/* ---- e: multi-GPU edge partition ------------------------------------------------------
 * A rank aggregates only its slice of the edge list: the regcn_*_aggregate_f32 calls above
 * with every chunk slotted and n_fix = 0 leave raw per-chunk sums in `partial`; this call
 * sums each row's slots into out[row] (width columns: d, or d + 1 with the Lorentz time
 * coordinate at column d), unfinished, so the cross-rank all-reduce of `out` is a plain
 * sum (SURVEY.md §8(e) partitioning 1).  The all-reduced rows are then finished by the
 * same aggregate call with n_chunks = 0, partial = out and fixups {row, row, row + 1}. */
int regcn_partial_sum_f32(float* partial, int32_t partial_stride, const int32_t* fixups, int32_t n_fix,
                          int32_t width, float* out, int32_t out_stride, void* stream);

/* ---- a4/a5/a6: layer tail (MFMA GEMMs + fused epilogue) ----------------------------- */
/* Weight prepacking for the MFMA tails: a d_in x d_out row-major weight W (x @ W) becomes
 * packed[s][jq][lane][e] = W[4s + lane/16][16(4jq + e) + lane%16] (zero-padded), i.e. the
 * B-operand fragments of v_mfma_f32_16x16x4_f32 in k-step order.  d_out <= 256.
 * regcn_packed_weight_floats(d_in) floats; every w_* / b-matrix argument of
 * regcn_layer_tail_f32 and regcn_timestep_f32 is such a packed matrix. */
size_t regcn_packed_weight_floats(int32_t d_in);
int regcn_pack_weight_f32(const float* w, int32_t d_in, int32_t d_out, float* packed, void* stream);
/* Small-output products of the training path: out (M x N, row-major) = sum_k A(k, m) B(k, n)
 * (+ c0[m * c0_ld + n]; c0 nullable, c0_ld = 0 broadcasts a bias row), fp32 on MFMA, K split
 * over workgroups and the partials summed in a fixed order (deterministic).
 * a_kmajor = 1: A is K x M row-major (x of the weight gradient x^T dy); 0: A is M x K
 * row-major (coef of the CE backward's dq = coef E).  b_kmajor = 1: B is K x N row-major;
 * 0: N x K (an nn.Linear weight in x W^T).  Replaces the
 * library GEMMs torch autograd runs for the weight gradients of torch.mm(x, W)
 * (hyperbolic_layers.py:273-280 self/evolve loop, :290 neighbour weight, :315-318 skip gate;
 * hyperbolic_model.py:852-858 time gate), the decoders' nn.Linear products on a mini-batch of
 * queries (forward and both gradients; hyperbolic_decoder.py RotH/RefH/AttH projections) and
 * the dq/de GEMMs of the CE backward.
 * workspace: regcn_kreduce_workspace_floats(K, M, N) floats (0: none needed). */
size_t regcn_kreduce_workspace_floats(int64_t K, int32_t M, int32_t N);
int regcn_kreduce_gemm_f32(const float* a, int32_t a_kmajor, const float* b, int32_t b_kmajor, int64_t K, int32_t M,
                           int32_t N, const float* c0, int64_t c0_ld, float* out, float* workspace, void* stream);
/* Fused elementwise layer tail / time gate of the training path, forward and backward (V x d,
 * d % 4 == 0, contiguous, 16-B aligned; lx / ex / d_lx / d_ex rows loop_ld floats apart,
 * e.g. the two halves of one V x 2d product x [W_loop | W_evolve] with loop_ld = 2d):
 *   a = clamp(agg, +-10) [CLAMP_IN]; a += pos[v] ? lx : ex [lx != NULL];
 *   g = sigmoid(z + bias[col]), a = g a + (1 - g) p [z != NULL; bias nullable];
 *   a = clamp(a, +-10) [CLAMP_OUT]; a = a > 0 ? a : slope a [LEAKY].
 * grad_out == NULL: forward into out.  Otherwise backward: d_agg, d_lx / d_ex (the gradient
 * routed by pos), d_z (pre-sigmoid; the bias gradient is its column sum), d_p; each output
 * nullable.  Replaces the torch op chains of hyperbolic_layers.py:296-321 / :672-694 (clamp,
 * self loop where, skip gate, clamp, rrelu) and hyperbolic_model.py:841-860 (time gate). */
#define REGCN_TAIL_CLAMP_IN 1
#define REGCN_TAIL_CLAMP_OUT 2
#define REGCN_TAIL_LEAKY 4
int regcn_tail_f32(const float* agg, const float* lx, const float* ex, int64_t loop_ld, const uint8_t* pos,
                   const float* z, const float* bias, const float* p, int64_t V, int32_t d, int32_t flags, float slope,
                   const float* grad_out, float* out, float* d_agg, float* d_lx, float* d_ex, float* d_z, float* d_p,
                   void* stream);

/* Lorentz centroid -> Poincare ball of a Lorentz layer's raw message sums (regcn_lorentz_sum_raw_f32)
 * for the training path: y = (Sv / sc) / max(1 + sqrt_c S0 / sc, eps), sc = sqrt(max(c (S0^2 -
 * |Sv|^2), eps)) (hyperbolic_layers.py:613-625, :669).  grad_y == NULL: forward into y; else
 * backward into d_S0 (V) and d_Sv (V x d).  d % 4 == 0, d <= 256. */
int regcn_lorentz_centroid_f32(const float* S0, const float* Sv, int64_t V, int32_t d, float c, float sqrt_c,
                               const float* grad_y, float* y, float* d_S0, float* d_Sv, void* stream);

/* Givens rotation of interleaved pairs for the training path's RotH/RefH/AttH queries
 * (hyperbolic_decoder.py:1032-1051 givens_rotation; reflect = 1: :1392-1401 givens_reflection):
 * pair i = (x[2i], x[2i+1]) with t = angles[i] (angles row-major B x d/2 over x B x d, so
 * pairs and angles share one index) -> (cos x1 - sin x2, sin x1 + cos x2), reflected
 * (cos x1 + sin x2, sin x1 - cos x2).  grad_out == NULL: forward into out; else backward
 * into d_x and d_angles. */
int regcn_givens_rotation_f32(const float* x, const float* angles, int64_t n_pairs, int32_t reflect,
                              const float* grad_out, float* out, float* d_x, float* d_angles, void* stream);

/* rows: permutation of 0..V-1 with the n_pos in-degree>0 rows first.
 * hyperbolic (euclid=0): v = clamp(agg @ w_n | agg, +-10) + x @ (w_loop | w_evolve)
 *   [skip: g = sigmoid(prev_t @ w_skip + b_skip); v = g v + (1-g) prev_t]
 *   h = exp0(leaky(clamp(v, +-10)) [* drop_mask])     (hyperbolic_layers.py:273-323, :648-694)
 * euclid=1: h = leaky(agg @ w_n + x @ (w_loop | w_evolve)) [* drop_mask] (rgcn/layers.py:226-255)
 * agg may be NULL (no neighbour term); w_n NULL means agg is used as is (Lorentz);
 * w_loop/w_evolve NULL disable the self loop.  x_next (= log0(h), or h when euclid) and
 * r_next (= |h|) may be NULL. */
int regcn_layer_tail_f32(const float* agg, const float* w_n, const float* x, const float* w_loop,
                         const float* w_evolve, const float* prev_t, const float* w_skip, const float* b_skip,
                         const float* drop_mask, const int32_t* rows, int32_t n_pos, int32_t V, int32_t d,
                         int32_t euclid, float c, float* h_out, float* x_next, float* r_next, void* stream);

/* ---- a2-a8 fused: one whole layer per launch (gather + GEMMs + epilogue [+ timestep]) -- */
#define REGCN_AGG_UNION 0   /* HyperbolicUnionRGCNLayer, hyperbolic_layers.py:164-323 */
#define REGCN_AGG_EUCLID 2  /* UnionRGCNLayer, rgcn/layers.py:189-279 */
#define REGCN_AGG_LORENTZ 3 /* LorentzRGCNLayer, hyperbolic_layers.py:524-694 */
#define REGCN_AGG_NONE 4    /* aggregation supplied in `agg` (regcn_layer_tail_f32) */

/* Destination tiles (graph.py): `tiles` int32[n_pos_tiles][2] = {start, count} over
 * rows[0, n_pos), each count <= 16; `rowptr` int32[V+1] is the destination-sorted CSR
 * (in-degrees); the inline in-edges of tile t are items [item_ptr[t], item_ptr[t+1]),
 * in CSR order per row, rows in tile order.  Rows with in-degree > `budget` are not
 * gathered inline: their finished aggregation must already be in `agg` (chunked
 * regcn_*_aggregate_f32 over those rows only).  All w_* matrices are packed
 * (regcn_pack_weight_f32).  With fuse_step != 0 the layer output is not stored: the
 * timestep (regcn_timestep_f32 semantics; step_* fields) runs on it in registers. */
typedef struct regcn_layer_desc {
  int32_t agg_mode;
  const float* x;        /* V x d layer input: log0(h) (hyperbolic) or h (euclid) */
  const float* radius;   /* V, |h| (union message weights) */
  const float* rel;      /* R2 x d relation rows */
  const float* w_rel;    /* R2 x nb*s*s Lorentz block weights */
  int32_t num_bases;
  float gamma;           /* radius_msg_gamma */
  const int32_t* rowptr;
  const int32_t* col_src;
  const int32_t* col_type;
  const float* norm;     /* V: 1 / in-degree (0 -> 1) */
  int32_t budget;
  const int32_t* tiles;
  int32_t n_pos_tiles;
  const int32_t* item_ptr;  /* n_pos_tiles + 1: tile t gathers items [item_ptr[t], item_ptr[t+1]) */
  const int32_t* item_src;  /* per item: source entity */
  const int32_t* item_tl;   /* per item: relation type << 4 | tile-local destination row */
  const float* agg;
  const float* w_n;
  const float* w_loop;
  const float* w_evolve;
  const float* prev_t;
  const float* w_skip;
  const float* b_skip;
  const float* drop_mask;
  const int32_t* rows;
  int32_t n_pos, V, d, euclid;
  float c;
  float* h_out;
  float* x_next;
  float* r_next;
  int32_t fuse_step;
  const float* step_x_prev;   /* log0(h_prev) */
  const float* step_w_g;
  const float* step_b_g;
  const float* step_r_static;
  const float* step_w_r;
  const float* step_b_r;
  float step_eps_r, step_beta;
  int32_t step_layer_norm, step_residual;
  float step_c_radius;
  float* step_h_out;
  float* step_x_out;
  float* step_r_out;
  int64_t* trace;  /* optional: per-workgroup phase timestamps (s_memrealtime, 8 per
                      workgroup) for profiling; NULL in production */
  int32_t item_src_runs; /* union / euclid: item_src / item_tl hold each row's items in ascending
                            source order (regcn_snapshot_item_src_order_i32), so a row's k items
                            from one source gather that source row once, k * w_e * x[src]
                            (the relation rows still per item) */
  /* regcn_layer_rowtail_f32 only (NULL elsewhere); its products address the x / agg /
   * step_x_prev rows with 32-bit byte offsets: row id * d * 4 < 4 GB - 64 KB */
  const float* gate_w;   /* a cell's first layer: also the timestep's time-gate pre-activation */
  float* gate_out;       /*   clamp(x) @ gate_w (kp-packed W_g) of every row -> gate_out (V x d) */
  const float* step_tw;  /* the step layer: those rows (else the gate product runs in-kernel) */
  /* regcn_layer_rowtail_* gather, union / euclid (0 elsewhere): tiles [0, crel_tiles) take the
   * relation half sum_e w_e rel[t_e] = sum_t C[row][t] rel[t] as one [16 x R2] @ [R2 x d] MFMA
   * product per tile, reading the relation table once per tile instead of once per item
   * (hyperbolic_layers.py:222-240 by linearity) */
  int32_t crel_tiles;
  const int32_t* crel_item_src; /* those tiles' items in (row, type) order (item_type_order) */
  const int32_t* crel_item_tl;
  const float* rel_t;    /* 16 ceil(d / 16) x kpad: rel transposed, zero padded, kpad = R2 rounded up to 16 */
  int32_t n_types;       /* R2 <= 512 */
  /* regcn_layer_rowtail_* tail (NULL send_x elsewhere): the send block of the owner partition's
   * halo exchange written by the tail itself (instead of regcn_gather_rows_f32 after it): row id
   * i of the launch (send_lo <= i < send_lo + send_n) also goes to the slots
   * send_pos[send_ptr[i - send_lo] .. send_ptr[i - send_lo + 1]) -- its x row (the x_next /
   * step_x_out value) to send_x + slot * d, its |h| to send_r[slot] */
  int64_t send_lo;
  int32_t send_n;
  const int32_t* send_ptr; /* send_n + 1 */
  const int32_t* send_pos;
  float* send_x;
  float* send_r;
} regcn_layer_desc;
int regcn_layer_f32(const regcn_layer_desc* desc, void* stream);

/* The same layer for snapshots with many rows, as two launches (csrc/rowtail.hip):
 *   1. the inline in-edge rows of every tile (desc->tiles / items) gathered and finished into
 *      `agg` (V x d; on entry it holds the rows over the budget, pre-aggregated by the chunked
 *      kernels: those rows are left as they are), desc->agg ignored;
 *   2. a 64-row MFMA tail over desc->rows[0 .. desc->V): one wave per 16 rows and all columns
 *      (in-wave row reductions; the four waves of a workgroup share each weight fragment), the
 *      same epilogue / timestep as regcn_layer_f32.
 * desc->w_n / w_loop / w_evolve / step_w_g are packed by regcn_pack_weight_kp_f32 for this
 * call (a k-permuted fragment order the tail's direct global A loads need).  No skip gate, no
 * dropout mask.  Values equal regcn_layer_f32's up to the fp32 order of the products' sums.
 * A layer without the timestep may pass h_out = NULL when x_next is set (a cell's inner layer:
 * the next layer reads x_next and r_next only). */
int regcn_layer_rowtail_f32(const regcn_layer_desc* desc, float* agg, void* stream);
/* One part of regcn_layer_rowtail_f32, so a caller can pipeline row chunks on two streams
 * (the gather of chunk i + 1 beside the tail of chunk i): which = 1: the gather of tiles
 * [lo, hi); which = 2: the tail of desc->rows[lo .. hi) (their in-edge rows' agg complete:
 * gathered, or hub rows pre-aggregated); which = 3: both, everything (= the call above). */
int regcn_layer_rowtail_part_f32(const regcn_layer_desc* desc, float* agg, int32_t which, int32_t lo, int32_t hi,
                                 void* stream);
/* Packing of a d_in x d_out weight for regcn_layer_rowtail_f32:
 * packed[s][jq][lane][e] = W[16 (s / 4) + 4 (lane / 16) + s % 4][16 (4 jq + e) + lane % 16],
 * s < 4 ceil(d_in / 16), zero outside W; regcn_packed_weight_kp_floats(d_in) floats. */
size_t regcn_packed_weight_kp_floats(int32_t d_in);
int regcn_pack_weight_kp_f32(const float* w, int32_t d_in, int32_t d_out, float* packed, void* stream);

/* ---- a4-a9: history-window schedule ------------------------------------------------- */
/* A row without in-edges in any snapshot of the window ("cold") evolves through the T
 * timesteps by row-local maps of parameters only (its cells' message sums are empty), and
 * no other row reads it before the decoder (every message source has in-edges: edges are
 * doubled with inverses, rgcn/utils.py:116-118).
 * regcn_window_plan_i32: from each snapshot's rows[:n_pos] (pos_rows[t], n_pos[t] host
 *   arrays of T <= REGCN_MAX_WINDOW), in row order: c_rows (V) = cold rows, u_rows (V) = the
 *   others, z_rows[t] (T x z_stride, z_stride >= min(V, sum n_pos)) = u rows without in-edges
 *   at t; counts (device int32[2 + T]) = |C|, |U|, |Z_t|.  flags: V ints of scratch.
 * regcn_cold_chain_f32: the cold rows through T timesteps of a 2-layer cell + timestep in one
 *   launch (c_rows, device count n_rows; grid_bound >= that count, e.g. V): per timestep
 *   layer 0 (x @ w_evolve0), layer 1 (x1 @ w_evolve1, skip gate on x when w_skip1), the
 *   timestep epilogue (step_* as regcn_layer_desc) -> h_out[t], x_out[t], r_out[t] rows.
 *   Equal bit for bit to the per-layer launches on those rows. */
#define REGCN_MAX_WINDOW 16
int regcn_window_plan_i32(int32_t T, const int32_t* const* pos_rows, const int32_t* n_pos, int32_t V, int32_t* flags,
                          int32_t* c_rows, int32_t* u_rows, int32_t* z_rows, int32_t z_stride, int32_t* counts,
                          void* stream);
typedef struct regcn_chain_desc {
  const int32_t* rows;
  const int32_t* n_rows;
  int32_t T, d, grid_bound;
  float c;
  const float* x0;
  const float* w_evolve0;
  const float* w_evolve1;
  const float* w_skip1;
  const float* b_skip1;
  const float* step_w_g;
  const float* step_b_g;
  const float* step_r_static;
  const float* step_w_r;
  const float* step_b_r;
  float step_eps_r, step_beta;
  int32_t step_layer_norm, step_residual;
  float step_c_radius;
  float* h_out[REGCN_MAX_WINDOW];
  float* x_out[REGCN_MAX_WINDOW];
  float* r_out[REGCN_MAX_WINDOW];
} regcn_chain_desc;
int regcn_cold_chain_f32(const regcn_chain_desc* desc, void* stream);
/* regcn_zero_step_f32: the rows of ONE snapshot without in-edges (e.g. rows + n_pos of its
 *   row list) through one timestep (T == 1): layer 0, layer 1, the timestep epilogue with
 *   x0 as the timestep input, one workgroup per 16 rows; rows[0 .. grid_bound) (host count;
 *   n_rows unused).  The phase launches of that timestep then set skip_zero_rows; it runs on
 *   any stream ordered after the previous timestep and before the next one's phase A.
 *   Equal bit for bit to the phases' rows-without-in-edges paths. */
int regcn_zero_step_f32(const regcn_chain_desc* desc, void* stream);

/* ---- a2-a9: one timestep of a 2-layer cell in three launches on one stream ---------- */
/* hyperbolic_model.py:797-869 with HyperbolicRGCNCell / LorentzRGCNCell of 2 layers.  The
 * per-layer launches (regcn_layer_f32) put each tile's whole layer behind its gather; here
 * work that needs no gather moves to an earlier launch and the rows without in-edges (whose
 * layers are row-local maps) ride beside the in-edge tiles:
 *   phase 0 (A): relation GRU x-half -> gru_h_out (needs gru_pre of this timestep);
 *                in-edge rows: s1 = x0 @ w_loop[0], tw = clamp(x0) @ W_g
 *   phase 1 (B): in-edge tiles: layer-0 gather with rel = h_0 -> x1, r1;
 *                other rows: layers 0 and 1 -> h2, n2;  GRU pre-half of the next timestep
 *                (gru_h_prev = h_0 of this timestep -> gru_pre) unless gru_pre is NULL
 *   phase 2 (C): in-edge tiles: layer-1 gather (x1, r1) + self loop + skip + timestep
 *                epilogue; other rows: timestep epilogue on h2 -> step_h/x/r_out.
 * Field meanings follow regcn_layer_desc (snapshot lists, packed weights, step_*); [0] / [1]
 * are layer 0 / layer 1.  s1, tw, x1, h2 are V x d and r1, n2 V floats of caller scratch.
 * Rows with in-degree > budget read agg[l] (chunked pre-aggregation of layer l, run
 * between the phases).  Each row's values equal regcn_layer_f32 (layer 0) then
 * regcn_layer_f32 with fuse_step (layer 1) bit for bit. */
typedef struct regcn_phase_desc {
  int32_t agg_mode, num_bases;
  float gamma, c;
  const int32_t* rowptr;
  const int32_t* col_src;
  const int32_t* col_type;
  const float* norm;
  int32_t budget;
  const int32_t* tiles;
  int32_t n_pos_tiles;
  const int32_t* item_ptr;
  const int32_t* item_src;
  const int32_t* item_tl;
  const int32_t* rows;
  int32_t n_pos, V, d;
  const float* rel;        /* h_0 of this timestep (both layers' messages) */
  const float* w_rel[2];
  const float* agg[2];
  const float* w_n[2];
  const float* w_loop[2];
  const float* w_evolve[2];
  const float* w_skip1;    /* layer-1 skip gate on the cell input (LorentzRGCNCell), or NULL */
  const float* b_skip1;
  const float* x0;         /* log0(h_prev) */
  const float* r0;         /* |h_prev| */
  float* s1;
  float* tw;
  float* x1;
  float* r1;
  float* h2;
  float* n2;
  const float* step_w_g;
  const float* step_b_g;
  const float* step_r_static;
  const float* step_w_r;
  const float* step_b_r;
  float step_eps_r, step_beta;
  int32_t step_layer_norm, step_residual;
  float step_c_radius;
  float* step_h_out;
  float* step_x_out;
  float* step_r_out;
  const int32_t* gru_rel_idx;
  const int32_t* gru_rel_start;
  const float* gru_rel_count;
  const float* gru_x_mean;
  const float* gru_emb_rel;
  const float* gru_h_prev;
  const float* gru_w_ih_e;
  const float* gru_w_ih_x;
  const float* gru_w_hh;
  const float* gru_b_ih;
  const float* gru_b_hh;
  int32_t gru_R2;
  float* gru_pre;
  float* gru_h_out;
  /* Memo mode (memo_h != NULL).  A row without an in-edge at any timestep so far evolves by
   * an input-independent map of the parameters (W_evolve, skip gate, time gate, static
   * radius): its state after this timestep is memo_* (F^{t+1} of the initial state, computed
   * once per parameter version by regcn_cold_chain_f32 over all rows), which phase A copies
   * to step_*_out.  The rows without in-edges that run are those with an in-edge at an earlier
   * timestep and none since, taken from the earlier snapshots' rows[:n_pos] lists.  NULL:
   * every row without in-edges (rows[n_pos:V]) runs. */
  const float* memo_h;
  const float* memo_x;
  const float* memo_r;
  int32_t n_prev;                                /* earlier snapshots of the window (t) */
  const int32_t* prev_rows[REGCN_MAX_WINDOW];    /* their rows (in-edge rows first) */
  const int32_t* prev_rowptr[REGCN_MAX_WINDOW];  /* their rowptr */
  int32_t prev_n_pos[REGCN_MAX_WINDOW];
  /* Plain mode only: 1 = the launches skip the rows without in-edges (the caller runs them
   * through regcn_zero_step_f32 beside the phases); 0 = the phases run them. */
  int32_t skip_zero_rows;
} regcn_phase_desc;
int regcn_timestep_phase_f32(const regcn_phase_desc* desc, int32_t phase, void* stream);

/* ---- a7: relation evolution (segment mean + GRUCell in one launch) ------------------- */
/* nn.Linear-layout packing for the relation GRU: W is (n_gates * n_out) x n_in row-major
 * (GRUCell weight_ih: 3d x 2d, weight_hh: 3d x d); packed[g][b][jt][lane][e] =
 * W[g*n_out + 16 jt + lane%16][16 b + 4 (lane/16) + e], zero padded (16-deep k-blocks:
 * one float4 per lane, gate and block). */
size_t regcn_packed_linear_floats(int32_t n_gates, int32_t n_out, int32_t n_in);
int regcn_pack_linear_f32(const float* w, int32_t n_gates, int32_t n_out, int32_t n_in, float* packed,
                          void* stream);
/* hyperbolic_model.py:797-818 (rrgcn.py:161-174): x_mean[r] = mean of x[rel_idx[rel_start[r] ..
 * + rel_count[r]]] (0 for absent relations; or x_mean given precomputed, rel_* unused), then
 * h_out = GRUCell([emb_rel | x_mean], h_prev) with packed w_ih / w_hh and biases b_ih / b_hh
 * (3d each, gate order r, z, n). */
int regcn_relation_gru_f32(const float* x, const int32_t* rel_idx, const int32_t* rel_start, const float* rel_count,
                           const float* x_mean, const float* emb_rel, const float* h_prev, const float* w_ih,
                           const float* w_hh, const float* b_ih, const float* b_hh, int32_t R2, int32_t d,
                           float* h_out, void* stream);

/* The same GRU in two launches, split by what each input depends on.  w_ih_e / w_ih_x are
 * the emb_rel and x_mean column halves of GRUCell.weight_ih (each 3d x d, packed with
 * regcn_pack_linear_f32(n_gates = 3, n_out = d, n_in = d)).
 * regcn_relation_gru_pre_f32: pre[r] = {W_ir^e e + b_ir + W_hr h + b_hr, (z likewise),
 *   W_in^e e + b_in, W_hn h + b_hn} (R2 x 4 x d) from emb_rel and h_prev only, so it can
 *   run while the previous timestep's entity rows are still being computed.
 * regcn_relation_gru_x_f32: x_mean as in regcn_relation_gru_f32, then r = s(pre0 + W_ir^x m),
 *   z = s(pre1 + W_iz^x m), n = tanh(pre2 + W_in^x m + r pre3), h_out = (1 - z) n + z h_prev. */
int regcn_relation_gru_pre_f32(const float* emb_rel, const float* h_prev, const float* w_ih_e, const float* w_hh,
                               const float* b_ih, const float* b_hh, int32_t R2, int32_t d, float* pre,
                               void* stream);
int regcn_relation_gru_x_f32(const float* x, const int32_t* rel_idx, const int32_t* rel_start,
                             const float* rel_count, const float* x_mean, const float* h_prev, const float* w_ih_x,
                             const float* pre, int32_t R2, int32_t d, float* h_out, void* stream);

/* ---- a8: per-timestep entity evolution (MFMA time gate + fused row epilogue) --------- */
/* hyperbolic_model.py:829-869 + TemporalRadiusEvolution.forward (hyperbolic_ops.py:395-435):
 * hc = cell output, x_prev = log0(h_prev), r_static = clamped static radius (:715-720),
 * w_r/b_r = radius MLP (device pointers; b_r one float).  residual=0 uses apply_radius(h, r_static).
 * c_radius = TemporalRadiusEvolution's constructor curvature. */
int regcn_timestep_f32(const float* hc, const float* x_prev, const float* w_g, const float* b_g,
                       const float* r_static, const float* w_r, const float* b_r, float eps_r, float beta,
                       int32_t layer_norm, int32_t residual, int32_t V, int32_t d, float c, float c_radius,
                       float* h_out, float* x_out, float* r_out, void* stream);
/* The same timestep for --run-analysis (hyperbolic_main.py:716): also writes the time gate
 * sigmoid(clamp(x_prev) @ W_g + b_g) of every element into gate_out (V x d: the reference's
 * gate_list entry, hyperbolic_model.py:848-856) and, when residual != 0, the radius evolution's
 * per-row terms into stat_out (3 x V, nullable): the clipped delta, the dynamic radius |h| and
 * the base radius beta r_static + (1 - beta) |h| (TemporalRadiusEvolution's evolution stats,
 * hyperbolic_ops.py:407-434).  h_out / x_out / r_out equal regcn_timestep_f32's bit for bit. */
int regcn_timestep_analysis_f32(const float* hc, const float* x_prev, const float* w_g, const float* b_g,
                                const float* r_static, const float* w_r, const float* b_r, float eps_r, float beta,
                                int32_t layer_norm, int32_t residual, int32_t V, int32_t d, float c, float c_radius,
                                float* h_out, float* x_out, float* r_out, float* gate_out, float* stat_out,
                                void* stream);

/* ---- a9/a10: decoder queries (one launch each) -------------------------------------- */
/* Queries b < n_test use trip[b] = (s, r, o) (int64, n_test x 3); b >= n_test the inverse
 * (o, r + num_rels, s) of trip[b - n_test] (hyperbolic_model.py:915-919).  B <= 2 n_test.
 * All w_* are nn.Linear weights packed transposed: regcn_pack_weight_f32 of W^T (in x out).
 * RotH (HyperbolicRotH._query, hyperbolic_decoder.py:1065-1085): w1/b1, w2/b2 reshape_fc1/2,
 * w_rot/b_rot rot_proj (d -> d/2), w_trans/b_trans trans_proj; rel = relation embedding. */
int regcn_roth_query_f32(const float* ent, const float* rel, const int64_t* trip, int32_t n_test, int32_t B,
                         int32_t num_rels, const float* w1, const float* b1, const float* w2, const float* b2,
                         const float* w_rot, const float* b_rot, const float* w_trans, const float* b_trans, int32_t d,
                         float c, float* q_out, void* stream);
/* RotHRel (HyperbolicRotHRel._query + candidates, hyperbolic_decoder.py:1223-1243):
 * q = mobius_add(-exp0(givens(s_tan, global_rot)), E[o]); also cand_out = exp0(rel) for the
 * n_cand relation rows (the relation scorer's candidates). */
int regcn_roth_rel_query_f32(const float* ent, const int64_t* trip, int32_t n_test, int32_t B, int32_t num_rels,
                             const float* w1, const float* b1, const float* w2, const float* b2,
                             const float* global_rot, const float* rel, int32_t n_cand, int32_t d, float c,
                             float* q_out, float* cand_out, void* stream);

/* The decoder front of a RotH predict in ONE launch (replaces the two calls above and the
 * inverse-triple torch.cat of HyperbolicRecurrentRGCN.predict, hyperbolic_model.py:915-919):
 * RotH entity queries -> q_ent, RotHRel relation queries -> q_rel, exp0(rel) rows -> cand,
 * and all_triples = [trip; (o, r + num_rels, s)] (B x 3 int64).  4-query tiles on the
 * 4x4x1 fp32 MFMA.  Weights: nn.Linear (out x in) packed by regcn_pack_k4_f32.  A NULL
 * q_ent / q_rel / cand (n_cand = 0) / all_triples skips that part (all_triples needs q_ent). */
typedef struct regcn_roth_queries_desc {
  const float* ent;        /* V x d final entity embedding */
  const float* rel;        /* R2 x d relation embedding */
  const int64_t* trip;     /* n_test x 3 test triples (s, r, o) */
  int32_t n_test, B, num_rels, d;
  float c;
  /* HyperbolicRotH (hyperbolic_decoder.py:1065-1085) */
  const float *w1, *b1, *w2, *b2;           /* reshape_fc1 / reshape_fc2 */
  const float *w_rot, *b_rot;               /* rot_proj (d -> d/2) */
  const float *w_trans, *b_trans;           /* trans_proj */
  float* q_ent;                             /* B x d */
  /* HyperbolicRotHRel (hyperbolic_decoder.py:1223-1243) */
  const float *rw1, *rb1, *rw2, *rb2;       /* its reshape_fc1 / reshape_fc2 */
  const float* global_rot;                  /* d/2 */
  float* q_rel;                             /* B x d */
  int32_t n_cand;                           /* relation rows of exp0(rel) */
  float* cand;                              /* n_cand x d */
  int64_t* all_triples;                     /* B x 3, or NULL */
} regcn_roth_queries_desc;
/* k4 packing of an nn.Linear weight W (n_out x n_in, n_out <= 256, n_in % 4 == 0):
 * out[g][c][e] = W[c][4g + e], zero for n_out <= c < 256. */
size_t regcn_packed_k4_floats(int32_t n_out, int32_t n_in);
int regcn_pack_k4_f32(const float* W, int32_t n_out, int32_t n_in, float* out, void* stream);
int regcn_roth_queries_f32(const regcn_roth_queries_desc* desc, void* stream);

/* ---- a11/a12/f2: all-entity hyperbolic scoring ------------------------------------- */
#define REGCN_SCORE_DIST 1       /* flags: true hyperbolic distance (fp64 MFMA) */
#define REGCN_SCORE_RAW_SCALE 2  /* flags: `scale` is score_scale_raw; softplus(raw) + 1e-6 in-kernel */
/* _chunked_hyperbolic_dist_score, hyperbolic_decoder.py:89-179.  scale/margin: device
 * scalars or NULL (1, 0).  bias [N] or NULL.  flags: REGCN_SCORE_DIST selects the true
 * hyperbolic distance (computed with fp64 MFMA: the arctanh distance is linear in
 * |(-q)(+)e| and an fp32 expansion would lose ~3 digits on near-duplicate pairs);
 * REGCN_SCORE_RAW_SCALE applies softplus + 1e-6 to *scale on the device (:717).  c_rel [B]
 * (or NULL) the per-query curvature of --plus-relation-specific-curvature.  out: [B][N]. */
int regcn_hyp_score_f32(const float* q, const float* cand, const float* bias, const float* c_rel, const float* scale, const float* margin, int32_t B,
                        int32_t N, int32_t d, float c, int32_t flags, float* out, void* stream);
/* Up to two independent regcn_hyp_score_f32 jobs (no REGCN_SCORE_DIST, no c_rel, one d) in
 * ONE launch: a predict's entity scores and relation scores.  Job 1's workgroups follow job
 * 0's and take the CUs job 0's shorter candidate strips free. */
typedef struct regcn_score_job {
  const float* q;
  const float* cand;
  const float* bias;     /* [N] or NULL */
  const float* scale;    /* device scalar or NULL */
  const float* margin;   /* device scalar or NULL */
  int32_t B, N, d;
  float c;
  int32_t flags;         /* REGCN_SCORE_RAW_SCALE only */
  float* out;            /* B x N */
} regcn_score_job;
int regcn_hyp_score_jobs_f32(const regcn_score_job* jobs, int32_t n_jobs, void* stream);
/* _chunked_hyperbolic_ce_loss, hyperbolic_decoder.py:182-307: per-query lse - target logit
 * (the caller takes the mean).  workspace: regcn_hyp_ce_workspace_bytes(B, N) bytes. */
size_t regcn_hyp_ce_workspace_bytes(int32_t B, int32_t N);
int regcn_hyp_ce_f32(const float* q, const float* cand, const float* bias, const float* c_rel, const float* scale, const float* margin,
                     const int32_t* target, int32_t B, int32_t N, int32_t d, float c, int32_t flags,
                     void* workspace, float* loss_per_query, void* stream);
/* get_total_rank / sort_and_rank / filter_score, rgcn/utils.py:21-166: 1 + count of
 * candidates scoring strictly above the target, raw and excluding the CSR list of other
 * true answers (filt_ptr [B+1], filt_idx; NULL filt_ptr skips the filtered rank). */
int regcn_rank_f32(const float* score, int32_t B, int32_t N, const int32_t* target, const int32_t* filt_ptr,
                   const int32_t* filt_idx, int32_t* rank_raw, int32_t* rank_filt, void* stream);
/* e: candidate-sharded ranking (SURVEY.md §8(e) decoder).  On a rank's slice of the
 * candidates: #{n : score[b,n] > threshold[b]} (raw) and the same excluding the slice-local
 * CSR list of other true answers; summing the counts over the ranks and adding 1 gives
 * regcn_rank_f32's ranks, threshold = the target's score. */
int regcn_rank_count_f32(const float* score, int32_t B, int32_t N, const float* threshold, const int32_t* filt_ptr,
                         const int32_t* filt_idx, int32_t* count_raw, int32_t* count_filt, void* stream);
/* e / f2: the fused form of regcn_hyp_score_f32 + regcn_rank_count_f32 for the proxy score
 * (flags: REGCN_SCORE_RAW_SCALE only; d % 4 == 0, d <= 256): counts[b] = #{n : S[b,n] >
 * threshold[b]} over the candidate rows, S bit for bit what regcn_hyp_score_f32 writes, with
 * no B x N score matrix (rgcn/utils.py:21-50 sort_and_rank's position = this count + 1 when
 * the target has no tie).  The candidates are rows [0, N) of cand, or with n_ranges > 0 the
 * union of the row ranges {ranges[2r], ranges[2r+1]} (a HOST array, <= 8 ranges inside [0, N):
 * a rank's owner ranges in one launch; bias indexed by row).  accumulate != 0 adds to counts.
 * workspace: regcn_hyp_ce_workspace_bytes(B, N) bytes. */
int regcn_hyp_rank_fused_f32(const float* q, const float* cand, const float* bias, const float* scale,
                             const float* margin, const float* threshold, int32_t B, int32_t N, int32_t d, float c,
                             int32_t flags, const int32_t* ranges, int32_t n_ranges, void* workspace,
                             int32_t accumulate, int32_t* counts, void* stream);
/* e: the owner partition's exchange (the reference runs on one GPU, so no
 * reference call site): rows ids[i] of x (n_rows x d) and radius packed as records of stride
 * d + 4 floats (x row, radius, 3 pad) for one all_to_all, and the received records written back
 * to rows ids[i].  d % 4 == 0, d <= 252, x and the record buffer 16-B aligned. */
int regcn_pack_rows_f32(const float* x, const float* radius, const int64_t* ids, int64_t n, int32_t d, float* out,
                        void* stream);
int regcn_unpack_rows_f32(const float* in, const int64_t* ids, int64_t n, int32_t d, float* x, float* radius,
                          void* stream);
/* e: the send side of the halo exchange: rows ids[i] of x and radius gathered into x_out
 * (n x d, contiguous) and r_out (n), which two all_to_alls deliver straight into the
 * receiving ranks' halo rows (the rows after the Vp owned ids, which that rank's consumer
 * work lists name instead of the remote ids: no scatter).  d % 4 == 0, d <= 252, x and x_out
 * 16-B aligned. */
int regcn_gather_rows_f32(const float* x, const float* radius, const int64_t* ids, int64_t n, int32_t d,
                          float* x_out, float* r_out, void* stream);

/* ---- a1 / f3: snapshot construction on the device ------------------------------------
 * build_sub_graph + r2e (rgcn/utils.py:78-134) and the kernel work lists of
 * re-gcn_amd/regcn_amd/graph.py, built from the snapshot's triples in HBM.  Every output
 * is bit-identical to the host build: the destination sort is a stable LSD radix sort (edge
 * ids keep their order within a destination, as the reference's edge order), r_to_e spans
 * hold each relation's entities ascending (np.unique), rows are ordered by descending
 * in-degree (stable), tiles follow the host's greedy packing.
 *
 * Two calls on one stream with a host read of `stats` in between (the work-list call needs
 * the tile budget, which the host derives from the maximum in-degree):
 *   1. regcn_snapshot_csr_i32   triples -> in_deg, rowptr, col_src/col_type, norm, edge
 *      type/norm (reference edge order), r2e lists; stats[MAX_DEG, N_POS, INVALID, N_PAIRS,
 *      REL_MAX].
 *   2. regcn_snapshot_work_i32  -> rows, tiles + items, heavy / all-row / relation chunk
 *      and fix-up lists (capacity-sized buffers, counts in stats).
 * Capacities: regcn_snapshot_capacity(what, ...) elements (int32, x4 for chunk and
 * fix-up records, x2 for tiles); workspace: regcn_snapshot_workspace_bytes(T, V, R). */
#define REGCN_SNAP_MAX_DEG 0
#define REGCN_SNAP_N_POS 1
#define REGCN_SNAP_INVALID 2    /* triples with an id out of range (the build is then void) */
#define REGCN_SNAP_N_PAIRS 3    /* sum over relations of |r_to_e[r]| (forward spans) */
#define REGCN_SNAP_REL_MAX 4    /* longest r_to_e span */
#define REGCN_SNAP_N_HEAVY 5
#define REGCN_SNAP_N_TILES 6
#define REGCN_SNAP_N_ITEMS 7
#define REGCN_SNAP_WALK_TILES 8 /* tiles placed by the sequential greedy prefix */
#define REGCN_SNAP_A_STAR 9     /* first row from which 16-row tiles always fit */
#define REGCN_SNAP_CHUNKS 10    /* all-row chunk list: n_chunks, n_fix, n_slots */
#define REGCN_SNAP_HEAVY_CHUNKS 13
#define REGCN_SNAP_REL_CHUNKS 16
#define REGCN_SNAP_NSTATS 20

#define REGCN_CAP_TILES 0        /* int32[cap][2] */
#define REGCN_CAP_ITEMS 1
#define REGCN_CAP_CHUNKS 2       /* int32[cap][4] */
#define REGCN_CAP_FIXUPS 3
#define REGCN_CAP_HEAVY_CHUNKS 4
#define REGCN_CAP_HEAVY_FIXUPS 5
#define REGCN_CAP_REL_CHUNKS 6
#define REGCN_CAP_REL_FIXUPS 7
#define REGCN_CAP_REL_IDX 8

typedef struct regcn_snapshot_desc {
  const int64_t* triples;  /* T x 3 (s, r, o), device */
  int64_t T;
  int32_t V, R;            /* entities, base relations (edge types 0 .. 2R-1) */
  int32_t budget;          /* graph.py tile_budget_for(); used by call 2 */
  int32_t pack_items;      /* graph.py pack_items */
  int32_t chunk_edges;     /* graph.py chunk_size_for() */
  void* workspace;
  size_t ws_bytes;
  int32_t* stats;          /* REGCN_SNAP_NSTATS */
  /* call 1 outputs */
  int32_t* in_deg;         /* V */
  int32_t* rowptr;         /* V + 1 */
  int32_t* col_src;        /* E = 2T, destination-sorted */
  int32_t* col_type;       /* E */
  float* norm;             /* V: 1 / in_deg, 0 -> 1 (utils.py:110-114) */
  int64_t* edge_type;      /* E, reference edge order: cat(r, r + R) (utils.py:118, :125) */
  float* edge_norm;        /* E, reference edge order: norm[dst] * norm[src] (utils.py:124) */
  int32_t* rel_ent_count;  /* R: |r_to_e[r]| */
  int32_t* rel_idx;        /* REGCN_CAP_REL_IDX: r_to_e flattened in uniq_r order */
  int32_t* rel_start;      /* 2R */
  float* rel_count;        /* 2R */
  /* call 2 outputs */
  int32_t* rows;           /* V */
  int32_t* tiles;
  int32_t* item_ptr;       /* V + 1 */
  int32_t* item_src;
  int32_t* item_tl;
  int32_t* chunks;
  int32_t* fixups;
  int32_t* heavy_chunks;
  int32_t* heavy_fixups;
  int32_t* rel_chunks;
  int32_t* rel_fixups;
} regcn_snapshot_desc;
/* Transposed edge lists for the backward passes: csr_dst[p] = destination of CSR position p;
 * positions sorted (stably) by source (sptr [V+1], sp [E]) and by type (tptr [R2+1], tp [E]). */
typedef struct regcn_transpose_desc {
  int32_t V, E, R2;
  const int32_t* rowptr;
  const int32_t* col_src;
  const int32_t* col_type;
  void* workspace;         /* regcn_transpose_workspace_bytes(E, V, R2) */
  size_t ws_bytes;
  int32_t* csr_dst;
  int32_t* sptr;
  int32_t* sp;
  int32_t* tptr;
  int32_t* tp;
} regcn_transpose_desc;
size_t regcn_transpose_workspace_bytes(int32_t E, int32_t V, int32_t R2);
int regcn_snapshot_transpose_i32(const regcn_transpose_desc* desc, void* stream);
/* The CSR edges with each destination row's edges in relation-type order (stable: ties keep
 * CSR order): out_src / out_type [E].  Same rows and row pointer as the CSR, so every chunk
 * list applies unchanged.  Fed to regcn_lorentz_aggregate_f32, a row's run of same-type
 * edges reuses the type's relation row and W block fragment from L1 (SURVEY.md §8(d)
 * config 5).  The message pass it serves (hyperbolic_layers.py:589-611) sums a row's
 * Lorentz points in edge-id order; this order equals it within fp32 rounding. */
size_t regcn_row_type_order_workspace_bytes(int32_t E, int32_t V, int32_t R2);
int regcn_snapshot_row_type_order_i32(int32_t V, int32_t E, int32_t R2, const int32_t* rowptr,
                                      const int32_t* col_src, const int32_t* col_type, int32_t* out_src,
                                      int32_t* out_type, void* workspace, size_t ws_bytes, void* stream);
/* The CSR edges' sources with each destination row's edges in ascending source order
 * (out_src [E]; same rows and row pointer as the CSR): a row's duplicate sources are
 * adjacent for regcn_union_aggregate_src_runs_f32. */
size_t regcn_row_src_order_workspace_bytes(int32_t E, int32_t V);
int regcn_snapshot_row_src_order_i32(int32_t V, int32_t E, const int32_t* rowptr, const int32_t* col_src,
                                     int32_t* out_src, void* workspace, size_t ws_bytes, void* stream);
/* The fused layer's inline items (tiles, item_ptr, item_src, item_tl of the snapshot's work
 * lists) with each row's items in ascending source order (stable): out_src / out_tl
 * [n_items], same tiles and item_ptr.  For regcn_layer_desc.item_src_runs. */
size_t regcn_item_src_order_workspace_bytes(int32_t n_items, int32_t V);
int regcn_snapshot_item_src_order_i32(int32_t V, int32_t n_tiles, int32_t n_items, const int32_t* tiles,
                                      const int32_t* item_ptr, const int32_t* item_src, const int32_t* item_tl,
                                      int32_t* out_src, int32_t* out_tl, void* workspace, size_t ws_bytes,
                                      void* stream);
/* The same items with each row's items in ascending relation-type order (stable; workspace:
 * regcn_item_src_order_workspace_bytes(n_items, V)).  For regcn_layer_desc.item_crel: a row's
 * same-type items are adjacent, so the gather sums their weights per (row, type) and applies the
 * relation rows as one [16 x R2] @ [R2 x d] product per tile (hyperbolic_layers.py:222-240 by
 * linearity: sum_e w_e rel[t_e] = sum_t (sum_{e: t_e = t} w_e) rel[t]). */
int regcn_snapshot_item_type_order_i32(int32_t V, int32_t R2, int32_t n_tiles, int32_t n_items, const int32_t* tiles,
                                       const int32_t* item_ptr, const int32_t* item_src, const int32_t* item_tl,
                                       int32_t* out_src, int32_t* out_tl, void* workspace, size_t ws_bytes,
                                       void* stream);
size_t regcn_snapshot_workspace_bytes(int64_t T, int32_t V, int32_t R);
int64_t regcn_snapshot_capacity(int32_t what, int64_t T, int32_t V, int32_t R, int32_t chunk_edges);
int regcn_snapshot_csr_i32(const regcn_snapshot_desc* desc, void* stream);
int regcn_snapshot_work_i32(const regcn_snapshot_desc* desc, void* stream);

/* ---- f1: backward kernels of the training path -----------------------------------------
 * Gradients as torch autograd computes them through the reference op sequence, clamp
 * subgradients included (see csrc/backward.hip). */
#define REGCN_BWD_LOG0 0         /* HyperbolicOps.log_map_zero */
#define REGCN_BWD_EXP0 1         /* HyperbolicOps.exp_map_zero */
#define REGCN_BWD_PROJECT 2      /* HyperbolicOps.project_to_ball */
#define REGCN_BWD_APPLY_RADIUS 3 /* y: radius [rows]; dy: d radius [rows] */
#define REGCN_BWD_RADIUS 4       /* g: [rows] (get_radius output gradient) */
#define REGCN_BWD_MOBIUS 5       /* y: second operand; dy: its gradient */
int regcn_rowmap_bwd_f32(int32_t op, const float* x, const float* y, const float* g, int64_t rows, int32_t d,
                         float c, float* dx, float* dy, void* stream);

typedef struct regcn_edge_bwd_desc {
  int32_t V, E, R2, d;
  const float* x;          /* V x d layer input (tangent) */
  const float* radius;     /* V (union) */
  const float* rel;        /* R2 x d */
  const float* W;          /* R2 x nb*s*s (Lorentz) */
  const float* norm;       /* V (union) */
  const int32_t* rowptr;
  const int32_t* col_src;
  const int32_t* col_type;
  const int32_t* csr_dst;  /* regcn_snapshot_transpose_i32 */
  const int32_t* sptr;
  const int32_t* sp;
  const int32_t* tptr;
  const int32_t* tp;
  const float* G;          /* V x d: gradient of the aggregation (union) / of the raw sums' space part (Lorentz) */
  const float* G0;         /* V: gradient of the raw sums' time coordinate (Lorentz) */
  float* dx;               /* V x d */
  float* drel;             /* R2 x d */
  float* dradius;          /* V (union) */
  float* dW;               /* R2 x nb*s*s (Lorentz) */
  float* edge_scratch;     /* union: 2E + V floats */
} regcn_edge_bwd_desc;
/* HyperbolicUnionRGCNLayer message/sum/apply (hyperbolic_layers.py:222-240, :290) backward:
 * dx, drel and dradius of agg[v] = norm[v] sum_e w_e (x[src] + rel[type]). */
int regcn_union_aggregate_bwd_f32(const regcn_edge_bwd_desc* desc, float gamma, void* stream);
/* LorentzRGCNLayer messages (hyperbolic_layers.py:589-611) summed per destination, before the
 * centroid: S0[v] = sum_e L0_e, Sv[v] = sum_e L_e[1:] (training forward; the centroid, to_poincare
 * and log0 run as separate differentiable ops). */
int regcn_lorentz_sum_raw_f32(const float* x, const float* rel, const float* weight, const int32_t* rowptr,
                              const int32_t* col_src, const int32_t* col_type, int32_t V, int32_t d, int32_t num_bases,
                              float c, float* S0, float* Sv, void* stream);
/* ... and its backward: dx, drel, dW from (G0, G) = gradient of (S0, Sv). */
int regcn_lorentz_aggregate_bwd_f32(const regcn_edge_bwd_desc* desc, int32_t num_bases, float c, void* stream);
/* Cross-entropy scorer (regcn_hyp_ce_f32) with the per-query log-sum-exp as an extra output. */
int regcn_hyp_ce_lse_f32(const float* q, const float* cand, const float* bias, const float* scale,
                         const float* margin, const int32_t* target, int32_t B, int32_t N, int32_t d, float c,
                         int32_t flags, void* workspace, float* loss_per_query, float* lse, void* stream);
/* _chunked_hyperbolic_ce_loss backward (proxy score): with G = gl (softmax - onehot),
 * coef[b,n] = G dS/d<q_b,e_n>, rsum[b][nblk] (nblk = ceil(N/64)) partial sums over candidates of
 * G dS/d|q_b|^2, csum[ng][N][3] (ng = 8 ceil(B/128)) partial sums over 16-query groups of
 * (G dS/d|e_n|^2, G, G (margin - n^2)).  Then dq = coef E + 2 q sum(rsum), de = coef^T Q +
 * 2 e csum[.,0], dbias = csum[.,1], dscale = sum csum[.,2], dmargin = scale sum csum[.,1]. */
int regcn_hyp_ce_bwd_f32(const float* q, const float* cand, const float* bias, const float* scale,
                         const float* margin, const int32_t* target, const float* lse, const float* grad_loss,
                         int32_t B, int32_t N, int32_t d, float c, int32_t flags, float* coef, float* rsum,
                         float* csum, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* REGCN_HIP_H */
