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

#define REGCN_ABI_VERSION 1
#define REGCN_EINVAL (-1)
#define REGCN_ENOTSUP (-2)

/* Snapshot work lists built by the host (re-gcn_amd/regcn_amd/graph.py):
 * chunks: int32[n_chunks][4] = {row, edge_begin, edge_end, slot}; slot < 0 means
 *         the row is finished by that chunk, slot >= 0 names its partial row.
 * fixups: int32[n_fix][4]    = {row, slot_begin, slot_end, 0}. */

int regcn_version(void);
const char* regcn_last_error_string(void);

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
 * also emits x = log0(h) and r = |h| for the first timestep (x_out/r_out may be NULL). */
int regcn_init_entities_f32(const float* dyn, const float* r_static, int64_t rows, int32_t d, float c,
                            int32_t layer_norm, float* h_out, float* x_out, float* r_out, void* stream);

/* ---- a2/a4/a5/a6: CSR gather + segment reduce --------------------------------------- */
/* Union aggregation (HyperbolicUnionRGCNLayer msg/reduce/apply, hyperbolic_layers.py:222-240,
 * :290; DGL update_all + fn.sum): out[v] = norm[v] * sum_e w_e (x[src_e] + rel[type_e]),
 * w_e = exp(-gamma |radius[src_e] - radius[v]|).  The W_n product is applied afterwards
 * by regcn_layer_tail_f32 (linearity).  Rows absent from the chunk list are not written. */
int regcn_union_aggregate_f32(const float* x, const float* radius, const float* rel, const int32_t* col_src,
                              const int32_t* col_type, const float* norm, const int32_t* chunks, int32_t n_chunks,
                              const int32_t* fixups, int32_t n_fix, float gamma, int32_t d, float* partial,
                              int32_t partial_stride, float* out, void* stream);
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

/* ---- a4/a5/a6: layer tail (MFMA GEMMs + fused epilogue) ----------------------------- */
/* Weight prepacking for the MFMA tails: a d_in x d_out row-major weight W (x @ W) becomes
 * packed[s][jq][lane][e] = W[4s + lane/16][16(4jq + e) + lane%16] (zero-padded), i.e. the
 * B-operand fragments of v_mfma_f32_16x16x4_f32 in k-step order.  d_out <= 256.
 * regcn_packed_weight_floats(d_in) floats; every w_* / b-matrix argument of
 * regcn_layer_tail_f32 and regcn_timestep_f32 is such a packed matrix. */
size_t regcn_packed_weight_floats(int32_t d_in);
int regcn_pack_weight_f32(const float* w, int32_t d_in, int32_t d_out, float* packed, void* stream);
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

/* ---- a8: per-timestep entity evolution (MFMA time gate + fused row epilogue) --------- */
/* hyperbolic_model.py:829-869 + TemporalRadiusEvolution.forward (hyperbolic_ops.py:395-435):
 * hc = cell output, x_prev = log0(h_prev), r_static = clamped static radius (:715-720),
 * w_r/b_r = radius MLP (device pointers; b_r one float).  residual=0 uses apply_radius(h, r_static).
 * c_radius = TemporalRadiusEvolution's constructor curvature. */
int regcn_timestep_f32(const float* hc, const float* x_prev, const float* w_g, const float* b_g,
                       const float* r_static, const float* w_r, const float* b_r, float eps_r, float beta,
                       int32_t layer_norm, int32_t residual, int32_t V, int32_t d, float c, float c_radius,
                       float* h_out, float* x_out, float* r_out, void* stream);

/* ---- a11/a12/f2: all-entity hyperbolic scoring ------------------------------------- */
/* _chunked_hyperbolic_dist_score, hyperbolic_decoder.py:89-179.  scale/margin: device
 * scalars or NULL (1, 0).  bias [N] or NULL.  use_dist=1 selects the true hyperbolic
 * distance (computed with fp64 MFMA: the arctanh distance is linear in |(-q)(+)e| and an
 * fp32 expansion would lose ~3 digits on near-duplicate pairs); c_rel [B] (or NULL) the
 * per-query curvature of --plus-relation-specific-curvature.  out: [B][N] fp32. */
int regcn_hyp_score_f32(const float* q, const float* cand, const float* bias, const float* c_rel, const float* scale, const float* margin, int32_t B,
                        int32_t N, int32_t d, float c, int32_t use_dist, float* out, void* stream);
/* _chunked_hyperbolic_ce_loss, hyperbolic_decoder.py:182-307: per-query lse - target logit
 * (the caller takes the mean).  workspace: regcn_hyp_ce_workspace_bytes(B, N) bytes. */
size_t regcn_hyp_ce_workspace_bytes(int32_t B, int32_t N);
int regcn_hyp_ce_f32(const float* q, const float* cand, const float* bias, const float* c_rel, const float* scale, const float* margin,
                     const int32_t* target, int32_t B, int32_t N, int32_t d, float c, int32_t use_dist,
                     void* workspace, float* loss_per_query, void* stream);
/* get_total_rank / sort_and_rank / filter_score, rgcn/utils.py:21-166: 1 + count of
 * candidates scoring strictly above the target, raw and excluding the CSR list of other
 * true answers (filt_ptr [B+1], filt_idx; NULL filt_ptr skips the filtered rank). */
int regcn_rank_f32(const float* score, int32_t B, int32_t N, const int32_t* target, const int32_t* filt_ptr,
                   const int32_t* filt_idx, int32_t* rank_raw, int32_t* rank_filt, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* REGCN_HIP_H */
