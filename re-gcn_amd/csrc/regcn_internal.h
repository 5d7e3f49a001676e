// Host-side internals shared by the kernel translation units (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/regcn_hip.h"
#include "common.h"

namespace regcn {

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

// aggregate.hip
int gather_sum(int mode, const float* x, const float* radius, const float* rel, const int* col_src,
               const int* col_type, const float* rowscale, const void* chunks, int n_chunks,
               const void* fixups, int n_fix, float gamma, int d, float* partial, int pstride, float* out,
               hipStream_t st);
int lorentz_sum(const float* x, const float* rel, const float* W, const int* col_src, const int* col_type,
                const void* chunks, int n_chunks, const void* fixups, int n_fix, int nb, float c, int d,
                float* partial, int pstride, float* out, hipStream_t st);

// ---- argument blocks of the fused kernels (rowgemm.hip, score.hip) ----
struct LayerArgs {
  const float* agg;
  const float* w_n;
  const float* x;
  const float* w_loop;
  const float* w_evolve;
  const float* prev_t;
  const float* w_skip;
  const float* b_skip;
  const float* drop_mask;
  const int* rows;
  int n_pos, V, d, euclid;
  Curv k;
  float* h_out;
  float* x_next;
  float* r_next;
};

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
  float scale, margin;   // filled in-kernel from the pointers
  float* out;            // [B, N] score (SCORE mode)
  float* part;           // [B, nblk, 2] (CE mode): running max, sum exp
  float* tgt_logit;      // [B] (CE mode)
};

size_t packed_weight_floats(int d_in);
int pack_weight(const float* W, int d_in, int d_out, float* Wp, hipStream_t st);
int layer_tail(const LayerArgs& a, hipStream_t st);
int timestep(const StepArgs& a, hipStream_t st);
int score(ScoreArgs& a, int mode, float* loss, hipStream_t st);
int rank(const float* S, int B, int N, const int* target, const int* filt_ptr, const int* filt_idx, int* rank_raw,
         int* rank_filt, hipStream_t st);

}  // namespace regcn
