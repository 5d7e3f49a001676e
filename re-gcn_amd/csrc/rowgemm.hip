// Row-tile fp32 MFMA GEMMs with full-row epilogues.
//
// Shape: out[V, d] = A[V, d] @ W[d, d] (+ more products), d <= 256, d % 4 == 0.
// A workgroup (256 threads = 4 waves) owns a tile of 64 rows and ALL d output
// columns, so row norms (exp0/log0/project/normalize/dot with the radius MLP)
// are done in registers right after the MFMA chain: no intermediate V x d
// tensor ever goes back to HBM.  Wave w owns tile rows [16w, 16w+16) and the
// NT = ceil(d/16) 16x16 accumulator tiles of v_mfma_f32_16x16x4_f32 (exact fp32
// fma chain; gfx950 has no xf32).  K is streamed through LDS in 16-deep chunks.
//
// C/D fragment layout (16x16x4 f32): lane l holds rows 4*(l>>4)+r (r = reg 0..3)
// and column 16j + (l & 15) of tile j, so a row's 16 lanes reduce with 4 xor
// shuffles (group16_sum).
#include "common.h"
#include "regcn_internal.h"

namespace regcn {

constexpr int TILE_M = 64;
constexpr int KC = 16;
constexpr int AS_LD = KC + 1;

template <int NT>
struct Acc {
  f4 t[NT];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int j = 0; j < NT; ++j) t[j] = f4{0.f, 0.f, 0.f, 0.f};
  }
};

// Shared staging buffers for one K-chunk.
template <int NT>
struct Stage {
  float As[TILE_M * AS_LD];
  float Bs[KC * NT * 16];
  int rows[TILE_M];
};

// acc += A[rows] @ W, with A row-major (lda = d) and W row-major (d x d).
// A-row transform: CLAMP10 applies clamp(+-10) on load (time gate prev tangent).
template <int NT, bool CLAMP10>
__device__ __forceinline__ void mfma_rows_x_w(Acc<NT>& acc, Stage<NT>& sh, const float* __restrict__ A,
                                              const float* __restrict__ W, int d, int n_valid) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  for (int k0 = 0; k0 < d; k0 += KC) {
    __syncthreads();
    {  // stage A: 64 rows x 16 k  (256 threads x one float4)
      const int i = tid >> 2, kq = (tid & 3) * 4;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (i < n_valid && k0 + kq < d) {
        v = *reinterpret_cast<const f4*>(A + (int64_t)sh.rows[i] * d + k0 + kq);
        if (CLAMP10) v = clamp4(v, -10.f, 10.f);
      }
      float* dst = sh.As + i * AS_LD + kq;
      dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
    }
    // stage W: 16 k-rows x NT*16 cols
    for (int idx = tid; idx < KC * NT * 4; idx += 256) {
      const int kr = idx / (NT * 4), n4 = (idx - kr * NT * 4) * 4;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (k0 + kr < d && n4 < d) v = *reinterpret_cast<const f4*>(W + (int64_t)(k0 + kr) * d + n4);
      *reinterpret_cast<f4*>(sh.Bs + kr * NT * 16 + n4) = v;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < KC; kk += 4) {
      const float a = sh.As[(16 * wv + (lane & 15)) * AS_LD + kk + (lane >> 4)];
      const float* brow = sh.Bs + (kk + (lane >> 4)) * NT * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < NT; ++j) acc.t[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, brow[16 * j], acc.t[j], 0, 0, 0);
    }
  }
}

// Per-row (4 rows per lane) helpers on C-layout fragments.
template <int NT>
__device__ __forceinline__ void row_sumsq(const Acc<NT>& a, float out[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NT; ++j) s += a.t[j][r] * a.t[j][r];
    out[r] = group16_sum(s);
  }
}

template <int NT>
__device__ __forceinline__ void row_scale(Acc<NT>& a, const float f[4]) {
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) a.t[j][r] *= f[r];
}

template <int NT>
__device__ __forceinline__ void frag_log0(Acc<NT>& a, const Curv& k) {
  float n2[4], f[4];
  row_sumsq(a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = log0_factor(n2[r], k);
  row_scale(a, f);
}

template <int NT>
__device__ __forceinline__ void frag_exp0(Acc<NT>& a, const Curv& k) {
  float n2[4], f[4];
  row_sumsq(a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = exp0_factor(n2[r], k);
  row_scale(a, f);
}

template <int NT>
__device__ __forceinline__ void frag_project(Acc<NT>& a, const Curv& k) {
  float n2[4], f[4];
  row_sumsq(a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = project_factor(n2[r], k);
  row_scale(a, f);
}

template <int NT>
__device__ __forceinline__ void frag_normalize(Acc<NT>& a) {  // F.normalize, eps 1e-12
  float n2[4], f[4];
  row_sumsq(a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = 1.0f / fmaxf(sqrtf(n2[r]), 1e-12f);
  row_scale(a, f);
}

// Load / store fragments of a V x d row-major matrix for the tile's rows.
template <int NT>
__device__ __forceinline__ void frag_load(Acc<NT>& a, const float* __restrict__ M, const int* rows, int n_valid,
                                          int d) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 16 * wv + 4 * (lane >> 4) + r;
    const bool ok = i < n_valid;
    const int64_t base = ok ? (int64_t)rows[i] * d : 0;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = 16 * j + (lane & 15);
      a.t[j][r] = (ok && col < d) ? M[base + col] : 0.f;
    }
  }
}

template <int NT>
__device__ __forceinline__ void frag_store(const Acc<NT>& a, float* __restrict__ M, const int* rows, int n_valid,
                                           int d) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 16 * wv + 4 * (lane >> 4) + r;
    if (i >= n_valid) continue;
    const int64_t base = (int64_t)rows[i] * d;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = 16 * j + (lane & 15);
      if (col < d) M[base + col] = a.t[j][r];
    }
  }
}

template <int NT>
__device__ __forceinline__ void frag_store_radius(const Acc<NT>& a, float* __restrict__ rad, const int* rows,
                                                  int n_valid) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float n2[4];
  row_sumsq(a, n2);
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * wv + 4 * (lane >> 4) + r;
      if (i < n_valid) rad[rows[i]] = fmaxf(sqrtf(n2[r]), REGCN_EPS);
    }
  }
}

// =============================================================================== layer
// Union / Lorentz / Euclidean layer tail (hyperbolic_layers.py:273-323, :648-694,
// rgcn/layers.py:226-255).  rows[0, n_pos) have in-degree > 0, rows[n_pos, V) not.
//   hyperbolic:  v = clamp(agg @ W_n | agg) + x @ (W_loop | W_evolve)
//                [v = g * v + (1 - g) * prev_t, g = sigmoid(prev_t @ W_skip + b)]
//                h = exp0(leaky(clamp(v)) [* dropout mask])
//   euclidean :  h = leaky(agg @ W_n + x @ (W_loop | W_evolve)) [* mask]
// Optional outputs: x_next = log0(h) and r_next = max(|h|, eps) for the next layer.


template <int NT>
__global__ __launch_bounds__(256) void k_layer_tail(LayerArgs p) {
  __shared__ Stage<NT> sh;
  const int n_pos_tiles = (p.n_pos + TILE_M - 1) / TILE_M;
  const bool pos = (int)blockIdx.x < n_pos_tiles;
  const int r0 = pos ? blockIdx.x * TILE_M : p.n_pos + (blockIdx.x - n_pos_tiles) * TILE_M;
  const int n_valid = min(TILE_M, (pos ? p.n_pos : p.V) - r0);
  if (threadIdx.x < TILE_M) sh.rows[threadIdx.x] = threadIdx.x < n_valid ? p.rows[r0 + threadIdx.x] : 0;
  __syncthreads();

  Acc<NT> v;
  v.zero();
  if (pos && p.agg) {
    if (p.w_n) mfma_rows_x_w<NT, false>(v, sh, p.agg, p.w_n, p.d, n_valid);
    else frag_load(v, p.agg, sh.rows, n_valid, p.d);
    if (!p.euclid) {
#pragma unroll
      for (int j = 0; j < NT; ++j) v.t[j] = clamp4(v.t[j], -10.f, 10.f);
    }
  }
  const float* wsel = pos ? p.w_loop : p.w_evolve;
  if (wsel) mfma_rows_x_w<NT, false>(v, sh, p.x, wsel, p.d, n_valid);
  if (p.prev_t) {
    Acc<NT> g;
    g.zero();
    mfma_rows_x_w<NT, false>(g, sh, p.prev_t, p.w_skip, p.d, n_valid);
    Acc<NT> pt;
    frag_load(pt, p.prev_t, sh.rows, n_valid, p.d);
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = 16 * j + (lane & 15);
      const float b = col < p.d ? p.b_skip[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gt = sigmoidf(g.t[j][r] + b);
        v.t[j][r] = gt * v.t[j][r] + (1.f - gt) * pt.t[j][r];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    if (!p.euclid) v.t[j] = clamp4(v.t[j], -10.f, 10.f);
    v.t[j] = leaky4(v.t[j]);
  }
  if (p.drop_mask) {
    Acc<NT> m;
    frag_load(m, p.drop_mask, sh.rows, n_valid, p.d);
#pragma unroll
    for (int j = 0; j < NT; ++j) v.t[j] *= m.t[j];
  }
  if (!p.euclid) frag_exp0(v, p.k);
  frag_store(v, p.h_out, sh.rows, n_valid, p.d);
  if (p.r_next) frag_store_radius(v, p.r_next, sh.rows, n_valid);
  if (p.x_next) {
    if (!p.euclid) frag_log0(v, p.k);
    frag_store(v, p.x_next, sh.rows, n_valid, p.d);
  }
}

// ============================================================================ timestep
// Per-timestep entity evolution (hyperbolic_model.py:829-869, hyperbolic_ops.py:395-435):
//   cur = project(hc); [LN: cur = exp0(normalize(log0(cur)))]
//   ct = clamp(log0(cur)); pt = clamp(x_prev)  (x_prev = log0(h_prev))
//   tw = sigmoid(pt @ W_g + b_g);  h = project(exp0(tw*ct + (1-tw)*pt))
//   residual: delta = clamp(log0(h).w_r + b_r, +-eps_r); r = beta*r_s + (1-beta)|h| + delta
//   else: r = r_s;   h = apply_radius(h, r)
// Outputs h, x = log0(h), r = max(|h|, eps).


template <int NT>
__global__ __launch_bounds__(256) void k_timestep(StepArgs p) {
  __shared__ Stage<NT> sh;
  const int r0 = blockIdx.x * TILE_M;
  const int n_valid = min(TILE_M, p.V - r0);
  if (threadIdx.x < TILE_M) sh.rows[threadIdx.x] = r0 + (threadIdx.x < n_valid ? threadIdx.x : 0);
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;

  Acc<NT> tw;
  tw.zero();
  mfma_rows_x_w<NT, true>(tw, sh, p.x_prev, p.w_g, p.d, n_valid);

  Acc<NT> ct;
  frag_load(ct, p.hc, sh.rows, n_valid, p.d);
  frag_project(ct, p.k);
  if (p.layer_norm) {
    frag_log0(ct, p.k);
    frag_normalize(ct);
    frag_exp0(ct, p.k);
  }
  frag_log0(ct, p.k);
  Acc<NT> pt;
  frag_load(pt, p.x_prev, sh.rows, n_valid, p.d);
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = 16 * j + (lane & 15);
    const float b = col < p.d ? p.b_g[col] : 0.f;
    const f4 c4 = clamp4(ct.t[j], -10.f, 10.f), p4 = clamp4(pt.t[j], -10.f, 10.f);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float g = sigmoidf(tw.t[j][r] + b);
      ct.t[j][r] = g * c4[r] + (1.f - g) * p4[r];
    }
  }
  frag_exp0(ct, p.k);
  frag_project(ct, p.k);  // hyperbolic_model.py:860
  // radius
  float n2[4], rs[4];
  row_sumsq(ct, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 16 * wv + 4 * (lane >> 4) + r;
    rs[r] = p.r_static[sh.rows[i < n_valid ? i : 0]];
  }
  float newr[4];
  if (p.residual) {
    float dl[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float f = log0_factor(n2[r], p.k_rad);
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = 16 * j + (lane & 15);
        s += (col < p.d ? p.w_r[col] : 0.f) * (ct.t[j][r] * f);
      }
      dl[r] = group16_sum(s) + *p.b_r;
      dl[r] = fminf(fmaxf(dl[r], -p.eps_r), p.eps_r);
      const float dyn = fmaxf(sqrtf(n2[r]), REGCN_EPS);
      newr[r] = (p.beta * rs[r] + (1.f - p.beta) * dyn) + dl[r];
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) newr[r] = rs[r];
  }
  float f[4];
  const Curv& kr = p.residual ? p.k_rad : p.k;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float n = fmaxf(sqrtf(n2[r]), REGCN_EPS);
    f[r] = fminf(fmaxf(newr[r], REGCN_EPS), kr.rmax) / n;
  }
  row_scale(ct, f);
  frag_store(ct, p.h_out, sh.rows, n_valid, p.d);
  if (p.r_out) frag_store_radius(ct, p.r_out, sh.rows, n_valid);
  if (p.x_out) {
    frag_log0(ct, p.k);
    frag_store(ct, p.x_out, sh.rows, n_valid, p.d);
  }
}

// ============================================================================ launchers
template <template <int> class K, class Args>
static int launch_nt(int d, unsigned grid, const Args& a, hipStream_t st, const char* name) {
  dim3 g(grid), b(256);
  if (grid == 0) return 0;
  if (d <= 64) hipLaunchKernelGGL(K<4>::fn, g, b, 0, st, a);
  else if (d <= 128) hipLaunchKernelGGL(K<8>::fn, g, b, 0, st, a);
  else if (d <= 208) hipLaunchKernelGGL(K<13>::fn, g, b, 0, st, a);
  else hipLaunchKernelGGL(K<16>::fn, g, b, 0, st, a);
  return check_launch(name);
}

template <int NT>
struct LayerK {
  static constexpr auto fn = k_layer_tail<NT>;
};
template <int NT>
struct StepK {
  static constexpr auto fn = k_timestep<NT>;
};

int layer_tail(const LayerArgs& a, hipStream_t st) {
  if (a.d <= 0 || a.d > 256 || (a.d & 3)) return set_error(REGCN_EINVAL, "layer tail needs d %% 4 == 0, d <= 256");
  if (!a.x || !a.rows || !a.h_out) return set_error(REGCN_EINVAL, "null pointer");
  if ((a.w_loop == nullptr) != (a.w_evolve == nullptr)) return set_error(REGCN_EINVAL, "self-loop weights must come in pairs");
  if (a.prev_t && (!a.w_skip || !a.b_skip)) return set_error(REGCN_EINVAL, "skip needs weight and bias");
  if (a.n_pos < 0 || a.n_pos > a.V) return set_error(REGCN_EINVAL, "bad n_pos");
  const unsigned grid = (unsigned)((a.n_pos + TILE_M - 1) / TILE_M + (a.V - a.n_pos + TILE_M - 1) / TILE_M);
  return launch_nt<LayerK>(a.d, grid, a, st, "k_layer_tail");
}

int timestep(const StepArgs& a, hipStream_t st) {
  if (a.d <= 0 || a.d > 256 || (a.d & 3)) return set_error(REGCN_EINVAL, "timestep needs d %% 4 == 0, d <= 256");
  if (!a.hc || !a.x_prev || !a.w_g || !a.b_g || !a.r_static || !a.h_out) return set_error(REGCN_EINVAL, "null pointer");
  if (a.residual && !a.w_r) return set_error(REGCN_EINVAL, "residual radius needs w_r");
  const unsigned grid = (unsigned)((a.V + TILE_M - 1) / TILE_M);
  return launch_nt<StepK>(a.d, grid, a, st, "k_timestep");
}

}  // namespace regcn
