// Row-tile fp32 MFMA GEMMs with full-row epilogues.
//
// Shape: out[V, d] = A[V, d] @ W[d, d] (+ more products), d <= 256, d % 4 == 0.
// A workgroup (4 waves) owns a tile of TM = 16 rows and ALL d output columns; wave w
// owns the four 16-column MFMA tiles [64w, 64w + 64).  So every wave has a short MFMA
// chain (4 tiles x d/4 k-steps) and a snapshot of a few thousand rows still spreads over
// all 256 CUs, while the row maps (exp0/log0/project/normalize, the radius-MLP dot) run
// right after the MFMA chain with one cross-wave LDS reduction per row norm: no
// intermediate V x d tensor goes back to HBM.
//
// Operands.  The A tile (16 x d, rows gathered through `rows`) is staged into LDS once per
// product with coalesced float4 row loads; each k-step a lane reads one A element with
// ds_read_b32.  The weights are prepacked once (regcn_pack_weight_f32) into MFMA fragment
// order  Wp[s][jq][lane][e] = W[4s + lane/16][16(4jq + e) + lane%16], so at k-step s wave
// w needs exactly one coalesced float4 per lane, Wp[s][w][lane]; these stream from L2
// (the packed matrix is shared by every workgroup) through an 8-deep register ring.
//
// MFMA: v_mfma_f32_16x16x4_f32 (exact fp32 fma chain; gfx950 has no xf32).  C/D layout:
// lane l holds rows 4*(l>>4)+r (r = reg 0..3) and column 16j + (l & 15) of tile j, so a
// row's 16 lanes are one DPP row and reduce with row16_sum.
#include "common.h"
#include "regcn_internal.h"

namespace regcn {

constexpr int MAX_D = 256;
constexpr int TM = 16;          // rows per workgroup
constexpr int NWAVE = 4;        // waves per workgroup = column groups of 64
constexpr int LDA = MAX_D + 2;  // stride = 2 (mod 32): lanes (row r, k-offset q) hit bank 2r+q
constexpr int RING = 8;         // k-steps of B fragments in flight per wave

struct Tile {
  float A[TM * LDA];
  float red[2][NWAVE][TM];  // cross-wave row partial sums (double-buffered)
  int rows[TM];
};

// Four 16x16 accumulator tiles of one wave: t[jl] is global column tile 4*wave + jl.
struct Frag {
  f4 t[4];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = f4{0.f, 0.f, 0.f, 0.f};
  }
};

__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }
__device__ __forceinline__ int frag_row(int r) { return 4 * ((threadIdx.x & 63) >> 4) + r; }
__device__ __forceinline__ int frag_col(int jl) { return 64 * wave_id() + 16 * jl + (threadIdx.x & 15); }

// Stage A[rows[0..n_valid)] (row-major, width d) into LDS; rows past n_valid are zero.
// Loads are unconditional (row index clamped) so they all stay in flight together.
template <bool CLAMP10>
__device__ __forceinline__ void stage_rows(Tile& sh, const float* __restrict__ A, int d, int n_valid) {
  constexpr int IT = TM * (MAX_D / 4) / (64 * NWAVE);  // 4 float4 per thread at d = 256
  const int q4 = d >> 2, n = TM * q4;
  f4 v[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {  // all loads first (clamped addresses), then the LDS stores
    const int idx = min((int)threadIdx.x + it * 64 * NWAVE, n - 1);
    const int i = idx / q4, c = (idx - i * q4) * 4;
    v[it] = *reinterpret_cast<const f4*>(A + (int64_t)sh.rows[i < n_valid ? i : 0] * d + c);
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = threadIdx.x + it * 64 * NWAVE;
    if (idx >= n) break;
    const int i = idx / q4, c = (idx - i * q4) * 4;
    f4 x = v[it];
    if (CLAMP10) x = clamp4(x, -10.f, 10.f);
    if (i >= n_valid) x = f4{0.f, 0.f, 0.f, 0.f};
    float* dst = sh.A + i * LDA + c;
    dst[0] = x.x;
    dst[1] = x.y;
    dst[2] = x.z;
    dst[3] = x.w;
  }
}

__device__ __forceinline__ void mfma4(Frag& acc, float a, f4 b) {
  acc.t[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.x, acc.t[0], 0, 0, 0);
  acc.t[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.y, acc.t[1], 0, 0, 0);
  acc.t[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.z, acc.t[2], 0, 0, 0);
  acc.t[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b.w, acc.t[3], 0, 0, 0);
}

// acc += A_tile @ W (A_tile in LDS, W packed).  Caller syncs around it.
__device__ __forceinline__ void mfma_tile(Frag& acc, const Tile& sh, const float* __restrict__ Wp, int d) {
  const int lane = threadIdx.x & 63, w = wave_id();
  const int S = d >> 2;
  const f4* bsrc = reinterpret_cast<const f4*>(Wp) + w * 64 + lane;  // + s * 256
  const float* arow = sh.A + (lane & 15) * LDA + (lane >> 4);
  f4 ring[RING];
#pragma unroll
  for (int i = 0; i < RING; ++i) ring[i] = bsrc[(int64_t)min(i, S - 1) * 256];
  int s = 0;
  for (; s + RING <= S; s += RING) {
#pragma unroll
    for (int i = 0; i < RING; ++i) {
      mfma4(acc, arow[4 * (s + i)], ring[i]);
      __builtin_amdgcn_sched_barrier(0);
      ring[i] = bsrc[(int64_t)min(s + i + RING, S - 1) * 256];  // unconditional: hipcc can count it
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int i = 0; i < RING; ++i)
    if (s + i < S) mfma4(acc, arow[4 * (s + i)], ring[i]);
}

// Sum of per-wave row partials across the 4 waves (two LDS buffers alternate, so one
// barrier per reduction).  part[r] = this wave's partial for frag_row(r).
__device__ __forceinline__ void rows_allreduce(Tile& sh, int& buf, float part[4]) {
  const int lane = threadIdx.x & 63, w = wave_id();
#pragma unroll
  for (int r = 0; r < 4; ++r) part[r] = row16_sum(part[r]);
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) sh.red[buf][w][frag_row(r)] = part[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = frag_row(r);
    part[r] = (sh.red[buf][0][i] + sh.red[buf][1][i]) + (sh.red[buf][2][i] + sh.red[buf][3][i]);
  }
  buf ^= 1;
}

__device__ __forceinline__ void row_sumsq(Tile& sh, int& buf, const Frag& a, float out[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) s += a.t[j][r] * a.t[j][r];
    out[r] = s;
  }
  rows_allreduce(sh, buf, out);
}

__device__ __forceinline__ void row_scale(Frag& a, const float f[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) a.t[j][r] *= f[r];
}

__device__ __forceinline__ void frag_log0(Tile& sh, int& buf, Frag& a, const Curv& k) {
  float n2[4], f[4];
  row_sumsq(sh, buf, a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = log0_factor(n2[r], k);
  row_scale(a, f);
}

__device__ __forceinline__ void frag_exp0(Tile& sh, int& buf, Frag& a, const Curv& k) {
  float n2[4], f[4];
  row_sumsq(sh, buf, a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = exp0_factor(n2[r], k);
  row_scale(a, f);
}

__device__ __forceinline__ void frag_project(Tile& sh, int& buf, Frag& a, const Curv& k) {
  float n2[4], f[4];
  row_sumsq(sh, buf, a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = project_factor(n2[r], k);
  row_scale(a, f);
}

__device__ __forceinline__ void frag_normalize(Tile& sh, int& buf, Frag& a) {  // F.normalize, eps 1e-12
  float n2[4], f[4];
  row_sumsq(sh, buf, a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = 1.0f / fmaxf(sqrtf(n2[r]), 1e-12f);
  row_scale(a, f);
}

// Fragment of a V x d row-major matrix for the tile's rows (unconditional loads from
// clamped addresses, then a select: no per-load branch / vmcnt(0)).
__device__ __forceinline__ void frag_load(Frag& a, const float* __restrict__ M, const int* rows, int n_valid, int d) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = frag_row(r);
    const bool ok = i < n_valid;
    const int64_t base = (int64_t)rows[ok ? i : 0] * d;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = frag_col(j);
      const float v = M[base + min(col, d - 1)];
      a.t[j][r] = (ok && col < d) ? v : 0.f;
    }
  }
}

// Per-column vector (bias / weight row) in the fragment's column order.
__device__ __forceinline__ void col_load(float out[4], const float* __restrict__ v, int d) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = frag_col(j);
    const float x = v[min(col, d - 1)];
    out[j] = col < d ? x : 0.f;
  }
}

// C-layout fragment read back from the LDS A tile (the operand just multiplied).
__device__ __forceinline__ void frag_from_tile(Frag& a, const Tile& sh, int d) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float* row = sh.A + frag_row(r) * LDA;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = frag_col(j);
      const float v = row[min(col, MAX_D - 1)];
      a.t[j][r] = col < d ? v : 0.f;
    }
  }
}

__device__ __forceinline__ void frag_store(const Frag& a, float* __restrict__ M, const int* rows, int n_valid, int d) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = frag_row(r);
    if (i >= n_valid) continue;
    const int64_t base = (int64_t)rows[i] * d;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = frag_col(j);
      if (col < d) M[base + col] = a.t[j][r];
    }
  }
}

__device__ __forceinline__ void store_radius(const float n2[4], float* __restrict__ rad, const int* rows,
                                             int n_valid) {
  if ((threadIdx.x & 15) == 0 && wave_id() == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = frag_row(r);
      if (i < n_valid) rad[rows[i]] = fmaxf(sqrtf(n2[r]), REGCN_EPS);
    }
  }
}

// ============================================================================ pack weights
// Wp[s][jq][lane][e] = W[4s + lane/16][16(4jq + e) + lane%16] (zero outside d_in x d_out).
__global__ void k_pack_weight(const float* __restrict__ W, int d_in, int d_out, float* __restrict__ Wp) {
  const int S = (d_in + 3) >> 2;
  const int total = S * 4 * 64 * 4;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int e = idx & 3, lane = (idx >> 2) & 63, jq = (idx >> 8) & 3, s = idx >> 10;
    const int k = 4 * s + (lane >> 4), n = 16 * (4 * jq + e) + (lane & 15);
    Wp[idx] = (k < d_in && n < d_out) ? W[(int64_t)k * d_out + n] : 0.f;
  }
}

// =============================================================================== layer
// Union / Lorentz / Euclidean layer tail (hyperbolic_layers.py:273-323, :648-694,
// rgcn/layers.py:226-255).  rows[0, n_pos) have in-degree > 0, rows[n_pos, V) not; a tile
// never mixes the two, so it multiplies by exactly one self-loop weight.
//   hyperbolic:  v = clamp(agg @ W_n | agg) + x @ (W_loop | W_evolve)
//                [v = g * v + (1 - g) * prev_t, g = sigmoid(prev_t @ W_skip + b)]
//                h = exp0(leaky(clamp(v)) [* dropout mask])
//   euclidean :  h = leaky(agg @ W_n + x @ (W_loop | W_evolve)) [* mask]
// Optional outputs: x_next = log0(h) and r_next = max(|h|, eps) for the next layer.
__global__ __launch_bounds__(64 * NWAVE) void k_layer_tail(LayerArgs p) {
  __shared__ Tile sh;
  int buf = 0;
  const int n_pos_tiles = (p.n_pos + TM - 1) / TM;
  const bool pos = (int)blockIdx.x < n_pos_tiles;
  const int r0 = pos ? blockIdx.x * TM : p.n_pos + (blockIdx.x - n_pos_tiles) * TM;
  const int n_valid = min(TM, (pos ? p.n_pos : p.V) - r0);
  if (threadIdx.x < TM) sh.rows[threadIdx.x] = threadIdx.x < n_valid ? p.rows[r0 + threadIdx.x] : 0;
  __syncthreads();

  Frag v;
  v.zero();
  if (pos && p.agg) {
    if (p.w_n) {
      stage_rows<false>(sh, p.agg, p.d, n_valid);
      __syncthreads();
      mfma_tile(v, sh, p.w_n, p.d);
      __syncthreads();
    } else {
      frag_load(v, p.agg, sh.rows, n_valid, p.d);
    }
    if (!p.euclid) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v.t[j] = clamp4(v.t[j], -10.f, 10.f);
    }
  }
  const float* wsel = pos ? p.w_loop : p.w_evolve;
  if (wsel) {
    stage_rows<false>(sh, p.x, p.d, n_valid);
    __syncthreads();
    mfma_tile(v, sh, wsel, p.d);
    __syncthreads();
  }
  if (p.prev_t) {
    stage_rows<false>(sh, p.prev_t, p.d, n_valid);
    __syncthreads();
    Frag g;
    g.zero();
    mfma_tile(g, sh, p.w_skip, p.d);
    Frag pt;
    frag_from_tile(pt, sh, p.d);
    float b[4];
    col_load(b, p.b_skip, p.d);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gt = sigmoidf(g.t[j][r] + b[j]);
        v.t[j][r] = gt * v.t[j][r] + (1.f - gt) * pt.t[j][r];
      }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!p.euclid) v.t[j] = clamp4(v.t[j], -10.f, 10.f);
    v.t[j] = leaky4(v.t[j]);
  }
  if (p.drop_mask) {
    Frag m;
    frag_load(m, p.drop_mask, sh.rows, n_valid, p.d);
#pragma unroll
    for (int j = 0; j < 4; ++j) v.t[j] *= m.t[j];
  }
  if (!p.euclid) frag_exp0(sh, buf, v, p.k);
  frag_store(v, p.h_out, sh.rows, n_valid, p.d);
  if (p.r_next || (p.x_next && !p.euclid)) {
    float n2[4];
    row_sumsq(sh, buf, v, n2);
    if (p.r_next) store_radius(n2, p.r_next, sh.rows, n_valid);
    if (p.x_next && !p.euclid) {
      float f[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) f[r] = log0_factor(n2[r], p.k);
      row_scale(v, f);
    }
  }
  if (p.x_next) frag_store(v, p.x_next, sh.rows, n_valid, p.d);
}

// ============================================================================ timestep
// Per-timestep entity evolution (hyperbolic_model.py:829-869, hyperbolic_ops.py:395-435):
//   cur = project(hc); [LN: cur = exp0(normalize(log0(cur)))]
//   ct = clamp(log0(cur)); pt = clamp(x_prev)  (x_prev = log0(h_prev))
//   tw = sigmoid(pt @ W_g + b_g);  h = project(exp0(tw*ct + (1-tw)*pt))
//   residual: delta = clamp(log0(h).w_r + b_r, +-eps_r); r = beta*r_s + (1-beta)|h| + delta
//   else: r = r_s;   h = apply_radius(h, r)
// Outputs h, x = log0(h), r = max(|h|, eps).
__global__ __launch_bounds__(64 * NWAVE) void k_timestep(StepArgs p) {
  __shared__ Tile sh;
  int buf = 0;
  const int r0 = blockIdx.x * TM;
  const int n_valid = min(TM, p.V - r0);
  if (threadIdx.x < TM) sh.rows[threadIdx.x] = r0 + (threadIdx.x < n_valid ? threadIdx.x : 0);
  __syncthreads();

  stage_rows<true>(sh, p.x_prev, p.d, n_valid);
  __syncthreads();
  Frag tw;
  tw.zero();
  mfma_tile(tw, sh, p.w_g, p.d);

  Frag ct;
  frag_load(ct, p.hc, sh.rows, n_valid, p.d);
  frag_project(sh, buf, ct, p.k);
  if (p.layer_norm) {
    frag_log0(sh, buf, ct, p.k);
    frag_normalize(sh, buf, ct);
    frag_exp0(sh, buf, ct, p.k);
  }
  frag_log0(sh, buf, ct, p.k);
  Frag pt;
  frag_from_tile(pt, sh, p.d);  // clamp(x_prev), staged with CLAMP10
  float bg[4];
  col_load(bg, p.b_g, p.d);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f4 c4 = clamp4(ct.t[j], -10.f, 10.f);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float g = sigmoidf(tw.t[j][r] + bg[j]);
      ct.t[j][r] = g * c4[r] + (1.f - g) * pt.t[j][r];
    }
  }
  frag_exp0(sh, buf, ct, p.k);
  frag_project(sh, buf, ct, p.k);  // hyperbolic_model.py:860
  float n2[4], rs[4], newr[4];
  row_sumsq(sh, buf, ct, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = frag_row(r);
    rs[r] = p.r_static[sh.rows[i < n_valid ? i : 0]];
  }
  if (p.residual) {
    float wr[4], dl[4];
    col_load(wr, p.w_r, p.d);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float f = log0_factor(n2[r], p.k_rad);
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) s += wr[j] * (ct.t[j][r] * f);
      dl[r] = s;
    }
    rows_allreduce(sh, buf, dl);
    const float br = *p.b_r;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float delta = fminf(fmaxf(dl[r] + br, -p.eps_r), p.eps_r);
      const float dyn = fmaxf(sqrtf(n2[r]), REGCN_EPS);
      newr[r] = (p.beta * rs[r] + (1.f - p.beta) * dyn) + delta;
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
  if (p.r_out || p.x_out) {
    float h2[4];
    row_sumsq(sh, buf, ct, h2);
    if (p.r_out) store_radius(h2, p.r_out, sh.rows, n_valid);
    if (p.x_out) {
      float g[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) g[r] = log0_factor(h2[r], p.k);
      row_scale(ct, g);
      frag_store(ct, p.x_out, sh.rows, n_valid, p.d);
    }
  }
}

// ============================================================================ launchers
int layer_tail(const LayerArgs& a, hipStream_t st) {
  if (a.d <= 0 || a.d > MAX_D || (a.d & 3)) return set_error(REGCN_EINVAL, "layer tail needs d %% 4 == 0, d <= 256");
  if (!a.x || !a.rows || !a.h_out) return set_error(REGCN_EINVAL, "null pointer");
  if ((a.w_loop == nullptr) != (a.w_evolve == nullptr)) return set_error(REGCN_EINVAL, "self-loop weights must come in pairs");
  if (a.prev_t && (!a.w_skip || !a.b_skip)) return set_error(REGCN_EINVAL, "skip needs weight and bias");
  if (a.n_pos < 0 || a.n_pos > a.V) return set_error(REGCN_EINVAL, "bad n_pos");
  if (a.V == 0) return 0;
  const unsigned grid = (unsigned)((a.n_pos + TM - 1) / TM + (a.V - a.n_pos + TM - 1) / TM);
  hipLaunchKernelGGL(k_layer_tail, dim3(grid), dim3(64 * NWAVE), 0, st, a);
  return check_launch("k_layer_tail");
}

int timestep(const StepArgs& a, hipStream_t st) {
  if (a.d <= 0 || a.d > MAX_D || (a.d & 3)) return set_error(REGCN_EINVAL, "timestep needs d %% 4 == 0, d <= 256");
  if (!a.hc || !a.x_prev || !a.w_g || !a.b_g || !a.r_static || !a.h_out) return set_error(REGCN_EINVAL, "null pointer");
  if (a.residual && (!a.w_r || !a.b_r)) return set_error(REGCN_EINVAL, "residual radius needs w_r and b_r");
  if (a.V == 0) return 0;
  const unsigned grid = (unsigned)((a.V + TM - 1) / TM);
  hipLaunchKernelGGL(k_timestep, dim3(grid), dim3(64 * NWAVE), 0, st, a);
  return check_launch("k_timestep");
}

size_t packed_weight_floats(int d_in) { return (size_t)((d_in + 3) / 4) * 4 * 64 * 4; }

int pack_weight(const float* W, int d_in, int d_out, float* Wp, hipStream_t st) {
  if (!W || !Wp) return set_error(REGCN_EINVAL, "null pointer");
  if (d_in <= 0 || d_out <= 0 || d_out > MAX_D) return set_error(REGCN_EINVAL, "pack_weight needs d_out <= 256");
  const int total = (int)packed_weight_floats(d_in);
  hipLaunchKernelGGL(k_pack_weight, dim3((total + 255) / 256), dim3(256), 0, st, W, d_in, d_out, Wp);
  return check_launch("k_pack_weight");
}

}  // namespace regcn
