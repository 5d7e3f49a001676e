// Edge-message device pieces shared by the CSR aggregation kernels (aggregate.hip) and
// the fused gather + layer kernels (layer.hip).
//
// Row layout as everywhere: one 64-lane wave per row, lane l owns columns [4l, 4l+4).
#pragma once
#include "common.h"

namespace regcn {

struct Chunk {
  int row, beg, end, slot;
};

struct Fixup {
  int row, sbeg, send, pad;
};

enum AggMode : int { AGG_UNION = 0, AGG_MEAN = 1, AGG_EUCLID = 2, AGG_LORENTZ = 3, AGG_NONE = 4 };

// Row loads through a buffer resource built from the wave-uniform row base (SGPRs) with the
// lane's byte offset as voffset: no per-lane 64-bit address arithmetic per row.
__device__ __forceinline__ f4 row_load4(const float* row, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row), (short)0, 0x7FFFFFFF, 0x00020000);
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// The same load with a wave-uniform record count: nrec = 0 makes every lane out of range, so
// the load returns zeros without a memory request (a skipped duplicate row, branch-free).
__device__ __forceinline__ f4 row_load4_n(const float* row, uint32_t off, int nrec) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row), (short)0, nrec, 0x00020000);
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

__device__ __forceinline__ int rl(int v, int j) { return __builtin_amdgcn_readlane(v, j); }
__device__ __forceinline__ float rlf(float v, int j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

// Full 64-lane sums of EB in {4, 8} per-lane values at once (the |m|^2 of a batch of
// edges), transposing while reducing: v_permlane32_swap folds two values' halves into one
// register (lanes 0-31 one value, 32-63 the other), v_permlane16_swap folds rows likewise,
// then a DPP butterfly finishes each 16-lane row.  20 VALU for 8 values instead of 8 wave
// sums (~100).  Value u ends replicated over the 16 lanes of one row; batch_lane<EB>(u)
// names a lane holding it.
template <int EB>
__device__ __forceinline__ int batch_lane(int u) { return EB == 8 ? 16 * (u >> 1) + (u & 1) : 16 * u; }
// which value's sum lane `lane` holds (valid for lanes 0..63 when EB == 4; EB == 8: the
// row's value for its lane parity)
template <int EB>
__device__ __forceinline__ int batch_row(int lane) { return EB == 8 ? 2 * (lane >> 4) + (lane & 1) : lane >> 4; }

__device__ __forceinline__ float fold_pair32(float a, float b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float fold_pair16(float a, float b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Returns, in lane batch_lane<EB>(u) (and its row), sum over lanes of v[u].
template <int EB>
__device__ __forceinline__ float batch_sums(const float* v, int lane) {
  static_assert(EB == 4 || EB == 8, "batch of 4 or 8");
  if constexpr (EB == 8) {
    // rows of y0: v0 v2 v4 v6, rows of y1: v1 v3 v5 v7
    const float w0 = fold_pair32(v[0], v[4]), w1 = fold_pair32(v[1], v[5]);
    const float w2 = fold_pair32(v[2], v[6]), w3 = fold_pair32(v[3], v[7]);
    const float y0 = row16_sum(fold_pair16(w0, w2)), y1 = row16_sum(fold_pair16(w1, w3));
    return (lane & 1) ? y1 : y0;
  } else {
    // rows: v0 v1 v2 v3
    return row16_sum(fold_pair16(fold_pair32(v[0], v[2]), fold_pair32(v[1], v[3])));
  }
}

// ------------------------------------------------------------------------------ Lorentz
// Per edge (hyperbolic_layers.py:589-611):
//   m = blockdiag_k(W[type]_k (s x s)) . x_src + rel[type];  p = exp0(m);
//   L = (x0 = (1 + c|p|^2) / (sqrt_c den), xi = 2 p / den),  den = max(1 - c|p|^2, eps)
// Per destination (hyperbolic_layers.py:613-625, hyperbolic_ops.py:562-581): the
// mailbox weights are uniform, so the weighted centroid equals S / sqrt(-<S,S>_L c)
// with S = sum_e L_e; then to_poincare -> log0 (hyperbolic_layers.py:669-671).
//
// Relation block fragment of one lane: the s x s blocks covering columns [4l, 4l+4).
template <int S>
struct WFrag {
  static constexpr int NV = S == 4 ? 4 : (S == 2 ? 2 : 1);
  f4 w[NV];
  __device__ __forceinline__ void load(const float* __restrict__ Wt, int col) {
#pragma unroll
    for (int i = 0; i < NV; ++i) w[i] = *reinterpret_cast<const f4*>(Wt + S * col + 4 * i);
  }
  // Same, from a wave-uniform block base plus this lane's byte offset (4 S col).
  __device__ __forceinline__ void load_row(const float* Wt, uint32_t off) {
#pragma unroll
    for (int i = 0; i < NV; ++i) w[i] = row_load4(Wt, off + 16 * i);
  }
  // m[j] = sum_i x[blk*s + i] W[blk][i][j]  (bmm(node (1 x s), weight (s x s)), :593-598)
  __device__ __forceinline__ f4 apply(f4 xs) const {
    if constexpr (S == 1) return xs * w[0];
    else if constexpr (S == 2) {
      // (m0, m1) = x0 (W00, W01) + x1 (W10, W11): packed-fp32 pairs straight from the
      // loaded quads (v_pk_mul / v_pk_fma with a broadcast operand, no repacking moves)
      const f2 lo = w[0].zw * xs.y + w[0].xy * xs.x;
      const f2 hi = w[1].zw * xs.w + w[1].xy * xs.z;
      return f4{lo.x, lo.y, hi.x, hi.y};
    }
    else return xs.x * w[0] + xs.y * w[1 % NV] + xs.z * w[2 % NV] + xs.w * w[3 % NV];
  }
};

// Any block size s: the source row staged in (per-wave) LDS.
__device__ __forceinline__ float block_general(const float* xsh, const float* __restrict__ Wt, int s, int c) {
  const int blk = c / s, jj = c - blk * s;
  const float* w = Wt + (int64_t)blk * s * s + jj;
  const float* xb = xsh + blk * s;
  float m = 0.f;
  for (int i = 0; i < s; ++i) m += xb[i] * w[i * s];
  return m;
}

__device__ __forceinline__ f4 block_general4(float* xsh, f4 xs, const float* __restrict__ Wt, int s, int col,
                                             bool active) {
  if (active) *reinterpret_cast<f4*>(xsh + col) = xs;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  f4 m = {0.f, 0.f, 0.f, 0.f};
  if (active) {
    m.x = block_general(xsh, Wt, s, col);
    m.y = block_general(xsh, Wt, s, col + 1);
    m.z = block_general(xsh, Wt, s, col + 2);
    m.w = block_general(xsh, Wt, s, col + 3);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return m;
}

// Lorentz point of exp0(m), accumulated into (acc0, acc).
__device__ __forceinline__ void lorentz_accum(f4 m, float n2, const Curv& k, float& acc0, f4& acc) {
  float p2;
  const float f = exp0_factor(n2, k, &p2);
  const float den = fmaxf(1.f - k.c * p2, REGCN_EPS);
  acc0 += (1.f + k.c * p2) / (k.sqrt_c * den);
  acc += m * (2.f * f / den);
}

// Lorentz centroid of the summed points -> Poincare -> log0 (the aggregated tangent row).
__device__ __forceinline__ f4 lorentz_finish(float acc0, f4 acc, const Curv& k) {
  const float ip = -acc0 * acc0 + wave_sum(dot4(acc, acc));
  const float sc = sqrtf(fmaxf(-ip * k.c, REGCN_EPS));
  const float c0 = acc0 / sc;
  f4 y = (acc / sc) / fmaxf(1.f + c0 * k.sqrt_c, REGCN_EPS);
  return row_log0(y, k);
}

}  // namespace regcn
