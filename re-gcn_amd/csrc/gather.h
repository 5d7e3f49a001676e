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

__device__ __forceinline__ int rl(int v, int j) { return __builtin_amdgcn_readlane(v, j); }
__device__ __forceinline__ float rlf(float v, int j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
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
  // m[j] = sum_i x[blk*s + i] W[blk][i][j]  (bmm(node (1 x s), weight (s x s)), :593-598)
  __device__ __forceinline__ f4 apply(f4 xs) const {
    if constexpr (S == 1) return xs * w[0];
    else if constexpr (S == 2)
      return f4{xs.x * w[0].x + xs.y * w[0].z, xs.x * w[0].y + xs.y * w[0].w, xs.z * w[1].x + xs.w * w[1].z,
                xs.z * w[1].y + xs.w * w[1].w};
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
