// Shared device helpers for the RE-GCN MI355X (gfx950) kernels.
//
// Row layout: a node/relation row of width d (d % 4 == 0, d <= 256) is held by ONE
// 64-lane wavefront, lane l owning columns [4l, 4l+4) as a float4 (lanes with
// 4l >= d hold zeros).  Row norms are wave reductions.  All arithmetic is fp32,
// matching the reference (hyperbolic_src/hyperbolic_ops.py) to ~1 ulp per op.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define REGCN_EPS 1e-6f
#define WAVE 64

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

namespace regcn {

// Curvature-derived constants, computed on the host in double and rounded
// once to fp32 exactly as torch rounds a python-float clamp bound.
struct Curv {
  float c;        // curvature
  float sqrt_c;   // sqrt(c)
  float mx;       // project bound: 1/sqrt(c) - 2e-6  (hyperbolic_ops.py:73 + :52)
  float rmax;     // apply_radius bound: 1/sqrt(c) - 1e-6 (hyperbolic_ops.py:229)
  float atanh_mx; // log0 clamp: 1 - 1e-6 (hyperbolic_ops.py:115)
};

// Sum over each DPP row of 16 lanes, result in every lane of the row: two quad_perm
// swaps and two row rotations (VALU DPP; no LDS crossbar like ds_bpermute/__shfl).
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false)); // row_ror:4
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false)); // row_ror:8
  return v;
}

__device__ __forceinline__ float rlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Full 64-lane sum, broadcast (wave-uniform) to every lane.
__device__ __forceinline__ float wave_sum(float v) {
  v = row16_sum(v);
  return (rlane(v, 0) + rlane(v, 16)) + (rlane(v, 32) + rlane(v, 48));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// Reduction over the 16 lanes that share (lane >> 4): the row group of an
// MFMA 16x16 C/D fragment (col = lane & 15).
__device__ __forceinline__ float group16_sum(float v) { return row16_sum(v); }

__device__ __forceinline__ float dot4(f4 a, f4 b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}

// clamp(x, lo, hi) as one v_med3_f32 (fminf(fmaxf()) adds a NaN-quieting v_max per element;
// the same value for every non-NaN x)
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
__device__ __forceinline__ f4 clamp4(f4 v, float lo, float hi) {
  return f4{clampf(v.x, lo, hi), clampf(v.y, lo, hi), clampf(v.z, lo, hi), clampf(v.w, lo, hi)};
}

// F.rrelu(x) with training=False: slope (1/8 + 1/3) / 2 = 11/48.  For 0 < slope < 1 it is
// max(x, slope x) = med3(x, slope x, +inf): two VALU, no compare / select, the same bits as
// x >= 0 ? x : slope x.  Written as the instruction itself: the compiler folds the builtin into
// maxnum(x, slope x) and, not knowing x canonical, quiets it first (v_max x, x): three VALU.
#ifndef REGCN_LEAKY_ASM
#define REGCN_LEAKY_ASM 1
#endif
__device__ __forceinline__ float leaky(float x) {
  const float slope = (1.0f / 8.0f + 1.0f / 3.0f) * 0.5f;
#if REGCN_LEAKY_ASM
  float r;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(x * slope), "s"(__builtin_inff()));
  return r;
#else
  return __builtin_amdgcn_fmed3f(x, x * slope, __builtin_inff());
#endif
}

__device__ __forceinline__ f4 leaky4(f4 v) { return f4{leaky(v.x), leaky(v.y), leaky(v.z), leaky(v.w)}; }

// v_exp + v_rcp (<= 2 ulp): the IEEE expf and division cost ~30 VALU ops per element.
__device__ __forceinline__ float sigmoidf(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// ---- factor math in a few VALU --------------------------------------------------------------
// The row maps' per-row scalars (norms, tanh / atanh of them, their ratios) sit in the MFMA
// kernels' epilogues, and on gfx950 the fp32 MFMA and the VALU share the SIMD's issue (the two
// do not overlap: tools/probe/overlap_probe.hip), so every VALU instruction there
// costs time.  The IEEE sqrtf / division / tanhf / atanhf sequences are 18 / 12 / ~60 / ~130 VALU;
// these are 1 / 2 / ~16 / ~16 on the 1-ulp v_sqrt / v_rcp / v_exp / v_log instructions, within
// 6 ulp of the exact function (<= 3.5e-7 relative over the whole range, checked against float64
// in tests/test_fastmath.py's restatement), against the 1e-4 parity tolerance.
constexpr float FM_LOG2E = 1.4426950408889634f, FM_LN2 = 0.6931471805599453f;
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fdiv(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
// tanh(x), x >= 0: odd Taylor polynomial to x^9 below 0.25 (truncation < 1e-8 relative), else
// (1 - e) / (1 + e) with e = exp(-2x) <= 0.61 (no cancellation)
__device__ __forceinline__ float ftanh_pos(float x) {
  const float x2 = x * x;
  float p = fmaf(x2, 62.f / 2835.f, -17.f / 315.f);
  p = fmaf(x2, p, 2.f / 15.f);
  p = fmaf(x2, p, -1.f / 3.f);
  p = fmaf(x * x2, p, x);
  const float e = __builtin_amdgcn_exp2f(x * (-2.f * FM_LOG2E));
  const float q = (1.f - e) * frcp(1.f + e);
  return x < 0.25f ? p : q;
}
__device__ __forceinline__ float ftanh(float x) { return copysignf(ftanh_pos(fabsf(x)), x); }
// atanh(s), 0 <= s < 1: odd Taylor polynomial to s^11 below 0.25 (truncation < 5e-9 relative),
// else ln((1 + s) / (1 - s)) / 2 with the ratio >= 1.67
__device__ __forceinline__ float fatanh_pos(float s) {
  const float s2 = s * s;
  float p = fmaf(s2, 1.f / 11.f, 1.f / 9.f);
  p = fmaf(s2, p, 1.f / 7.f);
  p = fmaf(s2, p, 1.f / 5.f);
  p = fmaf(s2, p, 1.f / 3.f);
  p = fmaf(s * s2, p, s);
  const float q = (0.5f * FM_LN2) * __builtin_amdgcn_logf((1.f + s) * frcp(1.f - s));
  return s < 0.25f ? p : q;
}
// |row| from its squared norm, clamped (the stored radius, apply_radius's norm)
__device__ __forceinline__ float row_radius(float n2) { return fmaxf(fsqrt(n2), REGCN_EPS); }

// ---- scalar factors of the row maps, given the row's squared norm n2 ------------------

// log0: x * atanh(min(sqrt_c |x|, 1-eps)) / (sqrt_c |x|), |x| clamped to eps
// (hyperbolic_ops.py:97-116).
__device__ __forceinline__ float log0_factor(float n2, const Curv& k) {
  float n = row_radius(n2);
  float s = fminf(k.sqrt_c * n, k.atanh_mx);
  return fdiv(fatanh_pos(s), k.sqrt_c * n);
}

// project_to_ball factor (hyperbolic_ops.py:37-74): min(|x|c, mx)/|x|c, |x|c = max(|x|, eps).
__device__ __forceinline__ float project_factor(float n2, const Curv& k) {
  float n = row_radius(n2);
  return fdiv(fminf(n, k.mx), n);
}

// exp0 then project (hyperbolic_ops.py:76-95).  Returns the factor f with
// exp0(v) = f * v; *out_n2 receives |exp0(v)|^2 (analytic).
__device__ __forceinline__ float exp0_factor(float n2, const Curv& k, float* out_n2 = nullptr) {
  float rn = fsqrt(n2);
  float n = fmaxf(rn, REGCN_EPS);
  float t = ftanh_pos(k.sqrt_c * n);
  float f = fdiv(t, n * k.sqrt_c);
  float pn = f * rn;                 // |tanh(..) v / (n sqrt_c)|
  float pf = project_factor(pn * pn, k);
  if (out_n2) {
    float q = pn * pf;
    *out_n2 = q * q;
  }
  return f * pf;
}

// ---- wave-per-row maps on a float4 fragment ---------------------------------------------
__device__ __forceinline__ f4 row_log0(f4 v, const Curv& k) { return v * log0_factor(wave_sum(dot4(v, v)), k); }
__device__ __forceinline__ f4 row_exp0(f4 v, const Curv& k) { return v * exp0_factor(wave_sum(dot4(v, v)), k); }
__device__ __forceinline__ f4 row_project(f4 v, const Curv& k) { return v * project_factor(wave_sum(dot4(v, v)), k); }

// apply_radius (hyperbolic_ops.py:208-233): direction * clamp(r, eps, rmax).
__device__ __forceinline__ f4 row_apply_radius(f4 v, float r, const Curv& k) {
  float n = row_radius(wave_sum(dot4(v, v)));
  float rr = fminf(fmaxf(r, REGCN_EPS), k.rmax);
  return v * fdiv(rr, n);
}

__device__ __forceinline__ f4 load4(const float* p, int col, int d) {
  return col < d ? *reinterpret_cast<const f4*>(p + col) : f4{0.f, 0.f, 0.f, 0.f};
}

__device__ __forceinline__ void store4(float* p, int col, int d, f4 v) {
  if (col < d) *reinterpret_cast<f4*>(p + col) = v;
}

}  // namespace regcn
