// All-entity hyperbolic distance scoring on MFMA (f2).
//
// The reference expands every (query, candidate) pair and runs mobius_add(-q, e)
// per pair (hyperbolic_decoder.py:89-179).  With x = -q, y = e everything the
// distance needs is three scalars per pair:
//     xy = <q, e>   (the only d-length contraction: a GEMM Q E^T on MFMA)
//     x2 = |q|^2, y2 = |e|^2   (per-row, accumulated while the tiles are staged)
//   A = 1 - 2c xy + c y2,  B = 1 - c x2,  |num|^2 = A^2 x2 - 2AB xy + B^2 y2
//   den = 1 - 2c xy + c^2 x2 y2 (+eps);  |mobius| = min(|num| / den, mx)
//   proxy score  = scale (margin - |mobius|^2) + bias[n]
//   true distance (use_hyperbolic_distance): 2/sqrt_c atanh(sqrt_c |.|) with the
//   reference's clamps, optionally with a per-query curvature c_r (:145-164).
//
// Tile: 256 threads, 64 queries x 64 candidates; wave w computes 16 queries x 64
// candidates as four 16x16 v_mfma_f32_16x16x4_f32 accumulators; K streamed through
// LDS in 16-deep chunks.  Epilogues: write S (score), or per-tile (max, sum exp)
// partials + target logit for a fused cross entropy (never materialising B x N).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "regcn_internal.h"

namespace regcn {

constexpr int SQ = 64, SN = 64;
// K chunk: 16 * NF columns (NF float4 per staging thread and row), double-buffered in LDS
// with the next chunk's loads in flight.  Measured at B = 492, N = 7128, d = 200: 16-column
// chunks 29.6 us, 64-column chunks 41.7 us (fewer resident workgroups per CU).
template <bool F64>
struct Chunking {
  static constexpr int NF = 1;
  static constexpr int SKC = 16 * NF;
  static constexpr int SLD = SKC + 2;  // = 2 (mod 32): conflict-free fragment reads
};



template <typename T>
__device__ __forceinline__ T pair_score(T xy, T x2, T y2, T bias_n, T cr, const ScoreArgs& p) {
  const T eps = (T)REGCN_EPS;
  if (!p.use_dist) {
    const T c = (T)p.c;
    const T A = (T)1 - (T)2 * c * xy + c * y2;
    const T Bq = (T)1 - c * x2;
    const T num2 = fmax(A * A * x2 - (T)2 * A * Bq * xy + Bq * Bq * y2, (T)0);
    const T den = (T)1 - (T)2 * c * xy + c * c * x2 * y2 + eps;
    const T n = fmin(sqrt(num2) / den, (T)p.mx);
    return (T)p.scale * ((T)p.margin - n * n) + bias_n;
  }
  if (p.c_r) {  // hyperbolic_decoder.py:146-161
    const T c = cr;
    const T sc = sqrt(c + eps);
    const T A = (T)1 - (T)2 * c * xy + c * y2, Bq = (T)1 - c * x2;
    const T num2 = fmax(A * A * x2 - (T)2 * A * Bq * xy + Bq * Bq * y2, (T)0);
    const T den = (T)1 - (T)2 * c * xy + c * c * x2 * y2 + eps;
    T n = fmax(sqrt(num2) / den, eps);
    n = fmin(n, (T)1 / (sc + eps) - eps);
    const T dist = ((T)2 / (sc + eps)) * atanh(fmin(sc * n, (T)1 - eps));
    return (T)p.scale * ((T)p.margin - dist) + bias_n;
  }
  // HyperbolicOps.hyperbolic_distance (hyperbolic_ops.py:168-191): mobius_add projects
  // to |.| <= mx, then the norm is clamped to [eps, 1/(sqrt_c + eps) - eps].
  const T c = (T)p.c, sc = (T)p.sqrt_c;
  const T A = (T)1 - (T)2 * c * xy + c * y2, Bq = (T)1 - c * x2;
  const T num2 = fmax(A * A * x2 - (T)2 * A * Bq * xy + Bq * Bq * y2, (T)0);
  const T den = (T)1 - (T)2 * c * xy + c * c * x2 * y2 + eps;
  T n = fmin(sqrt(num2) / den, (T)p.mx);
  n = fmin(fmax(n, eps), (T)p.dist_mx);
  const T dist = ((T)2 / sc) * atanh(sc * n);
  return (T)p.scale * ((T)p.margin - dist) + bias_n;
}

typedef double d4 __attribute__((ext_vector_type(4)));

template <bool F64>
struct ScoreT;
template <>
struct ScoreT<false> {
  typedef float T;
  typedef f4 V;
  static __device__ __forceinline__ V mfma(T a, T b, V c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
  // C/D layout of v_mfma_f32_16x16x4_f32: row 4*(lane>>4) + r
  static __device__ __forceinline__ int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};
template <>
struct ScoreT<true> {
  typedef double T;
  typedef d4 V;
  static __device__ __forceinline__ V mfma(T a, T b, V c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
  // C/D layout of v_mfma_f64_16x16x4_f64: row (lane>>4) + 4 r
  static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};

// MODE 0 = write scores, 1 = CE partials.  F64: fp64 MFMA + fp64 epilogue, used for the
// true-distance mode where the arctanh distance is linear in |num| and the fp32 expansion
// would lose ~3 digits on near-duplicate pairs (the per-pair fp32 reference does not).
// Epilogue shared by the score kernels: lane holds queries qi[r] and candidates ni[j];
// MODE 0 writes the scores, MODE 1 the per-tile (max, sum exp) CE partials + target logit.
template <int MODE, typename T, typename V>
__device__ __forceinline__ void score_epilogue(const ScoreArgs& p, const V* acc, const T* x2, const T* y2,
                                               const T* bn_, const T* cr, const int* qi, const int* ni, int lane,
                                               int bn) {
  if (MODE == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (qi[r] >= p.B) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ni[j] < p.N)
          p.out[(int64_t)qi[r] * p.N + ni[j]] = (float)pair_score<T>(acc[j][r], x2[r], y2[j], bn_[j], cr[r], p);
    }
  } else {
    const int nblk = (p.N + SN - 1) / SN;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s[4], m = -INFINITY;
      const int t = qi[r] < p.B ? p.target[qi[r]] : -1;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j] = ni[j] < p.N ? (float)pair_score<T>(acc[j][r], x2[r], y2[j], bn_[j], cr[r], p) : -INFINITY;
        m = fmaxf(m, s[j]);
        if (ni[j] == t) p.tgt_logit[qi[r]] = s[j];
      }
      // reduce over the 16 lanes of this row group
      m = fmaxf(m, __shfl_xor(m, 1));
      m = fmaxf(m, __shfl_xor(m, 2));
      m = fmaxf(m, __shfl_xor(m, 4));
      m = fmaxf(m, __shfl_xor(m, 8));
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) se += ni[j] < p.N ? expf(s[j] - m) : 0.f;
      se = group16_sum(se);
      if ((lane & 15) == 0 && qi[r] < p.B) {
        float* o = p.part + ((int64_t)qi[r] * nblk + bn) * 2;
        o[0] = m;
        o[1] = se;
      }
    }
  }
}


template <int MODE, bool F64>
__global__ __launch_bounds__(256) void k_score(ScoreArgs p) {
  typedef ScoreT<F64> S;
  typedef typename S::T T;
  p.scale = p.scale_p ? *p.scale_p : 1.f;
  if (p.scale_raw && p.scale_p)  // softplus(raw) + 1e-6 (hyperbolic_decoder.py:717; torch threshold 20)
    p.scale = (p.scale > 20.f ? p.scale : log1pf(expf(p.scale))) + 1e-6f;
  p.margin = p.margin_p ? *p.margin_p : 0.f;
  constexpr int NF = Chunking<F64>::NF, SKC = Chunking<F64>::SKC, SLD = Chunking<F64>::SLD;
  __shared__ T Qs2[2][SQ * SLD];  // double-buffered K chunks
  __shared__ T Es2[2][SN * SLD];
  __shared__ T q2s[SQ], e2s[SN];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  auto stamp = [&](int k) {  // profiling (regcn_set_trace)
    if (p.trace && tid == 0) p.trace[(int64_t)blockIdx.x * 16 + k] = (int64_t)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // consecutive blocks share a query tile (the candidate stream is the large operand)
  const int nbn = (p.N + SN - 1) / SN;
  const int bq = blockIdx.x / nbn, bn = blockIdx.x - bq * nbn;
  const int q0 = bq * SQ, n0 = bn * SN;
  typename S::V acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = typename S::V{0, 0, 0, 0};
  const int i = tid >> 2, kq = (tid & 3) * 4;
  T sq_q = 0, sq_e = 0;  // row |.|^2, accumulated by the 4 staging threads of row i
  // Software pipeline: chunk c + 1 is loaded into registers (unconditional, clamped
  // addresses) while chunk c is multiplied out of the other LDS buffer.
  const float* qrow = p.q + (int64_t)min(q0 + i, p.B - 1) * p.d;
  const float* erow = p.e + (int64_t)min(n0 + i, p.N - 1) * p.d;
  const bool q_ok = q0 + i < p.B, e_ok = n0 + i < p.N;
  const f4 z4 = {0.f, 0.f, 0.f, 0.f};
  auto fetch = [&](int k0, f4* vq, f4* ve) {
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int k = k0 + kq + 16 * f;
      const int c = min(k, p.d - 4);
      // raw loads; the mask is applied at staging (a select here would wait for them)
      vq[f] = *reinterpret_cast<const f4*>(qrow + c);
      ve[f] = *reinterpret_cast<const f4*>(erow + c);
    }
  };
  // PF chunks of loads in flight (a ring of registers, slot = chunk % PF): one chunk of
  // MFMA work per wave (16 MFMAs) is far shorter than an L2/MALL round trip.
  constexpr int PF = 4;
  f4 vq[PF][NF], ve[PF][NF];
#pragma unroll
  for (int c = 0; c < PF; ++c) fetch(c * SKC, vq[c], ve[c]);
  // the chunk count is padded to a multiple of PF: a padded chunk stages zeros and skips
  // its MFMAs (kn <= 0), and the loop body has no exit branch, so every wait is counted
  // (a conditional exit makes hipcc drain vmcnt(0) before each chunk's staging)
  const int n_pad = ((p.d + SKC - 1) / SKC + PF - 1) / PF * PF;
  int buf = 0;
  for (int c0 = 0; c0 < n_pad; c0 += PF) {
#pragma unroll
    for (int sl = 0; sl < PF; ++sl) {
      const int c = c0 + sl;
      const int k0 = c * SKC;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        T* dq = Qs2[buf] + i * SLD + kq + 16 * f;
        T* de = Es2[buf] + i * SLD + kq + 16 * f;
        const bool k_ok = k0 + kq + 16 * f < p.d;
        const f4 va = (q_ok & k_ok) ? vq[sl][f] : z4, vb = (e_ok & k_ok) ? ve[sl][f] : z4;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const T a = (T)va[u], b = (T)vb[u];
          dq[u] = a;
          de[u] = b;
          sq_q += a * a;
          sq_e += b * b;
        }
      }
      fetch(k0 + PF * SKC, vq[sl], ve[sl]);  // unconditional (past the end: a clamped chunk
                                             // never stored); a conditional load would drain
      __syncthreads();  // chunk c staged; the other buffer's readers (chunk c - 1) are done
      const T* Qs = Qs2[buf];
      const T* Es = Es2[buf];
      const int kn = min(SKC, p.d - k0);
#pragma unroll
      for (int kk = 0; kk < SKC; kk += 4) {
        if (kk < kn) {  // wave-uniform: the last chunk stops at d (its tail is zero-staged)
          const T a = Qs[(16 * wv + (lane & 15)) * SLD + kk + (lane >> 4)];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const T b = Es[(16 * j + (lane & 15)) * SLD + kk + (lane >> 4)];
            acc[j] = S::mfma(a, b, acc[j]);
          }
        }
      }
      buf ^= 1;
    }
  }
  stamp(1);
  sq_q += __shfl_xor(sq_q, 1);
  sq_q += __shfl_xor(sq_q, 2);
  sq_e += __shfl_xor(sq_e, 1);
  sq_e += __shfl_xor(sq_e, 2);
  if ((tid & 3) == 0) {
    q2s[i] = sq_q;
    e2s[i] = sq_e;
  }
  __syncthreads();
  // epilogue: lane holds queries q0 + 16 wv + S::row(lane, r), candidates n0 + 16 j + (lane & 15)
  T x2[4], cr[4];
  int qi[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int li = 16 * wv + S::row(lane, r);
    qi[r] = q0 + li;
    const bool ok = qi[r] < p.B;
    x2[r] = q2s[li];
    cr[r] = (ok && p.c_r) ? (T)p.c_r[qi[r]] : (T)0;
  }
  T y2[4], bn_[4];
  int ni[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ni[j] = n0 + 16 * j + (lane & 15);
    const bool ok = ni[j] < p.N;
    y2[j] = e2s[16 * j + (lane & 15)];
    bn_[j] = (ok && p.bias) ? (T)p.bias[ni[j]] : (T)0;
  }
  score_epilogue<MODE, T>(p, acc, x2, y2, bn_, cr, qi, ni, lane, bn);
  stamp(2);
}

// ---- lean fp32 epilogue of the proxy score (k_score_f32; no arctanh distance) -------------
// S = scale (margin - n^2) + bias with n^2 = min(|num|^2 / den^2, mx^2): no square root, the
// per-query and per-candidate factors hoisted out of the 16 pairs a lane holds, one v_rcp per
// pair.  |num|^2 = A (A x2 - 2 Bq xy) + Bq^2 y2 with A = (1 + c y2) - 2c xy, Bq = 1 - c x2;
// den = (1 + eps + c^2 x2 y2) - 2c xy.
struct RowK {
  float x2, m2Bq, Bq2, c2x2;
  float sx2, sm2Bq, sBq2;  // the same times scale (pair_score_fast)
};
struct ColK {
  float y2, A0, sb;
  float lo;  // sb - scale mx^2: the score at the clamp
};

__device__ __forceinline__ RowK row_k(float x2, const ScoreArgs& p) {
  const float Bq = 1.f - p.c * x2;
  return RowK{x2, -2.f * Bq, Bq * Bq, p.c * p.c * x2, p.scale * x2, -2.f * p.scale * Bq, p.scale * (Bq * Bq)};
}
__device__ __forceinline__ ColK col_k(float y2, float bias, const ScoreArgs& p) {
  const float sb = p.scale * p.margin + bias;
  return ColK{y2, 1.f + p.c * y2, sb, fmaf(-p.scale, p.mx * p.mx, sb)};
}

// The proxy score of one pair in 11 VALU: S = sb - scale min(n2, mx^2) = med3(a, lo, sgn(scale) inf)
// with a = sb - (scale |num|^2 / den) / den -- scale folded into the row factors, the clamp as
// one med3 against the column's clamped score (max for scale >= 0, min below), |num|^2 not
// clamped at 0 (>= 0 but for rounding, which moves S by ~1e-7 scale).  sgn_inf: +inf or -inf by
// the sign of scale.  Every score, CE and count path uses it, so they agree bit for bit.
__device__ __forceinline__ float pair_score_fast(float xy, const RowK& r, const ColK& q, const ScoreArgs& p,
                                                 float sgn_inf) {
  const float m2c = -2.f * p.c;
  const float A = fmaf(m2c, xy, q.A0);
  const float t = fmaf(A, r.sx2, r.sm2Bq * xy);
  const float sn2 = fmaf(A, t, r.sBq2 * q.y2);
  const float den = fmaf(m2c, xy, fmaf(r.c2x2, q.y2, 1.f + REGCN_EPS));
  const float rd = __builtin_amdgcn_rcpf(den);
  return __builtin_amdgcn_fmed3f(fmaf(-(sn2 * rd), rd, q.sb), q.lo, sgn_inf);
}

// n^2 of one pair (clamped to mx^2), and optionally num2 / den for the gradient.
__device__ __forceinline__ float pair_n2(float xy, const RowK& r, const ColK& q, const ScoreArgs& p, float* num2_o,
                                         float* rden_o, float* A_o) {
  const float m2c = -2.f * p.c;
  const float A = fmaf(m2c, xy, q.A0);
  const float t = fmaf(A, r.x2, r.m2Bq * xy);
  const float num2 = fmaxf(fmaf(A, t, r.Bq2 * q.y2), 0.f);
  const float den = fmaf(m2c, xy, fmaf(r.c2x2, q.y2, 1.f + REGCN_EPS));
  const float rd = __builtin_amdgcn_rcpf(den);
  const float n2 = num2 * rd * rd;
  if (num2_o) {
    *num2_o = num2;
    *rden_o = rd;
    *A_o = A;
  }
  return fminf(n2, p.mx * p.mx);
}

__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false)));
  return v;
}

constexpr float LOG2E = 1.4426950408889634f;

// perm: the lane's J candidates are consecutive (ni[j] = ni[0] + j: score_f32_body stages
// candidate J i + j at tile row 16 j + i when N % J == 0), so a full tile's query row leaves as
// one J-float vector store per lane, not J scattered 4-B stores; otherwise ni[j] = ni[0] + 16 j
// (16 lanes store 64 contiguous bytes per instruction: with N % J != 0 the permuted order's
// scalar stores, 16 B apart per lane, cost the dataset decoders 3-14 %).
template <int MODE, int J>
__device__ __forceinline__ void score_epilogue_fast(const ScoreArgs& p, const f4* acc, const float* x2,
                                                    const float* y2, const float* bn_, const int* qi, const int* ni,
                                                    int lane, int bn, float* run_m, float* run_se,
                                                    bool full = false, bool perm = false) {
  RowK rk[4];
  ColK ck[J];
#pragma unroll
  for (int r = 0; r < 4; ++r) rk[r] = row_k(x2[r], p);
#pragma unroll
  for (int j = 0; j < J; ++j) ck[j] = col_k(y2[j], bn_[j], p);
  const float mx2 = p.mx * p.mx;
  const float sgn_inf = p.scale >= 0.f ? __builtin_inff() : -__builtin_inff();
  if (MODE == 0) {
    // the lane's candidates are ni[0] + j (perm) or ni[0] + 16 j (each valid one): one row
    // address per query row, the j steps as immediate store offsets
    const int64_t n0 = ni[0] < p.N ? ni[0] : 0;
    if (full) {  // every query row and candidate of the tile valid (wave-uniform): no store masks
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float* orow = p.out + (int64_t)qi[r] * p.N + n0;
        float sv[J];
#pragma unroll
        for (int j = 0; j < J; ++j) sv[j] = pair_score_fast(acc[j][r], rk[r], ck[j], p, sgn_inf);
        if (perm) {  // (uniform)
          if constexpr (J == 4) {
            *reinterpret_cast<f4*>(orow) = f4{sv[0], sv[1], sv[2], sv[3]};
          } else if constexpr (J == 2) {
            typedef float f2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<f2*>(orow) = f2{sv[0], sv[1]};
          } else {
#pragma unroll
            for (int j = 0; j < J; ++j) orow[j] = sv[j];
          }
        } else {
#pragma unroll
          for (int j = 0; j < J; ++j) orow[16 * j] = sv[j];
        }
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (qi[r] >= p.B) continue;
      float* orow = p.out + (int64_t)qi[r] * p.N + n0;
      if (perm) {
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (ni[j] < p.N) orow[j] = pair_score_fast(acc[j][r], rk[r], ck[j], p, sgn_inf);
      } else {
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (ni[j] < p.N) orow[16 * j] = pair_score_fast(acc[j][r], rk[r], ck[j], p, sgn_inf);
      }
    }
  } else if (MODE == 1) {  // this lane's running (max, sum exp) per query row, across tiles
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float sv[J], m = -INFINITY;
      const int t = qi[r] < p.B ? p.target[qi[r]] : -1;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        sv[j] = ni[j] < p.N ? pair_score_fast(acc[j][r], rk[r], ck[j], p, sgn_inf)
                            : -INFINITY;
        m = fmaxf(m, sv[j]);
        if (ni[j] == t) p.tgt_logit[qi[r]] = sv[j];
      }
      const float mn = fmaxf(run_m[r], m);
      const float ml = (mn == -INFINITY ? 0.f : mn) * LOG2E;  // exp2(-inf) = 0 for empty lanes
      float se = run_se[r] * __builtin_amdgcn_exp2f(fmaf(run_m[r], LOG2E, -ml));
#pragma unroll
      for (int j = 0; j < J; ++j) se += __builtin_amdgcn_exp2f(fmaf(sv[j], LOG2E, -ml));
      run_m[r] = mn;
      run_se[r] = se;
    }
  } else if (MODE == 3) {  // fused rank count: this lane's running #{S > thr} per query row
    // (the same S bits as MODE 0 writes, so the count equals k_rank's over the score matrix)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float t = qi[r] < p.B ? p.thr[qi[r]] : INFINITY;
      float cnt = 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j)
        if (ni[j] < p.N)
          cnt += pair_score_fast(acc[j][r], rk[r], ck[j], p, sgn_inf) > t ? 1.f : 0.f;
      run_se[r] += cnt;  // an exact integer (< 2^24 per lane)
    }
  } else {  // MODE 2: CE backward coefficients (8-wave workgroups only: J = 4, SN-candidate tiles)
    static_assert(MODE != 2 || J == 4, "the CE backward runs the 8-wave shape");
    const int nblk = (p.N + SN - 1) / SN;
    const float c = p.c, m2c = -2.f * c;
    float cs[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) cs[j][0] = cs[j][1] = cs[j][2] = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool qok = qi[r] < p.B;
      const int t = qok ? p.target[qi[r]] : -1;
      const float lsel = qok ? p.lse[qi[r]] * LOG2E : 0.f, gl = qok ? p.gl[qi[r]] : 0.f;
      const float X2 = rk[r].x2, Bq = 1.f - c * X2;
      float rs = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (!qok || ni[j] >= p.N) continue;
        const float xy = acc[j][r], Y2 = ck[j].y2;
        float num2, rd, A;
        const float n2 = pair_n2(xy, rk[r], ck[j], p, &num2, &rd, &A);
        const float S = pair_score_fast(xy, rk[r], ck[j], p, sgn_inf);  // the forward's bits
        const float G = gl * (__builtin_amdgcn_exp2f(fmaf(S, LOG2E, -lsel)) - (ni[j] == t ? 1.f : 0.f));
        float gxy = 0.f, gx2 = 0.f, gy2 = 0.f;
        if (num2 * rd * rd <= mx2) {  // not clamped: dn2/du = dnum2/du / den^2 - 2 num2 dden/du / den^3
          const float i2 = rd * rd, tt = 2.f * num2 * i2 * rd;
          gxy = (-4.f * c * A * X2 + 4.f * c * Bq * xy - 2.f * A * Bq) * i2 - tt * m2c;
          gx2 = (A * A + 2.f * c * A * xy - 2.f * c * Bq * Y2) * i2 - tt * (c * c * Y2);
          gy2 = (2.f * c * A * X2 - 2.f * c * Bq * xy + Bq * Bq) * i2 - tt * (c * c * X2);
        }
        const float Gs = -p.scale * G;
        p.coef[(int64_t)qi[r] * p.N + ni[j]] = Gs * gxy;
        rs += Gs * gx2;
        cs[j][0] += Gs * gy2;
        cs[j][1] += G;
        cs[j][2] += G * (p.margin - n2);
      }
      rs = group16_sum(rs);
      if ((lane & 15) == 0 && qok) p.rsum[(int64_t)qi[r] * nblk + bn] = rs;
    }
    const int grp = (qi[0] - 4 * (lane >> 4)) >> 4;  // this wave's 16-query group
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        float v = cs[j][k];
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        if (lane < 16 && ni[j] < p.N) p.csum[((int64_t)grp * p.N + ni[j]) * 3 + k] = v;
      }
  }
}

// fp32 scorer, persistent and double-buffered.  A workgroup = 8 waves = 128 queries; wave w
// owns queries [16w, 16w + 16), their rows in registers for the whole K.  The workgroup walks
// a strip of 64-candidate tiles: while tile i is multiplied out of one LDS buffer, tile i + 1
// is loaded into registers (issued before the MFMA loop, unconditionally) and written to the
// other buffer after the epilogue, behind the one barrier per tile.  k-block operand order:
// MFMA sub-step e of 16-deep block b reads k = 16 b + 4 (lane >> 4) + e, so a lane's operands
// for a block are one float4 (row stride = 8 mod 16: conflict-free ds_read_b128).
//
// Work order (XCD-aware): workgroups are dealt round-robin to the 8 XCDs; workgroup w sits on
// XCD x = w % 8, takes query tile (w / 8) % nbq and stripe k = w / (8 nbq), and walks the
// candidate tiles x + 8 (k + S i), S = stripes per XCD.  The nbq workgroups of one stripe walk
// the same tiles in step, so a tile comes from HBM into its XCD's L2 once.
constexpr int SQ2 = 128, SW2 = SQ2 / 16, KB_MAX = 16;  // d <= 256
#ifndef REGCN_SCORE_STAMPS
#define REGCN_SCORE_STAMPS 0
#endif
constexpr bool kScoreStamps = REGCN_SCORE_STAMPS != 0;  // diagnostic build: per-phase cycle sums
//
// Workgroup shape NW (waves): 8 = 128 queries x 64-candidate tiles, one workgroup per CU (its
// 111 KB of LDS); 4 = 64 queries x 32-candidate tiles at 56 KB, two workgroups per CU.  With 8
// waves the one barrier per tile keeps both waves of a SIMD in the same phase -- both multiply,
// then both run the epilogue while the matrix core idles; two 4-wave workgroups have no common
// barrier, so one's epilogue issues beside the other's MFMAs.  Queries per workgroup 16 NW,
// candidates per tile 8 NW (8 staging threads per candidate row), NW / 2 accumulators per wave.

__host__ __device__ inline int score_lds_stride(int d) { return ((d + 15) & ~15) + 8; }

// grid = 8 XCDs x query tiles x stripes (about one 8-wave workgroup, or two 4-wave ones, per CU
// when B is small); at most 32 stripes: the 8 x stripes partials of a query fit
// ce_partial_slots(N) (>= 256 and >= the candidate tiles)
template <int NW = 8>
inline int score_f32_stripes(int B, int nbn) {
  const int nbq = (B + 16 * NW - 1) / (16 * NW);
  return std::max(1, std::min(std::min(256 / NW / nbq, 32), (nbn + 7) / 8));
}
template <int NW = 8>
inline unsigned score_f32_grid(int B, int nbn) {
  return (unsigned)(8L * ((B + 16 * NW - 1) / (16 * NW)) * score_f32_stripes<NW>(B, nbn));
}
template <int NW = 8>
inline size_t score_f32_lds(int d) { return (size_t)2 * 8 * NW * (score_lds_stride(d) + 1) * 4; }
// REGCN_SCORE_NW: the workgroup shape of the proxy-score kernels (the CE backward keeps 8)
static int score_nw() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("REGCN_SCORE_NW");
    v = (e && atoi(e) == 4) ? 4 : 8;
  }
  return v;
}

// One workgroup's work: `blk` of `nblk` workgroups of this job (the XCD of blk is blk % 8:
// a job's first workgroup must sit at a multiple of 8 in the launch).
// KBT: the number of 16-deep k-blocks when known at compile time (13: 192 < d <= 208, every
// configuration's d = 200), so the query registers and staging loads are sized to it; 0 = any
// d <= 256.
template <int MODE, int NW, int KBT = 0>
__device__ __forceinline__ void score_f32_body(ScoreArgs p, const int blk, const int nblk) {
  constexpr int KBA = KBT ? KBT : KB_MAX;
  constexpr int SQW = 16 * NW, SNW = 8 * NW, J = SNW / 16;  // queries, candidates per tile; accumulators
  extern __shared__ float Es[];  // 2 x SNW x SE candidate rows, zero past N and d
  p.scale = p.scale_p ? *p.scale_p : 1.f;
  if (p.scale_raw && p.scale_p)  // softplus(raw) + 1e-6 (hyperbolic_decoder.py:717; torch threshold 20)
    p.scale = (p.scale > 20.f ? p.scale : log1pf(expf(p.scale))) + 1e-6f;
  p.margin = p.margin_p ? *p.margin_p : 0.f;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  auto stamp = [&](int k) {  // profiling (regcn_set_trace)
    if (p.trace && tid == 0) p.trace[(int64_t)blk * 16 + k] = (int64_t)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // with KBT known the row stride is a constant (16 KBT + 8 = score_lds_stride(d) for every d of
  // the bucket), so the B-fragment reads of a tile are immediate offsets of one address
  const int d = p.d, KB = KBT ? KBT : (d + 15) >> 4, SE = KBT ? 16 * KBT + 8 : score_lds_stride(d);
  if constexpr (KBT > 0) __builtin_assume(d > 16 * (KBT - 1) && d <= 16 * KBT);
  const int nbn = p.n_rng ? p.rng_total : (p.N + SNW - 1) / SNW, nbq = (p.B + SQW - 1) / SQW;
  // candidate tile t -> its first row and valid rows (row ranges: a tile never spans two)
  auto tile_rows = [&](int t, int& row0, int& nvalid) {
    if (!p.n_rng) {
      row0 = t * SNW;
      nvalid = min(SNW, p.N - row0);
      return;
    }
    // static indices only (a dynamic index would put the argument struct in scratch)
    int st = p.rng_start[0], tb = p.rng_tile[0], ln = p.rng_len[0];
#pragma unroll
    for (int r = 1; r < SCORE_MAX_RANGES; ++r)
      if (r < p.n_rng && t >= p.rng_tile[r]) st = p.rng_start[r], tb = p.rng_tile[r], ln = p.rng_len[r];
    const int off = (t - tb) * SNW;
    row0 = st + off;
    nvalid = min(SNW, ln - off);
  };
  const int S = nblk / (8 * nbq);
  const int xcd = blk & 7, rk = blk >> 3;
  // balanced grid (MODE 0, small candidate sets): workgroup blk takes query tile blk % nbq and
  // every p.bal-th candidate tile from blk / nbq, so the grid fills the CUs whatever nbq is;
  // striped grid: XCD-aware strips (see above)
  const bool bal = MODE == 0 && p.bal > 0;
  const int bq = bal ? blk % nbq : rk % nbq, stripe = rk / nbq, g0b = blk / nbq;
  auto tile_of = [&](int i) { return bal ? g0b + p.bal * i : xcd + 8 * (stripe + S * i); };
  int bn = tile_of(0);
  const int q0 = bq * SQW;
  const int g4 = 4 * (lane >> 4);
  // cross entropy: per-lane running (max, sum exp) over every tile of the strip, reduced over the
  // 16 lanes of each query row and written once, as partial xcd + 8 stripe of the query
  float run_m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY}, run_se[4] = {0.f, 0.f, 0.f, 0.f};
  auto count_flush = [&]() {  // MODE 3: the 16 lanes of a query row summed, partial xcd + 8 stripe
    const int np = 8 * S, pidx = xcd + 8 * stripe;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + 16 * wv + 4 * (lane >> 4) + r;
      const float cnt = row16_sum(run_se[r]);
      if ((lane & 15) == 0 && q < p.B) p.part[(int64_t)q * np + pidx] = cnt;
    }
  };
  auto ce_flush = [&]() {
    const int np = 8 * S, pidx = xcd + 8 * stripe;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + 16 * wv + 4 * (lane >> 4) + r;
      const float M = row16_max(run_m[r]);
      const float Ml = (M == -INFINITY ? 0.f : M) * LOG2E;
      const float se = row16_sum(run_se[r] * __builtin_amdgcn_exp2f(fmaf(run_m[r], LOG2E, -Ml)));
      if ((lane & 15) == 0 && q < p.B) {
        float* o = p.part + ((int64_t)q * np + pidx) * 2;
        o[0] = M;
        o[1] = se;
      }
    }
  };
  if (bn >= nbn) {  // no work for this stripe (whole workgroup, before any barrier)
    if (MODE == 1) ce_flush();
    if (MODE == 3) count_flush();
    return;
  }
  const f4 z4 = {0.f, 0.f, 0.f, 0.f};
  // this wave's query rows, all k-blocks (unconditional clamped loads; masked at use)
  const int qr = q0 + 16 * wv + (lane & 15);
  const bool q_ok = qr < p.B;
  const float* qrow = p.q + (int64_t)min(qr, p.B - 1) * d;
  // The last k-block is transposed in both operands (stash below): MFMA step e, lane group q
  // takes column 16 b + 4 e + q, so its steps past d hold pad columns only and are skipped
  // (d = 200: 50 k-steps per tile instead of 52).
  const int nlast = (d - 16 * (KB - 1) + 3) >> 2;
  f4 a[KBA - 1], alast;  // blocks 0 .. KB - 2; the last block, transposed
  float xs = 0.f;
#pragma unroll
  for (int b = 0; b < KBA - 1; ++b) {
    const f4 v = *reinterpret_cast<const f4*>(qrow + min(16 * b + g4, d - 4));
    a[b] = (q_ok & (b < KB - 1) & (16 * b + g4 < d)) ? v : z4;
    xs += dot4(a[b], a[b]);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int col = 16 * (KB - 1) + 4 * e + (lane >> 4);
    const float v = qrow[min(col, d - 1)];
    alast[e] = (q_ok & (col < d)) ? v : 0.f;
  }
  xs += dot4(alast, alast);
  // |q|^2 of query (lane & 15): sum the 4 k-quarters; the C rows of this lane
  xs += __shfl_xor(xs, 16);
  xs += __shfl_xor(xs, 32);
  float x2[4];
  int qi[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int li = 4 * (lane >> 4) + r;  // C row of this lane = query 16 wv + li
    x2[r] = __shfl(xs, li);
    qi[r] = q0 + 16 * wv + li;
  }
  // staging map: thread tid stages candidate row tid / 8, float4 units tid % 8 + 8 it
  static_assert(64 * NW == 8 * SNW, "staging map: 8 threads per candidate row");
  constexpr int IT = (KBA * 4 + 7) / 8;
  const int sr = tid >> 3, sub = tid & 7, per_row = 4 * KB;
  // perm: candidate sr of the tile sits at tile row 16 (sr % J) + sr / J, so accumulator j of
  // lane l holds candidate J (l & 15) + j: a lane's J candidates are consecutive (vector score
  // stores); otherwise at tile row sr (lane l, accumulator j: candidate 16 j + (l & 15))
  const bool perm = p.N % J == 0 && p.n_rng == 0;  // (uniform) see score_epilogue_fast
  const int trow = perm ? 16 * (sr % J) + sr / J : sr;
  f4 v[IT];
  auto fetch = [&](int t) {  // unconditional clamped loads (a conditional load drains vmcnt)
    int row0, nv;
    tile_rows(t, row0, nv);
    const float* erow = p.e + (int64_t)(row0 + min(sr, max(nv - 1, 0))) * d;
#pragma unroll
    for (int it = 0; it < IT; ++it) v[it] = *reinterpret_cast<const f4*>(erow + min((sub + 8 * it) * 4, d - 4));
  };
  // |e|^2 of each staged row, summed over its 8 staging lanes (xor 1, 2, 4), next to the tile
  float* e2s = Es + 2 * SNW * SE;  // [2][SNW]
  auto stash = [&](int buf) {
    // rows past the tile's valid rows hold a copy of its last row (fetch clamps): finite, and
    // their scores are never written or counted, so only the columns >= d need zeros
    float* lrow = Es + buf * SNW * SE + trow * SE;
    float ss = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int u = sub + 8 * it;
      const f4 w = (4 * u < d) ? v[it] : z4;
      ss += dot4(w, w);
      if (u < per_row) {
        if (u >= per_row - 4) {  // the transposed last block: column 16 b + 4 e + i at 4 i + e
          float* bl = lrow + (per_row - 4) * 4 + (u - (per_row - 4));
          bl[0] = w.x;
          bl[4] = w.y;
          bl[8] = w.z;
          bl[12] = w.w;
        } else {
          *reinterpret_cast<f4*>(lrow + 4 * u) = w;
        }
      }
    }
    ss += __shfl_xor(ss, 1);
    ss += __shfl_xor(ss, 2);
    ss += __shfl_xor(ss, 4);
    if (sub == 0) e2s[buf * SNW + trow] = ss;
  };
  // the per-candidate biases of a tile, loaded before its products (unconditional clamped loads,
  // as fetch): loaded in the epilogue they put a memory round trip (~0.5-1k cycles, both waves of
  // a SIMD at once) into every tile
  float bcur[J];
  auto load_bias = [&](int t, float (&b)[J]) {
    if (!p.bias) {  // (uniform)
#pragma unroll
      for (int j = 0; j < J; ++j) b[j] = 0.f;
      return;
    }
    int r0, nv;
    tile_rows(t, r0, nv);
#pragma unroll
    for (int j = 0; j < J; ++j) b[j] = p.bias[r0 + min(perm ? J * (lane & 15) + j : 16 * j + (lane & 15), max(nv - 1, 0))];
  };
  fetch(bn);
  stash(0);
  __syncthreads();
  stamp(1);
  // diagnostic build only (-DREGCN_SCORE_STAMPS=1, tools/scorebench.py --stamps): wave 0's
  // s_memtime cycles per tile phase, summed -- products, epilogue, staging, barrier
  int64_t ph[4] = {0, 0, 0, 0}, t_ph = kScoreStamps ? (int64_t)__builtin_amdgcn_s_memtime() : 0;
  auto phase = [&](int k) {
    if constexpr (kScoreStamps) {
      const int64_t t = (int64_t)__builtin_amdgcn_s_memtime();
      ph[k] += t - t_ph;
      t_ph = t;
    }
  };
  int cur = 0;
  for (int i = 0;; ++i) {
    const int bn_next = tile_of(i + 1);
    const bool more = bn_next < nbn;  // workgroup-uniform
    // next tile's rows in flight under this tile's MFMAs (MODE 2: after its epilogue, whose
    // live registers would otherwise spill)
    if (MODE != 2) fetch(min(bn_next, nbn - 1));
    load_bias(bn, bcur);
    const float* brow = Es + cur * SNW * SE + (lane & 15) * SE + g4;
    f4 acc[J];
#pragma unroll
    for (int j = 0; j < J; ++j) acc[j] = z4;
    // B fragments of block b + 1 are read while block b's MFMAs run (register double buffer;
    // the last block's into blast)
    f4 bb[2][J], blast[J];  // ping-pong by block parity (static after unrolling: no copies)
#pragma unroll
    for (int j = 0; j < J; ++j) bb[0][j] = *reinterpret_cast<const f4*>(brow + 16 * j * SE);
#pragma unroll
    for (int b = 0; b < KBA - 1; ++b) {
      if (b < KB - 1) {  // wave-uniform
        if (b + 1 < KB - 1) {
#pragma unroll
          for (int j = 0; j < J; ++j) bb[(b + 1) & 1][j] = *reinterpret_cast<const f4*>(brow + 16 * j * SE + 16 * (b + 1));
        } else {
#pragma unroll
          for (int j = 0; j < J; ++j) blast[j] = *reinterpret_cast<const f4*>(brow + 16 * j * SE + 16 * (b + 1));
        }
        __builtin_amdgcn_sched_barrier(0);  // keep block b + 1's reads ahead of block b's MFMAs
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < J; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[b][e], bb[b & 1][j][e], acc[j], 0, 0, 0);
      }
    }
    if (KB == 1) {
#pragma unroll
      for (int j = 0; j < J; ++j) blast[j] = bb[0][j];
    }
    // the last block: its k-steps holding columns < d only
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e > 0 && e >= nlast) break;  // wave-uniform
#pragma unroll
      for (int j = 0; j < J; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(alast[e], blast[j][e], acc[j], 0, 0, 0);
    }
    phase(0);
    float y2[J], bn_[J];
    int ni[J], row0, nv;
    tile_rows(bn, row0, nv);
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int c = perm ? J * (lane & 15) + j : 16 * j + (lane & 15);  // at tile row 16 j + (lane & 15)
      ni[j] = c < nv ? row0 + c : 0x7fffffff;  // invalid: >= N
      y2[j] = e2s[cur * SNW + 16 * j + (lane & 15)];
      bn_[j] = bcur[j];  // (an invalid candidate's bias is never used)
    }
    // (perm: every row start is aligned to J floats).  (Holding a full
    // tile's scores in registers and storing them after the tile's barrier, off the next stash's
    // vmcnt wait, was 7 % slower: profiles/r6_score_hold_ab.jsonl.)
    score_epilogue_fast<MODE, J>(p, acc, x2, y2, bn_, qi, ni, lane, bn, run_m, run_se,
                                 MODE == 0 && nv == SNW && q0 + SQW <= p.B, perm);
    phase(1);
    if (!more) break;
    if (MODE == 2) fetch(bn_next);
    stash(cur ^ 1);  // that buffer's readers passed the last barrier
    phase(2);
    __syncthreads();
    phase(3);
    cur ^= 1;
    bn = bn_next;
  }
  if (MODE == 1) ce_flush();
  if (MODE == 3) count_flush();
  stamp(2);
  if constexpr (kScoreStamps) {
    if (p.trace && tid == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) p.trace[(int64_t)blk * 16 + 4 + k] = ph[k];
    }
  }
}

// ---- 32 x 32 x 2 fp32 scorer (MODE 0 scores, MODE 3 fused rank count) ----------------------
// v_mfma_f32_32x32x2_f32: a wave owns 32 queries x a 64-candidate tile as two 32 x 32
// accumulators, so every B fragment read from LDS feeds a 32 x 32 block (twice the MACs of a
// 16 x 16 x 4 fragment) and the k loop issues half the LDS reads per flop.  K order: 8-deep
// block b, MFMA step e: lane half h = lane >> 5 carries k = 8 b + 4 h + e for both operands, so
// a lane's A operand of a block is one float4 of its query row (columns 8 b + 4 h ..) and its B
// operand one ds_read_b128 of its candidate row -- conflict-free with a row stride of 4 x odd
// floats (each 16-lane b128 group's rows are distinct mod 16).  d = 200 is 25 blocks (no
// padded k).  C layout: candidate 32 jb + (lane & 31), query (r & 3) + 8 (r >> 2) + 4 h.
// A workgroup = 8 waves = 256 queries; the strip walk, XCD order, candidate staging (8 threads
// per row, |e|^2 beside it) and one barrier per tile are k_score_f32's.  Scores and counts
// equal each other bit for bit (the same kernel computes both); they differ from the 16 x 16
// kernel's in the last bits (another k association).
constexpr int S32_QW = 32, S32_SQ = 8 * S32_QW, S32_SN = 64;
__host__ __device__ inline int score32_stride(int d) {
  int s = ((d + 7) & ~7) / 4;
  return 4 * (s | 1);
}
inline size_t score32_lds(int d) { return (size_t)2 * S32_SN * score32_stride(d) * 4; }
__device__ const f4 kZeroF4[1] = {{0.f, 0.f, 0.f, 0.f}};
inline int score32_stripes(int B, int nbn) {
  const int nbq = (B + S32_SQ - 1) / S32_SQ;
  return std::max(1, std::min(std::min(32 / nbq, 32), (nbn + 7) / 8));
}
inline unsigned score32_grid(int B, int nbn) {
  return (unsigned)(8L * ((B + S32_SQ - 1) / S32_SQ) * score32_stripes(B, nbn));
}
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float lanes32_sum(float v) {  // over the 32 lanes of a half-wave
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  v += __shfl_xor(v, 16);
  return v;
}

template <int MODE, int KBM>
__device__ __forceinline__ void score32_body(ScoreArgs p, const int blk, const int nblk) {
  static_assert(MODE == 0 || MODE == 3, "the 32 x 32 scorer writes scores or rank counts");
  extern __shared__ float Es[];  // 2 x S32_SN x SE candidate rows (zero past N and d)
  p.scale = p.scale_p ? *p.scale_p : 1.f;
  if (p.scale_raw && p.scale_p)  // softplus(raw) + 1e-6 (hyperbolic_decoder.py:717; torch threshold 20)
    p.scale = (p.scale > 20.f ? p.scale : log1pf(expf(p.scale))) + 1e-6f;
  p.margin = p.margin_p ? *p.margin_p : 0.f;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int d = p.d, KB = (d + 7) >> 3, SE = score32_stride(d), SE4 = SE >> 2;
  const int nbn = p.n_rng ? p.rng_total : (p.N + S32_SN - 1) / S32_SN, nbq = (p.B + S32_SQ - 1) / S32_SQ;
  auto tile_rows = [&](int t, int& row0, int& nvalid) {
    if (!p.n_rng) {
      row0 = t * S32_SN;
      nvalid = min(S32_SN, p.N - row0);
      return;
    }
    int st = p.rng_start[0], tb = p.rng_tile[0], ln = p.rng_len[0];
#pragma unroll
    for (int r = 1; r < SCORE_MAX_RANGES; ++r)
      if (r < p.n_rng && t >= p.rng_tile[r]) st = p.rng_start[r], tb = p.rng_tile[r], ln = p.rng_len[r];
    const int off = (t - tb) * S32_SN;
    row0 = st + off;
    nvalid = min(S32_SN, ln - off);
  };
  const int S = nblk / (8 * nbq);
  const int xcd = blk & 7, rk = blk >> 3;
  const int bq = rk % nbq, stripe = rk / nbq;
  auto tile_of = [&](int i) { return xcd + 8 * (stripe + S * i); };
  int bn = tile_of(0);
  const int q0 = bq * S32_SQ + S32_QW * wv;  // this wave's first query
  const int qrow_of_r0 = 4 * h;               // C row of register r: (r & 3) + 8 (r >> 2) + 4 h
  float run_c[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) run_c[r] = 0.f;
  auto count_flush = [&]() {  // MODE 3: a query row's 32 lanes summed, partial xcd + 8 stripe
    const int np = 8 * S, pidx = xcd + 8 * stripe;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = q0 + (r & 3) + 8 * (r >> 2) + qrow_of_r0;
      const float cnt = lanes32_sum(run_c[r]);
      if (l32 == 0 && q < p.B) p.part[(int64_t)q * np + pidx] = cnt;
    }
  };
  if (bn >= nbn) {  // no work for this stripe (whole workgroup, before any barrier)
    if (MODE == 3) count_flush();
    return;
  }
  const f4 z4 = {0.f, 0.f, 0.f, 0.f};
  // this wave's query rows: lane (l32, h) holds columns 8 b + 4 h .. + 3 of query q0 + l32
  const int qr = q0 + l32;
  const bool q_ok = qr < p.B;
  const float* qrow = p.q + (int64_t)min(qr, p.B - 1) * d;
  f4 a[KBM];
  float xs = 0.f;
#pragma unroll
  for (int b = 0; b < KBM; ++b) {
    const int c = 8 * b + 4 * h;
    const f4 v = *reinterpret_cast<const f4*>(qrow + min(c, d - 4));
    a[b] = (q_ok & (b < KB) & (c < d)) ? v : z4;
    xs += dot4(a[b], a[b]);
  }
  xs += __shfl_xor(xs, 32);  // |q|^2 of query q0 + l32 (both halves)
  // candidate tile staging by DMA (global_load_lds, 16 B per lane, no registers): the tile is
  // S32_SN x SE4 float4 pieces in row-major LDS order; wave-instruction j of wave w covers pieces
  // 64 (w + 8 j) + lane; pieces past column d or rows past the tile's end copy a zero row
  const float* zrow = reinterpret_cast<const float*>(kZeroF4);
  const int npieces = S32_SN * SE4, nins = (npieces + 511) / 512;
  auto dma = [&](int buf, int t) {
    int row0, nv;
    tile_rows(t, row0, nv);
    char* base = reinterpret_cast<char*>(Es + buf * S32_SN * SE);
    for (int j = 0; j < nins; ++j) {
      const int pc = 64 * (wv + 8 * j) + lane;
      const int r = pc / SE4, c4 = pc - r * SE4;
      const bool ok = (r < nv) & (4 * c4 < d);
      const float* src = ok ? p.e + (int64_t)(row0 + r) * d + 4 * c4 : zrow;
      if (64 * (wv + 8 * j) < npieces)  // wave-uniform
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(base + (size_t)64 * 16 * (wv + 8 * j)),
                                         16, 0, 0);
    }
  };
  dma(0, bn);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int cur = 0;
  for (int i = 0;; ++i) {
    const int bn_next = tile_of(i + 1);
    const bool more = bn_next < nbn;  // workgroup-uniform
    if (more) dma(cur ^ 1, bn_next);  // that buffer's readers passed the last barrier
    const float* brow = Es + cur * S32_SN * SE + l32 * SE + 4 * h;
    f16v acc[2];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[jb][r] = 0.f;
    float ss[2] = {0.f, 0.f};  // |e|^2 halves of the lane's two candidates, from the B fragments
    f4 bb[2][2];               // [block parity][jb]
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) bb[0][jb] = *reinterpret_cast<const f4*>(brow + 32 * jb * SE);
#pragma unroll
    for (int b = 0; b < KBM; ++b) {
      if (b < KB) {  // wave-uniform
        const int bnx = min(b + 1, KB - 1);
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) bb[(b + 1) & 1][jb] = *reinterpret_cast<const f4*>(brow + 32 * jb * SE + 8 * bnx);
        __builtin_amdgcn_sched_barrier(0);  // keep block b + 1's reads ahead of block b's MFMAs
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int jb = 0; jb < 2; ++jb)
            acc[jb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[b][e], bb[b & 1][jb][e], acc[jb], 0, 0, 0);
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) ss[jb] += dot4(bb[b & 1][jb], bb[b & 1][jb]);
      }
    }
    // epilogue: lane holds candidates row0 + 32 jb + l32, queries q0 + (r & 3) + 8 (r >> 2) + 4 h
    int row0, nv;
    tile_rows(bn, row0, nv);
    ColK ck[2];
    int ni[2];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
      const int li = 32 * jb + l32;
      ni[jb] = li < nv ? row0 + li : 0x7fffffff;  // invalid: >= N
      const float bias = (ni[jb] < p.N && p.bias) ? p.bias[ni[jb]] : 0.f;
      ck[jb] = col_k(ss[jb] + __shfl_xor(ss[jb], 32), bias, p);
    }
    const bool full = MODE == 0 && nv == S32_SN && bq * S32_SQ + S32_SQ <= p.B;  // workgroup-uniform
    const float sgn_inf = p.scale >= 0.f ? __builtin_inff() : -__builtin_inff();
    const int64_t n0 = ni[0] < p.N ? ni[0] : 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = (r & 3) + 8 * (r >> 2) + qrow_of_r0;
      const int q = q0 + qi;
      const RowK rkq = row_k(__shfl(xs, qi), p);
      if (MODE == 0) {
        float* orow = p.out + (int64_t)min(q, p.B - 1) * p.N + n0;
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
          const float sc = pair_score_fast(acc[jb][r], rkq, ck[jb], p, sgn_inf);
          if (full || (q < p.B && ni[jb] < p.N)) orow[32 * jb] = sc;
        }
      } else {
        const float t = q < p.B ? p.thr[q] : INFINITY;
        float cnt = 0.f;
#pragma unroll
        for (int jb = 0; jb < 2; ++jb)
          if (ni[jb] < p.N)
            cnt += pair_score_fast(acc[jb][r], rkq, ck[jb], p, sgn_inf) > t ? 1.f : 0.f;
        run_c[r] += cnt;  // an exact integer (< 2^24 per lane)
      }
    }
    if (!more) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's copies of the next tile have landed
    __syncthreads();                                    // ... and every wave's; this tile's readers are done
    cur ^= 1;
    bn = bn_next;
  }
  if (MODE == 3) count_flush();
}

template <int MODE, int KBM>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_score32(ScoreArgs p) {
  score32_body<MODE, KBM>(p, blockIdx.x, gridDim.x);
}

template <int KBM>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_score32_jobs(ScoreArgs p0, ScoreArgs p1,
                                                                                            int g0) {
  if ((int)blockIdx.x < g0) score32_body<0, KBM>(p0, blockIdx.x, g0);
  else score32_body<0, KBM>(p1, blockIdx.x - g0, gridDim.x - g0);
}

// The balanced grid for small candidate sets (MODE 0): the striped grid's 8 x nbq x stripes
// workgroups under-fill the chip when nbq does not divide 32 (ICEWS18: 25 query tiles -> 200
// workgroups, GDELT: 13 -> 208) and deals few tiles per workgroup unevenly; there the grid is
// nbq x bal with bal ~ 256 / nbq candidate-tile strides (one 8-wave workgroup per CU).  Large
// candidate sets (>= 64 tiles per strip: config 5) keep the XCD-aware strips.  REGCN_SCORE_BAL=0
// disables it.
static int score_bal_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("REGCN_SCORE_BAL");
    v = e ? atoi(e) : 1;
  }
  return v;
}
static int score_bal(int B, int nbn) {
  const int nbq = (B + SQ2 - 1) / SQ2;
  if (!score_bal_on() || nbn / (8 * score_f32_stripes(B, nbn)) >= 64) return 0;
  return std::max(1, std::min(nbn, 256 / nbq));
}

// REGCN_SCORE32=1 selects the 32 x 32 x 2 kernel for the scores and rank counts (opt-in: measured
// slower than the 16 x 16 x 4 kernel, 4.48 vs 4.33 ms at config 5 and 28 vs 26 us at the ICEWS14s
// decoder shape, profiles/r6_score32_ab.jsonl)
static bool score32_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("REGCN_SCORE32");
    v = e ? atoi(e) : 0;
  }
  return v != 0;
}

// Wave-specialised fp32 scorer: the same workgroup tile (128 queries, strips of 64-candidate
// tiles, XCD-aware order) with the roles split so the epilogue never holds the matrix core.
// Waves 0-3 (one per SIMD) are MFMA waves: wave w keeps queries [32w, 32w + 32) in registers
// (two 16-row A groups sharing every B fragment) and only multiplies, handing each tile's
// accumulators to LDS.  Waves 4-7 (the other wave of each SIMD) are epilogue waves: wave 4 + w
// reads MFMA wave w's accumulators, stages the next candidate tiles (global -> registers -> LDS)
// and runs the score / cross-entropy epilogue of tile i - 1 and its stores while the MFMA waves
// multiply tile i, so their VALU work and stores issue beside the MFMAs.  Two barriers per
// tile: B' (after MFMA block WS_MID: the previous accumulators have been read, the next tile
// may be staged) and B (tile i multiplied, its accumulators in LDS, tile i + 1 staged).
constexpr int WS_MID = 2;
__host__ __device__ inline size_t score_ws_exch_floats() { return (size_t)4 * 8 * 4 * 64; }  // waves x acc f4 x lanes
inline size_t score_ws_lds(int d) { return score_f32_lds(d) + score_ws_exch_floats() * 4; }

template <int MODE>
__device__ __forceinline__ void score_ws_body(ScoreArgs p, const int blk, const int nblk) {
  extern __shared__ float Es[];  // 2 x SN x SE candidate rows | 2 x SN |e|^2 | exchange
  p.scale = p.scale_p ? *p.scale_p : 1.f;
  if (p.scale_raw && p.scale_p) p.scale = (p.scale > 20.f ? p.scale : log1pf(expf(p.scale))) + 1e-6f;
  p.margin = p.margin_p ? *p.margin_p : 0.f;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool mfma_wave = wv < 4;  // wave-uniform role
  const int grpw = wv & 3;        // the 32-query group of this wave (MFMA wave and its epilogue wave)
  const int d = p.d, KB = (d + 15) >> 4, SE = score_lds_stride(d);
  const int nbn = p.n_rng ? p.rng_total : (p.N + SN - 1) / SN, nbq = (p.B + SQ2 - 1) / SQ2;
  // candidate tile t -> its first row and valid rows (row ranges: a tile never spans two)
  auto tile_rows = [&](int t, int& row0, int& nvalid) {
    if (!p.n_rng) {
      row0 = t * SN;
      nvalid = min(SN, p.N - row0);
      return;
    }
    // static indices only (a dynamic index would put the argument struct in scratch)
    int st = p.rng_start[0], tb = p.rng_tile[0], ln = p.rng_len[0];
#pragma unroll
    for (int r = 1; r < SCORE_MAX_RANGES; ++r)
      if (r < p.n_rng && t >= p.rng_tile[r]) st = p.rng_start[r], tb = p.rng_tile[r], ln = p.rng_len[r];
    const int off = (t - tb) * SN;
    row0 = st + off;
    nvalid = min(SN, ln - off);
  };
  const int S = nblk / (8 * nbq);
  const int xcd = blk & 7, rk = blk >> 3;
  const int bq = rk % nbq, stripe = rk / nbq;
  auto tile_of = [&](int i) { return xcd + 8 * (stripe + S * i); };
  const int q0 = bq * SQ2 + 32 * grpw;
  const int g4 = 4 * (lane >> 4);
  float* e2s = Es + 2 * SN * SE;
  f4* exch = reinterpret_cast<f4*>(Es + 2 * SN * SE + 2 * SN) + (size_t)grpw * 8 * 64;  // [8 acc][64 lanes]
  const f4 z4 = {0.f, 0.f, 0.f, 0.f};
  float run_m[2][4], run_se[2][4];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r) run_m[g][r] = -INFINITY, run_se[g][r] = 0.f;
  auto ce_flush = [&]() {  // epilogue waves: this wave's 32 queries, partial xcd + 8 stripe
    const int np = 8 * S, pidx = xcd + 8 * stripe;
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = q0 + 16 * g + 4 * (lane >> 4) + r;
        const float M = row16_max(run_m[g][r]);
        const float Ml = (M == -INFINITY ? 0.f : M) * LOG2E;
        const float se = row16_sum(run_se[g][r] * __builtin_amdgcn_exp2f(fmaf(run_m[g][r], LOG2E, -Ml)));
        if ((lane & 15) == 0 && q < p.B) {
          float* o = p.part + ((int64_t)q * np + pidx) * 2;
          o[0] = M;
          o[1] = se;
        }
      }
  };
  int bn = tile_of(0);
  if (bn >= nbn) {  // no work for this stripe (whole workgroup, before any barrier)
    if (MODE == 1 && !mfma_wave) ce_flush();
    return;
  }
  if (mfma_wave) {
    // ---------------------------------------------------------------- MFMA waves
    f4 a[2][KB_MAX];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int qr = q0 + 16 * g + (lane & 15);
      const bool q_ok = qr < p.B;
      const float* qrow = p.q + (int64_t)min(qr, p.B - 1) * d;
#pragma unroll
      for (int b = 0; b < KB_MAX; ++b) {
        const f4 v = *reinterpret_cast<const f4*>(qrow + min(16 * b + g4, d - 4));
        a[g][b] = (q_ok & (b < KB) & (16 * b + g4 < d)) ? v : z4;
      }
    }
    __syncthreads();  // P: tile 0 staged
    int cur = 0;
    for (int i = 0;; ++i) {
      const bool more = tile_of(i + 1) < nbn;
      const float* brow = Es + cur * SN * SE + (lane & 15) * SE + g4;
      f4 acc[2][4] = {{z4, z4, z4, z4}, {z4, z4, z4, z4}};
      f4 bb[2][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bb[0][j] = *reinterpret_cast<const f4*>(brow + 16 * j * SE);
#pragma unroll
      for (int b = 0; b < KB_MAX; ++b) {
        if (b < KB) {  // wave-uniform
          const int bnx = min(b + 1, KB - 1);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            bb[(b + 1) & 1][j] = *reinterpret_cast<const f4*>(brow + 16 * j * SE + 16 * bnx);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int g = 0; g < 2; ++g)
                acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][b][e], bb[b & 1][j][e], acc[g][j], 0, 0, 0);
        }
        if (b == min(WS_MID, KB - 1)) __syncthreads();  // B': the previous accumulators were read
      }
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) exch[(g * 4 + j) * 64 + lane] = acc[g][j];
      __syncthreads();  // B: accumulators in LDS, next tile staged
      if (!more) break;
      cur ^= 1;
    }
    return;
  }
  // ------------------------------------------------------------------ epilogue waves
  const int et = tid - 256;  // 0..255
  // |q|^2 of this lane's C rows (queries q0 + 16 g + 4 (lane >> 4) + r)
  float x2[2][4];
  int qi[2][4];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int qr = q0 + 16 * g + (lane & 15);
    const bool q_ok = qr < p.B;
    const float* qrow = p.q + (int64_t)min(qr, p.B - 1) * d;
    float xs = 0.f;
    for (int b = 0; b < KB; ++b) {
      const f4 v = *reinterpret_cast<const f4*>(qrow + min(16 * b + g4, d - 4));
      const f4 w = (q_ok & (16 * b + g4 < d)) ? v : z4;
      xs += dot4(w, w);
    }
    xs += __shfl_xor(xs, 16);
    xs += __shfl_xor(xs, 32);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int li = 4 * (lane >> 4) + r;
      x2[g][r] = __shfl(xs, li);
      qi[g][r] = q0 + 16 * g + li;
    }
  }
  // staging map: 4 epilogue threads per candidate row, float4 units sub + 4 it
  constexpr int IT = KB_MAX;
  const int sr = et >> 2, sub = et & 3, per_row = 4 * KB;
  f4 v[IT];
  auto fetch = [&](int t) {
    int row0, nv;
    tile_rows(t, row0, nv);
    const float* erow = p.e + (int64_t)(row0 + min(sr, max(nv - 1, 0))) * d;
#pragma unroll
    for (int it = 0; it < IT; ++it)
      if (it < KB) v[it] = *reinterpret_cast<const f4*>(erow + min((sub + 4 * it) * 4, d - 4));
  };
  auto stash = [&](int buf, int t) {
    int row0, nv;
    tile_rows(t, row0, nv);
    const bool row_ok = sr < nv;
    float* lrow = Es + buf * SN * SE + sr * SE;
    float ss = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      if (it < KB) {
        const int u = sub + 4 * it;
        const f4 w = (row_ok & (4 * u < d)) ? v[it] : z4;
        ss += dot4(w, w);
        if (u < per_row) *reinterpret_cast<f4*>(lrow + 4 * u) = w;
      }
    }
    ss += __shfl_xor(ss, 1);
    ss += __shfl_xor(ss, 2);
    if (sub == 0) e2s[buf * SN + sr] = ss;
  };
  fetch(bn);
  stash(0, bn);
  if (tile_of(1) < nbn) fetch(tile_of(1));
  __syncthreads();  // P
  int cur = 0;
  // tile i - 1's accumulators and candidate factors, read right after B(i - 1) (its LDS buffer
  // is restaged with tile i + 1 after B'(i))
  f4 acc[2][4];
  float y2[4], bn_[4];
  int ni[4], prev_bn = -1;
  auto take = [&](int tb, int buf) {
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[g][j] = exch[(g * 4 + j) * 64 + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ni[j] = tb * SN + 16 * j + (lane & 15);
      y2[j] = e2s[buf * SN + 16 * j + (lane & 15)];
      bn_[j] = (ni[j] < p.N && p.bias) ? p.bias[ni[j]] : 0.f;
    }
    prev_bn = tb;
  };
  auto epilogue = [&]() {
#pragma unroll
    for (int g = 0; g < 2; ++g)
      score_epilogue_fast<MODE, 4>(p, acc[g], x2[g], y2, bn_, qi[g], ni, lane, prev_bn, run_m[g], run_se[g]);
  };
  for (int i = 0;; ++i) {
    const int bn_next = tile_of(i + 1), bn_next2 = tile_of(i + 2);
    const bool more = bn_next < nbn;
    __syncthreads();  // B'
    if (more) {
      stash(cur ^ 1, bn_next);  // tile i - 1's buffer: read by the MFMA waves before B(i - 1)
      if (MODE != 2 && bn_next2 < nbn) fetch(bn_next2);
    }
    if (prev_bn >= 0) epilogue();  // tile i - 1
    if (MODE == 2 && more && bn_next2 < nbn) fetch(bn_next2);
    __syncthreads();  // B: tile i's accumulators in LDS
    take(bn, cur);
    if (!more) break;
    cur ^= 1;
    bn = bn_next;
  }
  epilogue();
  if (MODE == 1) ce_flush();
}

template <int MODE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_score_ws(ScoreArgs p) {
  score_ws_body<MODE>(p, blockIdx.x, gridDim.x);
}

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_score_ws_jobs(ScoreArgs p0, ScoreArgs p1,
                                                                                             int g0) {
  if ((int)blockIdx.x < g0) score_ws_body<0>(p0, blockIdx.x, g0);
  else score_ws_body<0>(p1, blockIdx.x - g0, gridDim.x - g0);
}

template <int MODE, int NW = 8, int KBT = 0>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) void k_score_f32(ScoreArgs p) {
  score_f32_body<MODE, NW, KBT>(p, blockIdx.x, gridDim.x);
}
// the 8-wave kernel of mode M, specialised for 13 k-blocks when d allows
template <int M>
static auto score_f32_kernel(int d) {
  return (d + 15) / 16 == 13 ? k_score_f32<M, 8, 13> : k_score_f32<M, 8, 0>;
}

// Two independent score jobs in one launch (a predict's entity and relation scores): job 1's
// workgroups follow job 0's in dispatch order, so they take the CUs that job 0's shorter
// strips free instead of running as a second serial launch.
template <int NW, int KBT = 0>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) void k_score_f32_jobs(ScoreArgs p0,
                                                                                                     ScoreArgs p1,
                                                                                                     int g0) {
  if ((int)blockIdx.x < g0) score_f32_body<0, NW, KBT>(p0, blockIdx.x, g0);
  else score_f32_body<0, NW, KBT>(p1, blockIdx.x - g0, gridDim.x - g0);
}

// Combine per-tile (max, sumexp) into per-query loss = lse - target logit (one wave per query).
__global__ __launch_bounds__(256) void k_ce_combine(const float* __restrict__ part, const float* __restrict__ tgt,
                                                    int B, int nblk, float* __restrict__ loss,
                                                    float* __restrict__ lse_out) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* pb = part + (int64_t)b * nblk * 2;
  float m = -INFINITY;
  for (int i = lane; i < nblk; i += 64) m = fmaxf(m, pb[2 * i]);
  m = wave_max(m);
  float s = 0.f;
  for (int i = lane; i < nblk; i += 64) s += pb[2 * i + 1] * expf(pb[2 * i] - m);
  s = wave_sum(s);
  if (lane == 0) {
    const float lse = m + logf(s);
    loss[b] = lse - tgt[b];
    if (lse_out) lse_out[b] = lse;
  }
}

// Sum of the fused rank count's per-strip partial counts (exact integers held in fp32) into
// counts[b] (added to its value when `accumulate`: a candidate set scored in several ranges).
__global__ __launch_bounds__(256) void k_count_combine(const float* __restrict__ part, int B, int np, int accumulate,
                                                       int* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* pb = part + (int64_t)b * np;
  int s = 0;
  for (int i = lane; i < np; i += 64) s += (int)pb[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) counts[b] = (accumulate ? counts[b] : 0) + s;
}

// Rank of the target under a descending sort, as 1 + #{n : S[b,n] > S[b,t]} (raw)
// and the same count excluding the other true answers of the snapshot (time-aware
// filter, rgcn/utils.py:51-75 sets them to -1e7).  filt_ptr/filt_idx: CSR of the
// entities to exclude per query (target itself excluded by the host).
// One workgroup (4 waves) per query row: the row is a streaming read (N floats), so every
// thread keeps RANK_UNROLL 16-B loads in flight over the 16-B aligned body (a scalar head and
// tail around it: rows start anywhere when N % 4 != 0).  Integer counts, so any split is exact.
constexpr int RANK_THR = 256, RANK_UNROLL = 4;
__global__ __launch_bounds__(RANK_THR) void k_rank(const float* __restrict__ S, int B, int N, const int* __restrict__ target,
                                                   const float* __restrict__ ts_in, const int* __restrict__ filt_ptr,
                                                   const int* __restrict__ filt_idx, int add, int* __restrict__ rank_raw,
                                                   int* __restrict__ rank_filt) {
  __shared__ int red[2][RANK_THR / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x;
  const float* row = S + (int64_t)b * N;
  const float ts = ts_in ? ts_in[b] : row[target[b]];
  const int head = min(N, (int)((16 - (reinterpret_cast<uintptr_t>(row) & 15)) & 15) / 4);
  const int nb4 = (N - head) / 4;  // aligned 4-float groups
  const f4* body = reinterpret_cast<const f4*>(row + head);
  int cnt = 0;
  if (tid < head) cnt += row[tid] > ts;
  for (int i = head + 4 * nb4 + tid; i < N; i += RANK_THR) cnt += row[i] > ts;
  int i = tid;
  for (; i + (RANK_UNROLL - 1) * RANK_THR < nb4; i += RANK_UNROLL * RANK_THR) {
    f4 v[RANK_UNROLL];
#pragma unroll
    for (int u = 0; u < RANK_UNROLL; ++u) v[u] = __builtin_nontemporal_load(body + i + u * RANK_THR);
#pragma unroll
    for (int u = 0; u < RANK_UNROLL; ++u) cnt += (v[u].x > ts) + (v[u].y > ts) + (v[u].z > ts) + (v[u].w > ts);
  }
  for (; i < nb4; i += RANK_THR) {
    const f4 v = body[i];
    cnt += (v.x > ts) + (v.y > ts) + (v.z > ts) + (v.w > ts);
  }
  int f = 0;
  if (filt_ptr) {
    for (int j = filt_ptr[b] + tid; j < filt_ptr[b + 1]; j += RANK_THR) f += row[filt_idx[j]] > ts;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o);
    f += __shfl_xor(f, o);
  }
  if (lane == 0) red[0][w] = cnt, red[1][w] = f;
  __syncthreads();
  if (tid == 0) {
    int c = 0, ff = 0;
#pragma unroll
    for (int k = 0; k < RANK_THR / 64; ++k) c += red[0][k], ff += red[1][k];
    rank_raw[b] = c + add;
    if (rank_filt) rank_filt[b] = c - ff + add;
  }
}

// REGCN_SCORE_WS=1 selects the wave-specialised scorer (k_score_ws) for A/B measurement; the
// default is the uniform-wave k_score_f32 (config 5, 5 predicts: 4.15 ms vs 5.35 ms per call
// for k_score_ws_jobs, profiles/r4_score_ws_kernel_stats.csv).
constexpr size_t SCORE_LDS_MAX = 160 * 1024;  // gfx950 LDS per workgroup (d > 224 keeps k_score_f32)
static bool score_ws() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("REGCN_SCORE_WS");
    v = e ? atoi(e) : 0;
  }
  return v != 0;
}

int score(ScoreArgs& a, int mode, float* loss, hipStream_t st) {
  if (a.d <= 0 || (a.d & 3)) return set_error(REGCN_EINVAL, "score needs d %% 4 == 0");
  if (!a.q || !a.e) return set_error(REGCN_EINVAL, "null pointer");
  if (a.B == 0 || a.N == 0) return 0;
  a.trace = g_trace;
  const int nbq = (a.B + SQ - 1) / SQ, nbn = (a.N + SN - 1) / SN;
  const long blocks = (long)nbq * nbn;
  if (blocks > 0x7fffffffL) return set_error(REGCN_EINVAL, "score grid too large");
  dim3 g((unsigned)blocks), b(256);
  // fp32 proxy / distance scores (no per-query curvature, d <= 256): the barrier-free kernel
  const bool fast = !a.use_dist && a.d <= 16 * KB_MAX;
  const dim3 g2(score_f32_grid(a.B, nbn)), b2(64 * SW2);
  const size_t lds2 = score_f32_lds(a.d);
  const bool ws = fast && score_ws() && score_ws_lds(a.d) <= SCORE_LDS_MAX;
  const bool nw4 = fast && !ws && score_nw() == 4;
  const int nbn4 = (a.N + 31) / 32;
  const dim3 g4(score_f32_grid<4>(a.B, nbn4)), b4(256);
  const size_t lds4 = score_f32_lds<4>(a.d);
  if (mode == 0) {
    if (!a.out) return set_error(REGCN_EINVAL, "null output");
    if (fast && score32_on()) {
      const dim3 g32(score32_grid(a.B, (a.N + S32_SN - 1) / S32_SN));
      if ((a.d + 7) / 8 <= 25) hipLaunchKernelGGL((k_score32<0, 25>), g32, dim3(512), score32_lds(a.d), st, a);
      else hipLaunchKernelGGL((k_score32<0, 32>), g32, dim3(512), score32_lds(a.d), st, a);
      return check_launch("k_score32");
    }
    if (ws) hipLaunchKernelGGL((k_score_ws<0>), g2, dim3(512), score_ws_lds(a.d), st, a);
    else if (nw4) hipLaunchKernelGGL((k_score_f32<0, 4>), g4, b4, lds4, st, a);
    else if (fast) {
      a.bal = score_bal(a.B, nbn);
      const dim3 gb(a.bal ? (unsigned)(((a.B + SQ2 - 1) / SQ2) * a.bal) : g2.x);
      hipLaunchKernelGGL(score_f32_kernel<0>(a.d), gb, b2, lds2, st, a);
    }
    else if (a.use_dist) hipLaunchKernelGGL((k_score<0, true>), g, b, 0, st, a);
    else hipLaunchKernelGGL((k_score<0, false>), g, b, 0, st, a);
    return check_launch("k_score");
  }
  if (!a.target || !a.part || !a.tgt_logit || !loss) return set_error(REGCN_EINVAL, "CE needs target/workspace/loss");
  if (ws) hipLaunchKernelGGL((k_score_ws<1>), g2, dim3(512), score_ws_lds(a.d), st, a);
  else if (nw4) hipLaunchKernelGGL((k_score_f32<1, 4>), g4, b4, lds4, st, a);
  else if (fast) hipLaunchKernelGGL(score_f32_kernel<1>(a.d), g2, b2, lds2, st, a);
  else if (a.use_dist) hipLaunchKernelGGL((k_score<1, true>), g, b, 0, st, a);
  else hipLaunchKernelGGL((k_score<1, false>), g, b, 0, st, a);
  int rc = check_launch("k_score_ce");
  if (rc) return rc;
  const int nparts = nw4 ? 8 * score_f32_stripes<4>(a.B, nbn4)
                         : fast ? 8 * score_f32_stripes(a.B, nbn) : nbn;  // <= ce_partial_slots(N)
  hipLaunchKernelGGL(k_ce_combine, dim3((a.B + 3) / 4), b, 0, st, a.part, a.tgt_logit, a.B, nparts, loss, a.lse_out);
  return check_launch("k_ce_combine");
}

int score_jobs(ScoreArgs& a0, ScoreArgs& a1, hipStream_t st) {
  for (ScoreArgs* a : {&a0, &a1}) {
    if (a->d <= 0 || (a->d & 3) || a->d > 16 * KB_MAX) return set_error(REGCN_EINVAL, "score jobs need d %% 4 == 0, d <= 256");
    if (a->use_dist || a->c_r) return set_error(REGCN_ENOTSUP, "score jobs compute the proxy score only");
    if (a->B > 0 && a->N > 0 && (!a->q || !a->e || !a->out)) return set_error(REGCN_EINVAL, "null pointer");
    a->trace = g_trace;
  }
  if (a0.d != a1.d) return set_error(REGCN_EINVAL, "score jobs need one d");
  const bool e0 = a0.B > 0 && a0.N > 0, e1 = a1.B > 0 && a1.N > 0;
  if (!e0 || !e1) {
    if (e0) return score(a0, 0, nullptr, st);
    if (e1) return score(a1, 0, nullptr, st);
    return 0;
  }
  const unsigned g0 = score_f32_grid(a0.B, (a0.N + SN - 1) / SN), g1 = score_f32_grid(a1.B, (a1.N + SN - 1) / SN);
  if (score32_on()) {
    const unsigned h0 = score32_grid(a0.B, (a0.N + S32_SN - 1) / S32_SN);
    const unsigned h1 = score32_grid(a1.B, (a1.N + S32_SN - 1) / S32_SN);
    if ((a0.d + 7) / 8 <= 25) hipLaunchKernelGGL(k_score32_jobs<25>, dim3(h0 + h1), dim3(512), score32_lds(a0.d), st, a0, a1, (int)h0);
    else hipLaunchKernelGGL(k_score32_jobs<32>, dim3(h0 + h1), dim3(512), score32_lds(a0.d), st, a0, a1, (int)h0);
  } else if (score_ws() && score_ws_lds(a0.d) <= SCORE_LDS_MAX) {
    hipLaunchKernelGGL(k_score_ws_jobs, dim3(g0 + g1), dim3(512), score_ws_lds(a0.d), st, a0, a1, (int)g0);
  } else if (score_nw() == 4) {
    const unsigned h0 = score_f32_grid<4>(a0.B, (a0.N + 31) / 32), h1 = score_f32_grid<4>(a1.B, (a1.N + 31) / 32);
    hipLaunchKernelGGL(k_score_f32_jobs<4>, dim3(h0 + h1), dim3(256), score_f32_lds<4>(a0.d), st, a0, a1, (int)h0);
  } else {
    unsigned h[2];
    int j = 0;
    for (ScoreArgs* a : {&a0, &a1}) {
      const int nbn = (a->N + SN - 1) / SN;
      a->bal = score_bal(a->B, nbn);
      h[j++] = a->bal ? (unsigned)(((a->B + SQ2 - 1) / SQ2) * a->bal) : score_f32_grid(a->B, nbn);
    }
    auto kern = (a0.d + 15) / 16 == 13 ? k_score_f32_jobs<8, 13> : k_score_f32_jobs<8, 0>;
    hipLaunchKernelGGL(kern, dim3(h[0] + h[1]), dim3(64 * SW2), score_f32_lds(a0.d), st, a0, a1, (int)h[0]);
  }
  return check_launch("k_score_f32_jobs");
}

// CE backward coefficients (the B x N GEMM operand and the row / column partial sums; the
// caller finishes dq = coef E + 2 q rowsum, de = coef^T Q + 2 e colsum on the GEMM library).
int score_ce_bwd(ScoreArgs& a, hipStream_t st) {
  if (a.d <= 0 || (a.d & 3) || a.d > 16 * KB_MAX) return set_error(REGCN_ENOTSUP, "CE backward needs d %% 4 == 0, d <= 256");
  if (a.use_dist) return set_error(REGCN_ENOTSUP, "CE backward of the arctanh-distance score is not built");
  if (!a.q || !a.e || !a.target || !a.lse || !a.gl || !a.coef || !a.rsum || !a.csum)
    return set_error(REGCN_EINVAL, "null pointer");
  if (a.B == 0 || a.N == 0) return 0;
  a.trace = nullptr;
  const int nbn = (a.N + SN - 1) / SN;
  const dim3 g2(score_f32_grid(a.B, nbn)), b2(64 * SW2);
  const size_t lds2 = score_f32_lds(a.d);
  // (the uniform-wave kernel: the backward epilogue's registers beside the wave-specialised
  // kernel's two A groups would spill)
  hipLaunchKernelGGL(score_f32_kernel<2>(a.d), g2, b2, lds2, st, a);
  return check_launch("k_score_ce_bwd");
}

// Fused score + rank count (no B x N score matrix): counts[b] (+)= #{n : S[b,n] > thr[b]} with S
// the proxy score k_score_f32<0> would write, bit for bit.  workspace: >= B * 8 * stripes floats
// (regcn_hyp_ce_workspace_bytes(B, N) suffices).
int rank_fused(ScoreArgs& a, int accumulate, int* counts, hipStream_t st) {
  if (a.d <= 0 || (a.d & 3) || a.d > 16 * KB_MAX)
    return set_error(REGCN_ENOTSUP, "fused rank count needs d %% 4 == 0, d <= 256 (d=%d)", a.d);
  if (a.use_dist || a.c_r) return set_error(REGCN_ENOTSUP, "fused rank count computes the proxy score only");
  if (a.B < 0 || a.N < 0) return set_error(REGCN_EINVAL, "negative size");
  if (a.B > 0 && (!a.q || !a.thr || !counts || !a.part)) return set_error(REGCN_EINVAL, "null pointer");
  if (a.B > 0 && a.N > 0 && !a.e) return set_error(REGCN_EINVAL, "null candidates");
  if (a.B == 0) return 0;
  const bool s32 = score32_on();
  const int nw = score_nw(), snw = s32 ? S32_SN : 8 * nw;
  if (a.n_rng) {  // the ranges' candidate tiles at this shape's tile size (a tile never spans two)
    int tiles = 0;
    for (int r = 0; r < SCORE_MAX_RANGES && r < a.n_rng; ++r) {
      a.rng_tile[r] = tiles;
      tiles += (a.rng_len[r] + snw - 1) / snw;
    }
    a.rng_tile[a.n_rng] = tiles;
    a.rng_total = tiles;
  }
  const int nbn = a.n_rng ? a.rng_total : (a.N + snw - 1) / snw;
  if (nbn == 0) {  // nothing to count: counts stay (accumulate) or become 0
    if (!accumulate) {
      hipLaunchKernelGGL(k_count_combine, dim3((a.B + 3) / 4), dim3(256), 0, st, a.part, a.B, 0, 0, counts);
      return check_launch("k_count_combine");
    }
    return 0;
  }
  a.trace = g_trace;
  if (s32) {
    if ((a.d + 7) / 8 <= 25) hipLaunchKernelGGL((k_score32<3, 25>), dim3(score32_grid(a.B, nbn)), dim3(512), score32_lds(a.d), st, a);
    else hipLaunchKernelGGL((k_score32<3, 32>), dim3(score32_grid(a.B, nbn)), dim3(512), score32_lds(a.d), st, a);
  } else if (nw == 4) {
    hipLaunchKernelGGL((k_score_f32<3, 4>), dim3(score_f32_grid<4>(a.B, nbn)), dim3(256), score_f32_lds<4>(a.d), st, a);
  } else {
    hipLaunchKernelGGL(score_f32_kernel<3>(a.d), dim3(score_f32_grid(a.B, nbn)), dim3(64 * SW2), score_f32_lds(a.d), st, a);
  }
  const int rc = check_launch("k_score_f32<3>");
  if (rc) return rc;
  const int np = s32 ? 8 * score32_stripes(a.B, nbn)
                     : nw == 4 ? 8 * score_f32_stripes<4>(a.B, nbn) : 8 * score_f32_stripes(a.B, nbn);
  hipLaunchKernelGGL(k_count_combine, dim3((a.B + 3) / 4), dim3(256), 0, st, a.part, a.B, np, accumulate, counts);
  return check_launch("k_count_combine");
}

int rank(const float* S, int B, int N, const int* target, const float* ts, const int* filt_ptr, const int* filt_idx,
         int add, int* rank_raw, int* rank_filt, hipStream_t st) {
  if (!S || (!target && !ts) || !rank_raw) return set_error(REGCN_EINVAL, "null pointer");
  if (B == 0) return 0;
  hipLaunchKernelGGL(k_rank, dim3(B), dim3(RANK_THR), 0, st, S, B, N, target, ts, filt_ptr, filt_idx, add,
                     rank_raw, rank_filt);
  return check_launch("k_rank");
}

}  // namespace regcn
