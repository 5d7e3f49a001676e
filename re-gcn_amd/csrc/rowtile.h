// Row-tile MFMA building blocks shared by the fused row kernels (layer.hip, query.hip).
//
// A workgroup of NWAVE = 4 waves owns a tile of TM = 16 rows and all d <= 256 output
// columns; wave w owns TPW = 16 / NWAVE sixteen-column MFMA tiles.  (8 waves x 2 tiles was
// measured slower: at ~180 VGPRs one 8-wave workgroup fills a CU, so its barriers and
// serial phases no longer overlap with a second workgroup's.)  An A operand (16 x d) sits
// in LDS with a row stride `lda` = 2 (mod 32) floats, so the 16 rows x 4 k-offsets one
// MFMA step reads fall in distinct banks (tile_lda).  B operands are weights prepacked into MFMA
// fragment order (k_pack_weight, layer.hip):
//     Wp[s][jq][lane][e] = W[4s + lane/16][16(4jq + e) + lane%16]
// so at k-step s a wave reads one coalesced TPW-float vector per lane.
//
// MFMA: v_mfma_f32_16x16x4_f32.  C/D layout: lane l holds rows 4*(l>>4)+r (r = 0..3) and
// column 16j + (l & 15) of tile j; a row's 16 lanes are one DPP row (row16_sum).
#pragma once
#include "common.h"

// Waves per workgroup: 4 by default; a translation unit whose grids are small (query.hip)
// may define REGCN_ROWTILE_WAVES (8 or 16) before the include for shorter per-wave chains.
// The helpers live in an inline namespace per wave count, so units built with different
// counts never share a definition.
#ifndef REGCN_ROWTILE_WAVES
#define REGCN_ROWTILE_WAVES 4
#endif
#define REGCN_RT_CAT2(a, b) a##b
#define REGCN_RT_CAT(a, b) REGCN_RT_CAT2(a, b)

namespace regcn {
inline namespace REGCN_RT_CAT(rowtile_w, REGCN_ROWTILE_WAVES) {

constexpr int MAX_D = 256;
constexpr int TM = 16;         // rows per workgroup
constexpr int NWAVE = REGCN_ROWTILE_WAVES;
static_assert(NWAVE == 4 || NWAVE == 8 || NWAVE == 16, "row tiles split 16 column tiles over 4, 8 or 16 waves");
constexpr int TPW = 16 / NWAVE;  // 16-column MFMA tiles per wave
constexpr int NTHR = 64 * NWAVE;
constexpr int RING = 8;        // k-steps of B fragments in flight per wave
constexpr int RED_FLOATS = 4 * NWAVE * TM;  // RowRed scratch (2 buffers x 2 quantities)

typedef float bvec __attribute__((ext_vector_type(TPW)));

// LDS row stride for width d: the smallest multiple of 4 that is >= d + 1 (a Lorentz gather
// partial keeps its time coordinate in column d) with lda / 4 odd.  Rows stay 16-B aligned
// (ds_read/write_b128), and the 64 banks see no conflict in the MFMA A reads (16 rows x 4
// k-offsets: rows at i * lda mod 64 = 4 (i * lda/4 mod 16), distinct for lda/4 odd) nor in
// the C-layout tile reads/writes (4 rows x 16 columns: rows 4 * lda apart = 16 banks).
__host__ __device__ constexpr int tile_lda(int d) {
  return ((d + 4) & ~3) + ((((d + 4) >> 2) & 1) ? 0 : 4);
}

struct Frag {
  f4 t[TPW];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int j = 0; j < TPW; ++j) t[j] = f4{0.f, 0.f, 0.f, 0.f};
  }
};

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }  // scalar
__device__ __forceinline__ int frag_row(int r) { return 4 * ((threadIdx.x & 63) >> 4) + r; }
__device__ __forceinline__ int frag_col(int jl) { return 16 * (TPW * wave_id() + jl) + (threadIdx.x & 15); }

// Stage rows A[rows[i]] (i < n_valid; row-major, width d) into the LDS tile T; rows past
// n_valid are zero.  All loads are issued (clamped addresses) before the LDS stores.
template <bool CLAMP10>
__device__ __forceinline__ void stage_rows(float* T, int lda, const float* __restrict__ A, const int* rows, int d,
                                           int n_valid) {
  constexpr int IT = TM * (MAX_D / 4) / NTHR;
  const int q4 = d >> 2, n = TM * q4;
  f4 v[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = min((int)threadIdx.x + it * NTHR, n - 1);
    const int i = idx / q4, c = (idx - i * q4) * 4;
    v[it] = *reinterpret_cast<const f4*>(A + (int64_t)rows[i < n_valid ? i : 0] * d + c);
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = threadIdx.x + it * NTHR;
    if (idx >= n) break;
    const int i = idx / q4, c = (idx - i * q4) * 4;
    f4 x = v[it];
    if (CLAMP10) x = clamp4(x, -10.f, 10.f);
    if (i >= n_valid) x = f4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f4*>(T + i * lda + c) = x;  // 16-B aligned rows (tile_lda)
  }
}

// Global -> LDS row staging with no VGPR round trip (global_load_lds, 16 B per lane, LDS
// destination = wave-uniform row base + 16 B x lane): wave w issues rows w, w + NWAVE, ...;
// lanes past d / 4 idle.  Asynchronous: the loads land while the caller goes on (the fused
// layer issues the self-loop rows before its gather, whose first index wait retires them);
// hipcc drains them (vmcnt) before the next barrier.  Every row is a real row (callers pad
// `rows` with a valid row), so rows past the tile's count hold that row's values, not zeros.
__device__ __forceinline__ void stage_rows_async(float* T, int lda, const float* __restrict__ A, const int* rows,
                                                 int d) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = w; i < TM; i += NWAVE) {
    const float* src = A + (int64_t)rows[i] * d;
    if (lane < (d >> 2))
      __builtin_amdgcn_global_load_lds((const void*)(src + lane * 4),
                                       (__attribute__((address_space(3))) void*)(T + i * lda), 16, 0, 0);
  }
}

// nt: this wave's column tiles that hold output columns (wave-uniform); the rest of the
// packed weight is zero padding (d_out < 256), whose MFMAs are skipped.
__device__ __forceinline__ void mfma_tpw(Frag& acc, float a, bvec b, int nt = TPW) {
#pragma unroll
  for (int j = 0; j < TPW; ++j)
    if (j < nt) acc.t[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[j], acc.t[j], 0, 0, 0);
}

// column tiles of this wave below n_out output columns
__device__ __forceinline__ int wave_tiles(int n_out) {
  return min(TPW, max(0, (n_out - 16 * TPW * wave_id() + 15) >> 4));
}

// This wave's B fragments in the packed layout: k-step s lives at bsrc + s * B_STEP.
__device__ __forceinline__ const bvec* bsrc_of(const float* __restrict__ Wp) {
  const int tile0 = TPW * wave_id();
  return reinterpret_cast<const bvec*>(Wp + ((tile0 / 4) * 64 + (threadIdx.x & 63)) * 4 + (tile0 % 4));
}
constexpr int B_STEP = 4 * 64 * 4 / TPW;  // bvec elements per k-step of the packed matrix

// The first RING B fragments of a packed weight, loaded ahead of the A tile (they do not
// depend on it), so the MFMA chain starts without a load latency.
struct BRing {
  bvec ring[RING];
  __device__ __forceinline__ void load(const float* __restrict__ Wp, int d) {
    const bvec* bsrc = bsrc_of(Wp);
    const int S = d >> 2;
#pragma unroll
    for (int i = 0; i < RING; ++i) ring[i] = bsrc[(int64_t)min(i, S - 1) * B_STEP];
  }
};

// acc += T[16 x d] @ W (T in LDS, W packed with d_in = d), ring pre-filled by BRing::load.
// n_out: W's output columns (the MFMAs of column tiles past it are skipped).
__device__ __forceinline__ void mfma_tile_pf(Frag& acc, const float* T, int lda, const float* __restrict__ Wp, int d,
                                             BRing& br, int n_out = MAX_D) {
  const int lane = threadIdx.x & 63;
  const int nt = wave_tiles(n_out);
  const int S = d >> 2;
  const bvec* bsrc = bsrc_of(Wp);
  const float* arow = T + (lane & 15) * lda + (lane >> 4);
  bvec* ring = br.ring;
  // A operands ride in their own ring, RING k-steps ahead: an LDS read right before its
  // MFMA would expose the ds_read latency on every step (the sched barriers keep order).
  float aring[RING];
#pragma unroll
  for (int i = 0; i < RING; ++i) aring[i] = arow[4 * min(i, S - 1)];
  int s = 0;
  for (; s + RING <= S; s += RING) {
#pragma unroll
    for (int i = 0; i < RING; ++i) {
      mfma_tpw(acc, aring[i], ring[i], nt);
      __builtin_amdgcn_sched_barrier(0);
      const int nx = min(s + i + RING, S - 1);
      ring[i] = bsrc[(int64_t)nx * B_STEP];  // unconditional: hipcc can count it
      aring[i] = arow[4 * nx];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int i = 0; i < RING; ++i)
    if (s + i < S) mfma_tpw(acc, aring[i], ring[i], nt);
}

// acc += T[16 x d] @ W.  No barriers inside.
__device__ __forceinline__ void mfma_tile(Frag& acc, const float* T, int lda, const float* __restrict__ Wp, int d,
                                          int n_out = MAX_D) {
  BRing br;
  br.load(Wp, d);
  mfma_tile_pf(acc, T, lda, Wp, d, br, n_out);
}

// N independent GEMMs acc[n] += T[n] @ W[n] (same d) in one k-loop: N x TPW MFMA chains per
// k-step, so each ring of R B fragments covers N times the latency one GEMM's ring does
// (the weights of a small grid come from HBM, not a warm L2).
template <int N, int R>
__device__ __forceinline__ void mfma_tiles(Frag* acc, const float* const* T, const float* const* W, int lda, int d,
                                           int n_out = MAX_D) {
  const int lane = threadIdx.x & 63;
  const int nt = wave_tiles(n_out);
  const int S = d >> 2;
  const bvec* bsrc[N];
  const float* arow[N];
  bvec ring[N][R];
  float aring[N][R];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    bsrc[n] = bsrc_of(W[n]);
    arow[n] = T[n] + (lane & 15) * lda + (lane >> 4);
  }
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int n = 0; n < N; ++n) {
      ring[n][i] = bsrc[n][(int64_t)min(i, S - 1) * B_STEP];
      aring[n][i] = arow[n][4 * min(i, S - 1)];
    }
  int s = 0;
  for (; s + R <= S; s += R) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
#pragma unroll
      for (int n = 0; n < N; ++n) mfma_tpw(acc[n], aring[n][i], ring[n][i], nt);
      __builtin_amdgcn_sched_barrier(0);
      const int nx = min(s + i + R, S - 1);
#pragma unroll
      for (int n = 0; n < N; ++n) {
        ring[n][i] = bsrc[n][(int64_t)nx * B_STEP];
        aring[n][i] = arow[n][4 * nx];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i)
    if (s + i < S) {
#pragma unroll
      for (int n = 0; n < N; ++n) mfma_tpw(acc[n], aring[n][i], ring[n][i], nt);
    }
}

// Cross-wave row reductions: per-wave partials -> LDS red[buf][wave][row] -> sum in wave
// order (deterministic).  Two buffers alternate so one barrier per reduction suffices.
struct RowRed {
  float* red;  // LDS, RED_FLOATS: 2 buffers x (2 quantities x NWAVE x TM)
  int buf;
  __device__ __forceinline__ static float sum_waves(const float* b, int i) {  // pairwise tree
    float v[NWAVE];
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) v[w] = b[w * TM + i];
#pragma unroll
    for (int h = 1; h < NWAVE; h *= 2)
#pragma unroll
      for (int w = 0; w + h < NWAVE; w += 2 * h) v[w] += v[w + h];
    return v[0];
  }
  __device__ __forceinline__ void allreduce(float part[4]) {
    const int lane = threadIdx.x & 63, w = wave_id();
    float* b = red + buf * 2 * NWAVE * TM;
#pragma unroll
    for (int r = 0; r < 4; ++r) part[r] = row16_sum(part[r]);
    if ((lane & 15) == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) b[w * TM + frag_row(r)] = part[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) part[r] = sum_waves(b, frag_row(r));
    buf ^= 1;
  }
  // two independent per-row sums in one barrier (uses both halves of the buffer pair)
  __device__ __forceinline__ void allreduce2(float pa[4], float pb[4]) {
    const int lane = threadIdx.x & 63, w = wave_id();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pa[r] = row16_sum(pa[r]);
      pb[r] = row16_sum(pb[r]);
    }
    float* ba = red + buf * 2 * NWAVE * TM;
    float* bb = ba + NWAVE * TM;
    if ((lane & 15) == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ba[w * TM + frag_row(r)] = pa[r];
        bb[w * TM + frag_row(r)] = pb[r];
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pa[r] = sum_waves(ba, frag_row(r));
      pb[r] = sum_waves(bb, frag_row(r));
    }
    buf ^= 1;
  }
  __device__ __forceinline__ void sumsq(const Frag& a, float out[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < TPW; ++j) s += a.t[j][r] * a.t[j][r];
      out[r] = s;
    }
    allreduce(out);
  }
};

// ---- row maps with the row norms carried along ------------------------------------------
// A row map scales each row by a factor of its norm, so the norm after the map follows
// analytically (|f x| = f |x|): chains of maps need one cross-wave reduction, not one per
// map.  n2[r] is |row|^2 of fragment row r, updated in place.
__device__ __forceinline__ void row_scale(Frag& a, const float f[4]) {
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) a.t[j][r] *= f[r];
}

__device__ __forceinline__ void scale_known(Frag& a, float n2[4], const float f[4]) {
  row_scale(a, f);
#pragma unroll
  for (int r = 0; r < 4; ++r) n2[r] *= f[r] * f[r];
}

// Per-row scalars are uniform over a row's 16 lanes, and lane l holds rows 4(l>>4) + r,
// r = 0..3.  Rather than evaluating a factor (sqrt, tanh, atanh, divisions: ~100 VALU
// instructions) for all four rows in every lane, lane l evaluates it once, for its own row
// r = l & 3 (own_row), and each lane then takes row r's result from lane r of its DPP row
// (row_newbcast, one VALU op): a quarter of the transcendental work, bit-identical values.
__device__ __forceinline__ float own_row(const float v[4]) {
  // a two-level select tree (a select chain on r == k is turned into a scratch array; in the
  // step tail's radius residual, once the vectoriser pairs v's elements, this tree becomes one
  // too -- a 32-B scratch round trip there; a bit-mask select (v_bfi_b32) avoided it but made
  // the first-layer tail ~1 % slower and the step tail no faster: profiles/r6_bias_own_row_ab.jsonl)
  const bool b0 = threadIdx.x & 1, b1 = threadIdx.x & 2;
  const float lo = b0 ? v[1] : v[0], hi = b0 ? v[3] : v[2];
  return b1 ? hi : lo;
}
template <int L>
__device__ __forceinline__ float row_bcast(float v) {  // lane L of each 16-lane DPP row
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + L, 0xF, 0xF, false));
}
__device__ __forceinline__ void spread_rows(float y, float out[4]) {
  out[0] = row_bcast<0>(y);
  out[1] = row_bcast<1>(y);
  out[2] = row_bcast<2>(y);
  out[3] = row_bcast<3>(y);
}

__device__ __forceinline__ void project_known(Frag& a, float n2[4], const Curv& k) {
  float f[4];
  spread_rows(project_factor(own_row(n2), k), f);
  scale_known(a, n2, f);
}

__device__ __forceinline__ void log0_known(Frag& a, float n2[4], const Curv& k) {
  float f[4];
  spread_rows(log0_factor(own_row(n2), k), f);
  scale_known(a, n2, f);
}

__device__ __forceinline__ void exp0_known(Frag& a, float n2[4], const Curv& k) {  // exp0 + project
  float f[4], o;
  spread_rows(exp0_factor(own_row(n2), k, &o), f);
  row_scale(a, f);
  spread_rows(o, n2);
}

__device__ __forceinline__ void normalize_known(Frag& a, float n2[4]) {  // F.normalize, eps 1e-12
  float f[4];
  spread_rows(frcp(fmaxf(fsqrt(own_row(n2)), 1e-12f)), f);
  scale_known(a, n2, f);
}

__device__ __forceinline__ void frag_exp0(RowRed& rr, Frag& a, const Curv& k) {
  float n2[4];
  rr.sumsq(a, n2);
  exp0_known(a, n2, k);
}

// Fragment of a row-major matrix (width d) for the tile's rows: unconditional loads from
// clamped addresses, then a select (no per-load branch, so no vmcnt(0) per load).
__device__ __forceinline__ void frag_load(Frag& a, const float* __restrict__ M, const int* rows, int n_valid, int d) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = frag_row(r);
    const bool ok = i < n_valid;
    const int64_t base = (int64_t)rows[ok ? i : 0] * d;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int col = frag_col(j);
      const float v = M[base + min(col, d - 1)];
      a.t[j][r] = (ok & (col < d)) ? v : 0.f;  // no short circuit: it would branch around the load (vmcnt(0) each)
    }
  }
}

// Per-column vector (bias / weight row) in the fragment's column order.
__device__ __forceinline__ void col_load(float out[TPW], const float* __restrict__ v, int d) {
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int col = frag_col(j);
    const float x = v[min(col, d - 1)];
    out[j] = col < d ? x : 0.f;
  }
}

// C-layout fragment read from an LDS tile (columns >= d read as 0).
__device__ __forceinline__ void frag_from_tile(Frag& a, const float* T, int lda, int d) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float* row = T + frag_row(r) * lda;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int col = frag_col(j);
      const float v = row[min(col, lda - 1)];
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
    for (int j = 0; j < TPW; ++j) {
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
      if (i < n_valid) rad[rows[i]] = row_radius(n2[r]);
    }
  }
}

}  // namespace rowtile_w<N>
}  // namespace regcn
