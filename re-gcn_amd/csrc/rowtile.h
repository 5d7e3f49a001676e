// Row-tile MFMA building blocks shared by the fused row kernels (rowgemm.hip, layer.hip,
// relgru.hip, query.hip).
//
// A workgroup of 4 waves owns a tile of TM = 16 rows and all d <= 256 output columns;
// wave w owns the four 16-column MFMA tiles [64w, 64w + 64).  An A operand (16 x d) sits
// in LDS with a row stride `lda` = 2 (mod 32) floats, so the 16 rows x 4 k-offsets one
// MFMA step reads fall in distinct banks.  B operands are weights prepacked into MFMA
// fragment order (k_pack_weight, rowgemm.hip):
//     Wp[s][jq][lane][e] = W[4s + lane/16][16(4jq + e) + lane%16]
// so at k-step s wave w reads one coalesced float4 per lane, Wp[s][w][lane].
//
// MFMA: v_mfma_f32_16x16x4_f32.  C/D layout: lane l holds rows 4*(l>>4)+r (r = 0..3) and
// column 16j + (l & 15) of tile j; a row's 16 lanes are one DPP row (row16_sum).
#pragma once
#include "common.h"

namespace regcn {

constexpr int MAX_D = 256;
constexpr int TM = 16;         // rows per workgroup
constexpr int NWAVE = 4;       // waves per workgroup (= 64-column groups)
constexpr int NTHR = 64 * NWAVE;
constexpr int RING = 8;        // k-steps of B fragments in flight per wave
constexpr int RED_FLOATS = 4 * NWAVE * TM;  // RowRed scratch (2 buffers x 2 quantities)

// LDS row stride for width d: smallest value >= d + 2 that is 2 (mod 32).
__host__ __device__ constexpr int tile_lda(int d) { return d + 2 + ((32 - (d + 2) % 32) % 32); }

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
    float* dst = T + i * lda + c;
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

// The first RING B fragments of a packed weight, loaded ahead of the A tile (they do not
// depend on it), so the MFMA chain starts without a load latency.
struct BRing {
  f4 ring[RING];
  __device__ __forceinline__ void load(const float* __restrict__ Wp, int d) {
    const f4* bsrc = reinterpret_cast<const f4*>(Wp) + wave_id() * 64 + (threadIdx.x & 63);
    const int S = d >> 2;
#pragma unroll
    for (int i = 0; i < RING; ++i) ring[i] = bsrc[(int64_t)min(i, S - 1) * 256];
  }
};

// acc += T[16 x d] @ W (T in LDS, W packed with d_in = d), ring pre-filled by BRing::load.
__device__ __forceinline__ void mfma_tile_pf(Frag& acc, const float* T, int lda, const float* __restrict__ Wp, int d,
                                             BRing& br) {
  const int lane = threadIdx.x & 63, w = wave_id();
  const int S = d >> 2;
  const f4* bsrc = reinterpret_cast<const f4*>(Wp) + w * 64 + lane;  // + s * 256
  const float* arow = T + (lane & 15) * lda + (lane >> 4);
  f4* ring = br.ring;
  // A operands ride in their own ring, RING k-steps ahead: an LDS read right before its
  // MFMA would expose the ds_read latency on every step (the sched barriers keep order).
  float aring[RING];
#pragma unroll
  for (int i = 0; i < RING; ++i) aring[i] = arow[4 * min(i, S - 1)];
  int s = 0;
  for (; s + RING <= S; s += RING) {
#pragma unroll
    for (int i = 0; i < RING; ++i) {
      mfma4(acc, aring[i], ring[i]);
      __builtin_amdgcn_sched_barrier(0);
      const int nx = min(s + i + RING, S - 1);
      ring[i] = bsrc[(int64_t)nx * 256];  // unconditional: hipcc can count it
      aring[i] = arow[4 * nx];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int i = 0; i < RING; ++i)
    if (s + i < S) mfma4(acc, aring[i], ring[i]);
}

// acc += T[16 x d] @ W.  No barriers inside.
__device__ __forceinline__ void mfma_tile(Frag& acc, const float* T, int lda, const float* __restrict__ Wp, int d) {
  BRing br;
  br.load(Wp, d);
  mfma_tile_pf(acc, T, lda, Wp, d, br);
}

// Cross-wave row reductions: per-wave partials -> LDS red[buf][wave][row] -> sum.
// Two buffers alternate so one barrier per reduction suffices.
struct RowRed {
  float* red;  // LDS, RED_FLOATS: 2 buffers x (2 quantities x NWAVE x TM)
  int buf;
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
    for (int r = 0; r < 4; ++r) {
      const int i = frag_row(r);
      part[r] = (b[i] + b[TM + i]) + (b[2 * TM + i] + b[3 * TM + i]);
    }
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
      const int i = frag_row(r);
      pa[r] = (ba[i] + ba[TM + i]) + (ba[2 * TM + i] + ba[3 * TM + i]);
      pb[r] = (bb[i] + bb[TM + i]) + (bb[2 * TM + i] + bb[3 * TM + i]);
    }
    buf ^= 1;
  }
  __device__ __forceinline__ void sumsq(const Frag& a, float out[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) s += a.t[j][r] * a.t[j][r];
      out[r] = s;
    }
    allreduce(out);
  }
};

// ---- row maps with the row norms carried along ------------------------------------------
// A row map scales each row by a factor of its norm, so the norm after the map follows
// analytically (|f x| = f |x|): chains of maps need one cross-wave reduction, not one per
// map.  n2[r] is |row|^2 of fragment row r, updated in place.
__device__ __forceinline__ void row_scale(Frag& a, const float f[4]);

__device__ __forceinline__ void scale_known(Frag& a, float n2[4], const float f[4]) {
  row_scale(a, f);
#pragma unroll
  for (int r = 0; r < 4; ++r) n2[r] *= f[r] * f[r];
}

__device__ __forceinline__ void project_known(Frag& a, float n2[4], const Curv& k) {
  float f[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = project_factor(n2[r], k);
  scale_known(a, n2, f);
}

__device__ __forceinline__ void log0_known(Frag& a, float n2[4], const Curv& k) {
  float f[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = log0_factor(n2[r], k);
  scale_known(a, n2, f);
}

__device__ __forceinline__ void exp0_known(Frag& a, float n2[4], const Curv& k) {  // exp0 + project
  float f[4], o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = exp0_factor(n2[r], k, &o[r]);
  row_scale(a, f);
#pragma unroll
  for (int r = 0; r < 4; ++r) n2[r] = o[r];
}

__device__ __forceinline__ void normalize_known(Frag& a, float n2[4]) {  // F.normalize, eps 1e-12
  float f[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = 1.0f / fmaxf(sqrtf(n2[r]), 1e-12f);
  scale_known(a, n2, f);
}

__device__ __forceinline__ void row_scale(Frag& a, const float f[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) a.t[j][r] *= f[r];
}

__device__ __forceinline__ void frag_log0(RowRed& rr, Frag& a, const Curv& k) {
  float n2[4], f[4];
  rr.sumsq(a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = log0_factor(n2[r], k);
  row_scale(a, f);
}

__device__ __forceinline__ void frag_exp0(RowRed& rr, Frag& a, const Curv& k) {
  float n2[4], f[4];
  rr.sumsq(a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = exp0_factor(n2[r], k);
  row_scale(a, f);
}

__device__ __forceinline__ void frag_project(RowRed& rr, Frag& a, const Curv& k) {
  float n2[4], f[4];
  rr.sumsq(a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = project_factor(n2[r], k);
  row_scale(a, f);
}

__device__ __forceinline__ void frag_normalize(RowRed& rr, Frag& a) {  // F.normalize, eps 1e-12
  float n2[4], f[4];
  rr.sumsq(a, n2);
#pragma unroll
  for (int r = 0; r < 4; ++r) f[r] = 1.0f / fmaxf(sqrtf(n2[r]), 1e-12f);
  row_scale(a, f);
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

// C-layout fragment read from an LDS tile (columns >= d read as 0).
__device__ __forceinline__ void frag_from_tile(Frag& a, const float* T, int lda, int d) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float* row = T + frag_row(r) * lda;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
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

}  // namespace regcn
