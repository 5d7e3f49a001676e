// Two-phase relation GRU device pieces (relgru.hip launches them alone; timestep.hip hosts
// them as extra workgroups of its phase launches).
#pragma once
#include "common.h"
#include "gather.h"
#include "regcn_internal.h"
#include "rowtile.h"

namespace regcn {
// per wave count (rowtile.h): units built with different REGCN_ROWTILE_WAVES never share a definition
inline namespace REGCN_RT_CAT(rowtile_w, REGCN_ROWTILE_WAVES) {

constexpr int GR4 = 4;  // k-blocks (16 k-steps each) of operands in flight per wave

// ============================================================ two-phase relation GRU
// The GRU input is [emb_rel | x_mean] and only x_mean depends on the entity rows the previous
// timestep produced; emb_rel and the hidden state h_prev are ready one timestep earlier.  So
// the gate pre-activations split into
//   P0 = W_ir^e emb + b_ir + W_hr h + b_hr,  P1 = (z gate likewise),
//   P2 = W_in^e emb + b_in,                  P3 = W_hn h + b_hn          (k_gru_pre)
// and the part on the timestep's critical path is the relation mean plus ONE K = d product:
//   r = s(P0 + W_ir^x m), z = s(P1 + W_iz^x m), n = tanh(P2 + W_in^x m + r P3),
//   h' = (1 - z) n + z h                                                 (k_gru_x)
// k_gru_pre runs on its own stream while the previous timestep's layers run.  Weights: W_ih
// split into its emb columns (W^e) and x_mean columns (W^x), each packed as a (3d x d)
// nn.Linear matrix (regcn_pack_linear_f32); W_hh as before.  Same per-workgroup shape as
// k_rel_gru: 16 relation rows x one 16-column tile, waves splitting K.

// acc{r,z,n} += A[16 x k-blocks beg..end) . W^T (3 gates), operand rings GR4 blocks ahead.
__device__ __forceinline__ void gru_mfma(const float* arow, const f4* bb, int64_t gs, int NT, int beg, int end, f4& ar,
                                         f4& az, f4& an) {
  auto clamp_blk = [&](int b) { return max(min(b, end - 1), 0); };
  f4 br[GR4], bz[GR4], bn[GR4], ra[GR4];
#pragma unroll
  for (int i = 0; i < GR4; ++i) {
    const f4* b = bb + (int64_t)clamp_blk(beg + i) * NT * 64;
    br[i] = b[0];
    bz[i] = b[gs];
    bn[i] = b[2 * gs];
    ra[i] = *reinterpret_cast<const f4*>(arow + 16 * clamp_blk(beg + i));
  }
  for (int b0 = beg; b0 < end; b0 += GR4) {
#pragma unroll
    for (int i = 0; i < GR4; ++i) {
      if (b0 + i < end) {  // wave-uniform
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ar = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[i][e], br[i][e], ar, 0, 0, 0);
          az = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[i][e], bz[i][e], az, 0, 0, 0);
          an = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[i][e], bn[i][e], an, 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      const int nb = clamp_blk(b0 + i + GR4);
      const f4* b = bb + (int64_t)nb * NT * 64;
      br[i] = b[0];
      bz[i] = b[gs];
      bn[i] = b[2 * gs];
      ra[i] = *reinterpret_cast<const f4*>(arow + 16 * nb);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// Every wave of the unit's workgroup (NWAVE, rowtile.h: 8 in the dataset-size kernels and the
// standalone relgru.hip launches, 4 otherwise) takes part in the products: the pre-phase puts
// half of them on W_ih^e (emb columns) and half on W_hh, the x-phase splits K = d over all of
// them, each wave a 1/NWAVE share of the k-blocks (at 8 waves the GRU blocks' MFMA chains are
// half as long as at 4, and no wave of an 8-wave phase workgroup idles through them).  The C
// registers are finished by waves 0-3 (wave q: C register q), summing every wave's partial in
// wave order.
constexpr int PRE_WAVES = NWAVE;
constexpr int X_WAVES = NWAVE;
static_assert(NWAVE >= 4 && NWAVE % 2 == 0, "the GRU parts need >= 4 waves (one per C register)");

__host__ __device__ inline int gru_dpad(int d) { return (d + 15) & ~15; }
// A tile stride for `parts` d-wide operand blocks, each zero padded to a multiple of 16 and
// the stride = 8 (mod 16): conflict-free ds_read_b128 fragment reads.
__host__ __device__ inline int gru2_lda(int d, int parts) {
  const int n = parts * gru_dpad(d);
  return n + ((8 - n % 16) + 16) % 16;
}

// XCD-grouped order of a launch's GRU blocks: blocks g and g + 8 share an XCD (round-robin
// dispatch), so class g % 8 takes a contiguous run of the (column tile, row tile) order and
// each column tile's weight slice (read by every row tile) is fetched into one or two XCDs'
// L2s instead of all eight.  The launch pads the GRU blocks to a multiple of 8 (the pads
// return at once).
__host__ __device__ inline int gru_blocks_padded(int n) { return (n + 7) & ~7; }
__device__ __forceinline__ bool gru_block_xcd(int g, int n, int rt, int& bx, int& by) {
  const int w = (g & 7) * ((n + 7) >> 3) + (g >> 3);
  bx = w % rt;
  by = w / rt;
  return w < n;
}

// the waves' gate partials (PRE_WAVES x 3 x 64 float4) reuse the A tile's LDS once every wave's
// products have read it (one barrier between)
inline size_t gru_pre_lds_bytes(int d) {
  return std::max((size_t)TM * gru2_lda(d, 2) * 4, (size_t)PRE_WAVES * 3 * 64 * 16);
}

// Workgroup (bx, by) of the pre-phase: relation rows 16 bx.., output column tile by.
__device__ __forceinline__ void gru_pre_block(const RelGru2Args& p, int bx, int by, float* lds) {
  const int d = p.d, dp = gru_dpad(d), lda = gru2_lda(d, 2);
  float* A = lds;  // TM x lda: [emb_rel | 0 pad | h_prev | 0 pad]
  f4* red = reinterpret_cast<f4*>(lds);  // [PRE_WAVES][3][64], over A after the products
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // Every wave of the workgroup runs this whole body and so meets every one of its barriers;
  // waves beyond the part's four (an 8-wave phase launch hosting it) only skip the work
  // between them (`act` is wave-uniform).
  const bool act = w < PRE_WAVES;
  const int r0 = bx * TM, jt = by;
  const int n_valid = min(TM, p.R2 - r0);
  if (act) {  // [emb_rel | h_prev] rows as float4s, every load issued before the first LDS store
    constexpr int IT = TM * 2 * (MAX_D / 4) / (64 * PRE_WAVES);
    const int q4 = d >> 2, n = TM * 2 * q4;
    f4 v[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = min((int)threadIdx.x + it * 64 * PRE_WAVES, n - 1);
      const int i = idx / (2 * q4), rem = idx - i * 2 * q4, part = rem / q4, c = (rem - part * q4) * 4;
      v[it] = *reinterpret_cast<const f4*>((part ? p.h_prev : p.emb_rel) + (int64_t)(r0 + min(i, n_valid - 1)) * d + c);
    }
    // zero padding: columns [d, dp) of each part and [2 dp, lda)
    const int npad = 2 * (dp - d) + (lda - 2 * dp);
    for (int t = threadIdx.x; t < TM * npad; t += 64 * PRE_WAVES) {
      const int i = t / npad, j = t - i * npad;
      const int c = j < dp - d ? d + j : j < 2 * (dp - d) ? dp + d + (j - (dp - d)) : 2 * dp + (j - 2 * (dp - d));
      A[i * lda + c] = 0.f;
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = threadIdx.x + it * 64 * PRE_WAVES;
      if (idx >= n) break;
      const int i = idx / (2 * q4), rem = idx - i * 2 * q4, part = rem / q4, c = (rem - part * q4) * 4;
      const f4 x = i < n_valid ? v[it] : f4{0.f, 0.f, 0.f, 0.f};
      float* dst = A + i * lda + part * dp + c;
      dst[0] = x.x;
      dst[1] = x.y;
      dst[2] = x.z;
      dst[3] = x.w;
    }
  }
  __syncthreads();
  f4 ar = {0.f, 0.f, 0.f, 0.f}, az = ar, an = ar;
  if (act) {
    const bool hh = w >= PRE_WAVES / 2;
    const int wi = hh ? w - PRE_WAVES / 2 : w;
    const int NB = dp >> 4, NT = dp >> 4;
    const int beg = (NB * wi) / (PRE_WAVES / 2), end = (NB * (wi + 1)) / (PRE_WAVES / 2);
    const f4* bb = reinterpret_cast<const f4*>(hh ? p.w_hh : p.w_ih_e) + (int64_t)jt * 64 + lane;
    const int64_t gs = (int64_t)NB * NT * 64;
    const float* arow = A + (lane & 15) * lda + 4 * (lane >> 4) + (hh ? dp : 0);
    if (beg < end) gru_mfma(arow, bb, gs, NT, beg, end, ar, az, an);
  }
  __syncthreads();  // every wave's products have read A: its LDS takes the partials
  if (act) {
    red[(w * 3 + 0) * 64 + lane] = ar;
    red[(w * 3 + 1) * 64 + lane] = az;
    red[(w * 3 + 2) * 64 + lane] = an;
  }
  __syncthreads();
  if (!act || w >= 4) return;  // past the last barrier; waves 0-3 finish the C registers
  const int q = w;  // wave q finishes C register q (row 4 (lane >> 4) + q)
  float sr = 0.f, sz = 0.f, sn_i = 0.f, sn_h = 0.f;
#pragma unroll
  for (int w2 = 0; w2 < PRE_WAVES; ++w2) {
    sr += red[(w2 * 3 + 0) * 64 + lane][q];
    sz += red[(w2 * 3 + 1) * 64 + lane][q];
    if (w2 < PRE_WAVES / 2) sn_i += red[(w2 * 3 + 2) * 64 + lane][q];
    else sn_h += red[(w2 * 3 + 2) * 64 + lane][q];
  }
  const int i = 4 * (lane >> 4) + q;
  const int n = 16 * jt + (lane & 15);
  if (i < n_valid && n < d) {
    float* o = p.pre + (int64_t)(r0 + i) * 4 * d;
    o[n] = sr + (p.b_ih[n] + p.b_hh[n]);
    o[d + n] = sz + (p.b_ih[d + n] + p.b_hh[d + n]);
    o[2 * d + n] = sn_i + p.b_ih[2 * d + n];
    o[3 * d + n] = sn_h + p.b_hh[2 * d + n];
  }
}

// Relation means of the tile's 16 relations into A (TM x lda, columns [0, d)), 4 waves.
// The tile's r_to_e items are flattened (row-sorted) and split into contiguous ranges per
// wave; each wave keeps 8 row loads in flight and reduces segment-wise into partial slot
// (row + wave); partials are combined in wave order (deterministic), then / count.
// Every wave calls it (its one barrier); waves with !act only meet the barrier.
__device__ __forceinline__ void stage_rel_means(const RelGru2Args& p, float* A, int lda, float* part, int* tmask,
                                                int r0, int n_valid, bool act) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int d = p.d, col = lane * 4, colc = min(col, d - 4);
  const bool active = col < d;
  const int li = min(lane, TM - 1);
  const bool lrow = lane < TM && lane < n_valid;
  const int cnt_l = lrow ? (int)p.rel_count[r0 + li] : 0;
  const int st_l = lrow ? p.rel_start[r0 + li] : 0;
  int off[TM], total = 0;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    off[i] = total;
    total += __builtin_amdgcn_readlane(cnt_l, i);
  }
  const int ib = act ? (total * w) / X_WAVES : 0, ie = act ? (total * (w + 1)) / X_WAVES : 0;
  const f4 zero = {0.f, 0.f, 0.f, 0.f};
  int cur = -1;
  unsigned mask = 0;
  f4 acc = zero;
  auto flush = [&]() {
    if (cur >= 0) {
      float* dst = part + (cur + w) * lda;
      if (active) *reinterpret_cast<f4*>(dst + col) = acc;
      mask |= 1u << cur;
    }
  };
  const uint32_t xoff = (uint32_t)colc * 4u;
  for (int t0 = ib; t0 < ie; t0 += 64) {
    const int n = min(64, ie - t0);
    const int k = t0 + min(lane, n - 1);
    // the item's row: the last row whose span starts at or before it (offsets do not
    // decrease, and a row whose span starts at or before k < total is never empty unless a
    // later row starts there too)
    int my_i = 0;
#pragma unroll
    for (int i = 1; i < TM; ++i) my_i = k >= off[i] ? i : my_i;
    const int st_i = __shfl(st_l, my_i);
    int offi = 0;
#pragma unroll
    for (int i = 0; i < TM; ++i) offi = (i == my_i) ? off[i] : offi;
    const int my_e = p.rel_idx[st_i + (k - offi)];
    for (int j = 0; j < n; j += 8) {
      f4 xs[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) xs[u] = row_load4(p.x + (int64_t)rl(my_e, min(j + u, n - 1)) * d, xoff);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (j + u < n) {
          const int li2 = rl(my_i, j + u);
          if (li2 != cur) {
            flush();
            cur = li2;
            acc = zero;
          }
          acc += xs[u];
        }
      }
    }
  }
  flush();
  if (act && lane == 0) tmask[w] = (int)mask;
  __syncthreads();
  if (!act) return;
  for (int i = w; i < TM; i += X_WAVES) {
    f4 s = zero;
#pragma unroll
    for (int w2 = 0; w2 < X_WAVES; ++w2)
      if ((tmask[w2] >> i) & 1) s += *reinterpret_cast<const f4*>(part + (i + w2) * lda + colc);
    const float c = (float)__builtin_amdgcn_readlane(cnt_l, i);
    if (c > 0.f) s = s / c;
    if (active) *reinterpret_cast<f4*>(A + i * lda + col) = s;
  }
}

// A (TM x lda) | the partial rows of the relation means ((TM + X_WAVES - 1) x lda), whose LDS the
// waves' gate partials (X_WAVES x 3 x 64 float4) reuse after the means are staged | tmask
__host__ __device__ inline int gru_x_part_floats(int d) {
  const int rows = (TM + X_WAVES - 1) * gru2_lda(d, 1), red = X_WAVES * 3 * 64 * 4;
  return rows > red ? rows : red;
}
inline size_t gru_x_lds_bytes(int d) { return ((size_t)TM * gru2_lda(d, 1) + gru_x_part_floats(d)) * 4 + 16 * 4; }

// Workgroup (bx, by) of the x-phase.  The gate partials and h_prev are loaded at entry
// (they depend on nothing here), so their latency hides under the relation-mean gather.
__device__ __forceinline__ void gru_x_block(const RelGru2Args& p, int bx, int by, float* lds) {
  const int d = p.d, dp = gru_dpad(d), lda = gru2_lda(d, 1);
  float* A = lds;                                         // TM x lda: x_mean | 0 pad
  float* part = lds + TM * lda;                           // (TM + X_WAVES - 1) x lda partial rows
  f4* red = reinterpret_cast<f4*>(part);                  // [X_WAVES][3][64], over part after staging
  int* tmask = reinterpret_cast<int*>(part + gru_x_part_floats(d));
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // as in gru_pre_block: every wave meets every barrier, waves past the part's four skip the work
  const bool act = w < X_WAVES;
  const int r0 = bx * TM, jt = by;
  const int n_valid = min(TM, p.R2 - r0);
  const int NB = dp >> 4, NT = dp >> 4;
  const int beg = (NB * w) / X_WAVES, end = (NB * (w + 1)) / X_WAVES;
  const int ei = 4 * (lane >> 4) + w;  // this lane's output element (wave w < 4 finishes C register w)
  const int en = 16 * jt + (lane & 15);
  const bool eok = act && w < 4 && ei < n_valid && en < d;
  const int64_t erow = (int64_t)(r0 + (eok ? ei : 0));
  const int ecol = eok ? en : 0;
  const float* pr = p.pre + erow * 4 * d;
  const float pre0 = pr[ecol], pre1 = pr[d + ecol], pre2 = pr[2 * d + ecol], pre3 = pr[3 * d + ecol];
  const float hprev = p.h_prev[erow * d + ecol];
  // zero A (padding columns and absent relations stay 0), then the means
  if (act)
    for (int t = threadIdx.x; t < TM * lda; t += 64 * X_WAVES) A[t] = 0.f;
  if (p.x_mean) {
    __syncthreads();
    if (act)
      for (int t = threadIdx.x; t < n_valid * d; t += 64 * X_WAVES) {
        const int i = t / d, k = t - i * d;
        A[i * lda + k] = p.x_mean[(int64_t)(r0 + i) * d + k];
      }
  } else {
    stage_rel_means(p, A, lda, part, tmask, r0, n_valid, act);
  }
  __syncthreads();
  if (act) {
    const f4* bb = reinterpret_cast<const f4*>(p.w_ih_x) + (int64_t)jt * 64 + lane;
    const int64_t gs = (int64_t)NB * NT * 64;
    f4 ar = {0.f, 0.f, 0.f, 0.f}, az = ar, an = ar;
    const float* arow = A + (lane & 15) * lda + 4 * (lane >> 4);
    if (beg < end) gru_mfma(arow, bb, gs, NT, beg, end, ar, az, an);
    red[(w * 3 + 0) * 64 + lane] = ar;
    red[(w * 3 + 1) * 64 + lane] = az;
    red[(w * 3 + 2) * 64 + lane] = an;
  }
  __syncthreads();
  if (!act || w >= 4) return;  // past the last barrier; waves 0-3 finish the C registers
  const int q = w;  // wave q < 4 finishes C register q
  float v[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float t = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < X_WAVES; ++w2) t += red[(w2 * 3 + a) * 64 + lane][q];
    v[a] = t;
  }
  (void)q;
  if (eok) {
    const float r = sigmoidf(pre0 + v[0]);
    const float z = sigmoidf(pre1 + v[1]);
    const float nn = ftanh(pre2 + v[2] + r * pre3);
    p.h_out[erow * d + en] = (1.f - z) * nn + z * hprev;
  }
}


}  // inline namespace
}  // namespace regcn
