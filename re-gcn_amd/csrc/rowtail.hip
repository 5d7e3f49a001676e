// Large-snapshot layers in two launches: the in-edge gather, then
// a 64-row MFMA tail.
//
// The fused layer kernel (layer.hip) runs a 16-row tile's gather and then its three d x d
// products serially, and every 16-row tile streams each d x d weight from L2 once per product:
// at config 5 that is 38 GB of L1 <- L2 weight traffic per launch (16x re-read per 256 rows),
// and a tile's life is gather (24 us) then products (12 us) with ~4 tiles per CU to overlap
// them.  Here, for snapshots with many rows:
//   1. k_gather_agg: the same per-tile gather (layer_parts.h tile_gather / tile_finish_rows) of
//      the inline in-edge rows, finished rows written to an agg buffer that already holds the
//      hub rows' chunked pre-aggregation (no products, no weights: small LDS and register
//      footprint, many tiles in flight);
//   2. k_rowtail: one workgroup = 4 waves = 64 RG rows, each wave RG groups of 16 rows x ALL
//      columns, so a row's reductions (norms, dots of the row maps and the timestep) are
//      in-wave (a DPP row sum, no LDS, no barrier) and the four waves of a workgroup share the
//      weight fragments of each k-block (one L2 read per workgroup, 4 RG x less weight traffic
//      per row).  Both operands arrive in LDS by DMA (global_load_lds) two / one k-blocks
//      ahead: lane l of a group DMAs the 4 consecutive columns 16 b + 4 (l / 16) .. + 3 of its
//      row (l % 16) of k-block b -- exactly the A fragment it later reads -- and the weights
//      are packed in the matching k order (k_pack_weight_kp: the k index of a 16-deep block is
//      permuted, which a contraction does not see), so a k-block is 16 KB of weight, copied
//      as is.
// Epilogues are the fused kernel's (clamp, self loop, rrelu, exp0, the timestep with the time
// gate and the radius evolution), in fp32 with the same formulas; the products accumulate in
// another k order (1e-7-relative differences, not bitwise the fused kernel).
#include <cstdlib>

#include "layer_parts.h"

namespace regcn {

// ------------------------------------------------------------------------------ packing
// Wp[s][jq][lane][e] = W[16 (s / 4) + 4 (lane / 16) + s % 4][16 (4 jq + e) + lane % 16], zero
// outside d_in x d_out; s < 4 * ceil(d_in / 16).  The last 16-deep block is transposed:
// W[16 (s / 4) + 4 (s % 4) + lane / 16][...], so its k-steps past d_in hold only zero rows and
// rt_mm skips them (d = 200: 2 of the block's 4 steps, 50 k-steps per product instead of 52).
__global__ void k_pack_weight_kp(const float* __restrict__ W, int d_in, int d_out, int S, float* __restrict__ Wp) {
  const int total = S * 4 * 64 * 4;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int e = idx & 3, lane = (idx >> 2) & 63, jq = (idx >> 8) & 3, s = idx >> 10;
    const bool last = (s >> 2) == (S >> 2) - 1;
    const int k = 16 * (s >> 2) + (last ? 4 * (s & 3) + (lane >> 4) : 4 * (lane >> 4) + (s & 3));
    const int n = 16 * (4 * jq + e) + (lane & 15);
    Wp[idx] = (k < d_in && n < d_out) ? W[(int64_t)k * d_out + n] : 0.f;
  }
}

size_t packed_weight_kp_floats(int d_in) { return (size_t)((d_in + 15) / 16) * 4 * 4 * 64 * 4; }

int pack_weight_kp(const float* W, int d_in, int d_out, float* Wp, hipStream_t st) {
  if (!W || !Wp) return set_error(REGCN_EINVAL, "null pointer");
  if (d_in <= 0 || d_out <= 0 || d_out > MAX_D) return set_error(REGCN_EINVAL, "pack_weight_kp needs d_out <= 256");
  const int S = 4 * ((d_in + 15) / 16);
  const int total = S * 4 * 64 * 4;
  hipLaunchKernelGGL(k_pack_weight_kp, dim3((total + 255) / 256), dim3(256), 0, st, W, d_in, d_out, S, Wp);
  return check_launch("k_pack_weight_kp");
}

// ------------------------------------------------------------------------------- gather
// The inline in-edge rows of every in-degree > 0 tile (the tiles / items of the fused kernel),
// finished (norm-scaled sum, or Lorentz centroid -> log0) and written to out[row]; rows over
// the budget are skipped (out already holds them).
#ifndef REGCN_GATHER_WAVES
#define REGCN_GATHER_WAVES 5  // waves per SIMD the gather is compiled for (89 VGPRs: 5)
#endif
template <int AGG, int S>
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(REGCN_GATHER_WAVES))) void k_gather_agg(LayerArgs p, float* __restrict__ out, int tile0) {
  extern __shared__ float lds[];
  const int tile = tile0 + blockIdx.x;
  const int lda = tile_lda(p.d);
  float* part = lds;
  int* trow = reinterpret_cast<int*>(lds + (TM + NWAVE - 1) * lda);
  int* tmask = trow + TM;
  float* xsh = lds + (TM + NWAVE - 1) * lda + 32;
  const int start = p.tiles[2 * tile], count = p.tiles[2 * tile + 1];
  if (threadIdx.x < TM) trow[threadIdx.x] = p.rows[start + ((int)threadIdx.x < count ? threadIdx.x : 0)];
  __syncthreads();
  const int lrow = trow[min((int)(threadIdx.x & 63), TM - 1)];
  const int rdeg = p.rowptr[lrow + 1] - p.rowptr[lrow];
  const float rnorm = AGG != AGG_LORENTZ ? p.norm[lrow] : 1.f;
  tile_gather<AGG, S>(p, part, lda, trow, tile, tmask, xsh);
  __syncthreads();
  constexpr int RPW = TM / NWAVE;
  f4 o[RPW], pre[RPW];
  bool heavy[RPW];
  tile_finish_rows<AGG>(p, part, lda, trow, count, tmask, rdeg, rnorm, o, pre, heavy);
  const int lane = threadIdx.x & 63, w = wave_id(), col = lane * 4;
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int i = w + NWAVE * q;
    if (i < count && !heavy[q] && col < p.d) *reinterpret_cast<f4*>(out + (int64_t)trow[i] * p.d + col) = o[q];
  }
}

// ---------------------------------------------------------------- relation half as a product
// Tiles [0, crel_tiles) of a union / euclid gather (item_crel): the tile's items in (row, type)
// order (regcn_snapshot_item_type_order_i32).  By linearity (hyperbolic_layers.py:222-240)
//   sum_e w_e (x[src_e] + rel[t_e]) = sum_e w_e x[src_e] + sum_t C[row][t] rel[t],
//   C[row][t] = sum of w_e over the row's type-t items,
// so the per-item loads are the source rows only; the weights of a row's same-type items are
// summed in registers (a segmented lane scan per 64-item window, the window's last run carried
// into the next) into an LDS matrix C[16][n_types], and the relation rows enter as one
// [16 x n_types] @ [n_types x d] MFMA product per tile: the relation table is read once per tile
// instead of once per item.  Deterministic: a wave stores the sum of every run it owns (plain
// stores: a (row, type) run lies in one wave's item range but for its pieces at range
// boundaries); each wave's FIRST run -- possibly the tail of the previous wave's last run -- is
// parked and added by one thread in wave order after the barrier.
constexpr int CREL_MAX_TYPES = 512;
// source rows in flight per wave in the crel gather: 32 (default) or 16 (REGCN_CREL_EB)
static int crel_eb() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("REGCN_CREL_EB");
    v = e ? atoi(e) : 32;
  }
  return v;
}

__host__ __device__ inline int crel_kpad(int n_types) { return (n_types + 15) & ~15; }
__host__ __device__ inline int crel_ld(int n_types) { return crel_kpad(n_types) + 4; }  // C row stride (floats)
__host__ __device__ inline size_t crel_lds_bytes(int d, int n_types) {
  return (size_t)((TM + NWAVE - 1) * tile_lda(d) + 32 + 2 * NWAVE + TM * crel_ld(n_types)) * 4;
}

template <int AGG, int EB>
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(3))) void k_gather_crel(LayerArgs p,
                                                                                          float* __restrict__ out,
                                                                                          int tile0) {
  extern __shared__ float lds[];
  const int tile = tile0 + blockIdx.x;
  const int d = p.d, lda = tile_lda(d);
  float* part = lds;
  int* trow = reinterpret_cast<int*>(lds + (TM + NWAVE - 1) * lda);
  int* tmask = trow + TM;
  int* bkey = reinterpret_cast<int*>(lds + (TM + NWAVE - 1) * lda + 32);  // parked first runs
  float* bval = reinterpret_cast<float*>(bkey + NWAVE);
  float* cl = lds + (TM + NWAVE - 1) * lda + 32 + 2 * NWAVE;
  const int cld = crel_ld(p.n_types), kpad = crel_kpad(p.n_types);
  const int start = p.tiles[2 * tile], count = p.tiles[2 * tile + 1];
  const int lane = threadIdx.x & 63, w = wave_id();
  const int i0 = p.item_ptr[tile], n_items = p.item_ptr[tile + 1] - i0;
  if (n_items == 0) return;  // a tile of hub rows only (pre-aggregated): nothing to write
  if (threadIdx.x < TM) trow[threadIdx.x] = p.rows[start + ((int)threadIdx.x < count ? threadIdx.x : 0)];
  if (lane == 0) bkey[w] = -1;
  for (int i = threadIdx.x; i < TM * cld; i += NTHR) cl[i] = 0.f;
  __syncthreads();
  const int lrow = trow[min(lane, TM - 1)];
  const int rdeg = p.rowptr[lrow + 1] - p.rowptr[lrow];
  const float rnorm = p.norm[lrow];
  // ---- the items: source rows per item, relation weights per (row, type) run (EB source rows
  // in flight per wave: no relation rows in the loop, and 3 workgroups per CU for the LDS C)
  const int col = lane * 4, colc = min(col, d - 4);
  const bool active = col < d;
  const int ib = i0 + (n_items * w) / NWAVE, ie = i0 + (n_items * (w + 1)) / NWAVE;
  const f4 zero = {0.f, 0.f, 0.f, 0.f};
  int cur = -1;
  unsigned mask = 0;
  f4 acc = zero;
  auto flush = [&]() {
    if (cur >= 0) {
      float* dst = part + (cur + w) * lda;
      if (active) {
        dst[col] = acc.x;
        dst[col + 1] = acc.y;
        dst[col + 2] = acc.z;
        dst[col + 3] = acc.w;
      }
      mask |= 1u << cur;
    }
  };
  auto take = [&](int li) {
    if (li != cur) {
      flush();
      cur = li;
      acc = zero;
    }
  };
  const uint32_t xoff = (uint32_t)colc * 4u;
  bool first_pending = true;  // the wave's first run is parked, not stored
  int ck = -1;                // the carried (open) run of the previous window: key, weight sum
  float cw = 0.f;
  auto emit1 = [&](int key, float v) {  // one run's sum, from lane 0
    if (first_pending) {
      if (lane == 0) bkey[w] = key, bval[w] = v;
      first_pending = false;
    } else if (lane == 0) {
      cl[(key >> 16) * cld + (key & 0xffff)] = v;
    }
  };
  for (int t0 = ib; t0 < ie; t0 += 64) {
    const int n = min(64, ie - t0);
    const int t = t0 + min(lane, n - 1);
    const int my_s = p.item_src[t];
    const int tl = p.item_tl[t];
    const int my_t = tl >> 4, my_i = tl & 15;
    float my_w = 1.f;
    if (AGG == AGG_UNION) my_w = expf(-p.gamma * fabsf(p.radius[my_s] - p.radius[trow[my_i]]));
    const bool valid = lane < n;
    const int key = (my_i << 16) | my_t;
    const int key0 = __builtin_amdgcn_readfirstlane(key);
    if (ck >= 0 && key0 != ck) {  // the carried run ended with the last window
      emit1(ck, cw);
      ck = -1;
    }
    float v = valid ? my_w : 0.f;
    if (lane == 0 && ck >= 0) v += cw;  // ... or continues here
    const int pk = __shfl_up(key, 1);
    const uint64_t heads = __ballot(valid && (lane == 0 || key != pk)) | 1ull;
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    const int sstart = 63 - __builtin_clzll(heads & upto);
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {  // inclusive segmented sum, fixed order
      const float u = __shfl_up(v, off);
      if (lane - off >= sstart) v += u;
    }
    uint64_t ends = __ballot(valid && lane != n - 1 && ((heads >> ((lane + 1) & 63)) & 1ull));
    if (first_pending && ends) {  // the lowest closed run is the wave's first
      const int l0 = __builtin_ctzll(ends);
      const float v0 = __shfl(v, l0);
      const int k0 = __shfl(key, l0);
      if (lane == 0) bkey[w] = k0, bval[w] = v0;
      ends &= ends - 1;
      first_pending = false;
    }
    if ((ends >> lane) & 1ull) cl[my_i * cld + my_t] = v;
    ck = __shfl(key, n - 1);
    cw = __shfl(v, n - 1);
    // the source half, EB rows in flight per wave
    for (int j = 0; j < n; j += EB) {
      const int nv = n - j;
      f4 xs[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) xs[u] = row_load4(p.x + (int64_t)rl(my_s, j + u) * d, xoff);
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        if (u < nv) {
          take(rl(my_i, j + u));
          acc += rlf(my_w, j + u) * xs[u];
        }
      }
    }
  }
  if (ck >= 0) emit1(ck, cw);
  flush();
  if (lane == 0) tmask[w] = (int)mask;
  __syncthreads();
  if (threadIdx.x == 0) {  // the parked first runs, in wave order
#pragma unroll
    for (int w2 = 0; w2 < NWAVE; ++w2)
      if (bkey[w2] >= 0) cl[(bkey[w2] >> 16) * cld + (bkey[w2] & 0xffff)] += bval[w2];
  }
  __syncthreads();
  // ---- the relation half: C[16 x kpad] @ rel_t^T, k-permuted operands (16-deep block b, MFMA
  // step e: k = 16 b + 4 (lane / 16) + e for both A and B), wave w: column tiles w + NWAVE j
  {
    const int nt = (d + 15) >> 4, q = lane >> 4, r16 = lane & 15;
    const float* arow = cl + r16 * cld + 4 * q;
    constexpr int JMAX = (MAX_D / 16 + NWAVE - 1) / NWAVE;
    f4 racc[JMAX];
#pragma unroll
    for (int j = 0; j < JMAX; ++j) racc[j] = zero;
    // B fragments stream from L2 (the relation table is L2-resident): a ring of CR_DEPTH k-blocks
    // in flight ahead of the MFMAs (one block's MFMAs ~512 cycles, an L2 round trip ~1-2k);
    // unconditional loads (column tiles past nt read row 16 ct + r16 of the zero-padded rows)
    constexpr int CR_DEPTH = 4;
    const int nkb = kpad / 16;
    const float* bbase = p.rel_t + (int64_t)r16 * kpad + 4 * q;
    auto bload = [&](f4 (&dst)[JMAX], int b) {
      const int bb = min(b, nkb - 1);
#pragma unroll
      for (int j = 0; j < JMAX; ++j) {
        const int ct = min(w + NWAVE * j, nt - 1);
        dst[j] = *reinterpret_cast<const f4*>(bbase + (int64_t)(16 * ct) * kpad + 16 * bb);
      }
    };
    f4 ring[CR_DEPTH][JMAX];
#pragma unroll
    for (int i = 0; i < CR_DEPTH; ++i) bload(ring[i], i);
    for (int b0 = 0; b0 < nkb; b0 += CR_DEPTH) {
#pragma unroll
      for (int i = 0; i < CR_DEPTH; ++i) {
        const int b = b0 + i;
        if (b < nkb) {  // wave-uniform
          const f4 a = *reinterpret_cast<const f4*>(arow + 16 * b);
#pragma unroll
          for (int j = 0; j < JMAX; ++j) {
            if (w + NWAVE * j < nt) {  // wave-uniform
#pragma unroll
              for (int e = 0; e < 4; ++e)
                racc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], ring[i][j][e], racc[j], 0, 0, 0);
            }
          }
          bload(ring[i], b + CR_DEPTH);  // block b + CR_DEPTH into the slot just consumed
        }
      }
    }
    // add row i's relation sum into the slot its first writing wave used
#pragma unroll
    for (int j = 0; j < JMAX; ++j) {
      const int ct = w + NWAVE * j, c = 16 * ct + r16;
      if (ct >= nt || c >= d) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 4 * q + r;
        int wf = -1;
#pragma unroll
        for (int w2 = NWAVE - 1; w2 >= 0; --w2)
          if ((tmask[w2] >> i) & 1) wf = w2;
        if (i < count && wf >= 0) part[(i + wf) * lda + c] += racc[j][r];
      }
    }
  }
  __syncthreads();
  constexpr int RPW = TM / NWAVE;
  f4 o[RPW], pre[RPW];
  bool heavy[RPW];
  tile_finish_rows<AGG>(p, part, lda, trow, count, tmask, rdeg, rnorm, o, pre, heavy);
#pragma unroll
  for (int q2 = 0; q2 < RPW; ++q2) {
    const int i = w + NWAVE * q2;
    if (i < count && !heavy[q2] && col < d) *reinterpret_cast<f4*>(out + (int64_t)trow[i] * d + col) = o[q2];
  }
}

// --------------------------------------------------------------------------- 64-row tail
constexpr int RT_ROWS = 64;

template <int NT>
struct RAcc {
  f4 t[NT];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int j = 0; j < NT; ++j) t[j] = f4{0.f, 0.f, 0.f, 0.f};
  }
};

// Masked lanes of the blend staging (rows past the group, columns >= d) DMA from this zero
// row instead of their row: no select on the loaded value, which would make the compiler wait
// for the load right where it is issued.
__device__ const f4 kZeroRow[1] = {{0.f, 0.f, 0.f, 0.f}};

constexpr int RT_KB_BYTES = 4 * 4 * 64 * 16;  // one 16-deep k-block of a packed weight: 16 KB
// Diagnostic build only (-DREGCN_RT_STAMPS=1, tools/c5probe.py --rt-stamps): the step tail's
// wave 0 s_memtime cycles per phase into trace[16 b + 8 ..]: products, row maps, blend-stage
// waits, blend, the row maps after it (radius included), the radius stores, the x stores.
#ifndef REGCN_RT_STAMPS
#define REGCN_RT_STAMPS 0
#endif
constexpr bool kRtStamps = REGCN_RT_STAMPS != 0;
struct RtStamps {
  int64_t ph[7] = {0, 0, 0, 0, 0, 0, 0}, t = 0;
  __device__ __forceinline__ void start() {
    if constexpr (kRtStamps) t = (int64_t)__builtin_amdgcn_s_memtime();
  }
  __device__ __forceinline__ void mark(int k) {
    if constexpr (kRtStamps) {
      const int64_t u = (int64_t)__builtin_amdgcn_s_memtime();
      ph[k] += u - t;
      t = u;
    }
  }
  __device__ __forceinline__ void write(int64_t* trace) {
    if constexpr (kRtStamps) {
      if (trace && threadIdx.x == 0)
        for (int k = 0; k < 7; ++k) trace[(int64_t)blockIdx.x * 16 + 8 + k] = ph[k];
    }
  }
};
constexpr int RT_A_RING = 3;
// LDS of a workgroup whose waves hold RG 16-row groups each: the weight double buffer and the
// A ring (3 k-blocks x 4 waves x RG groups x 1 KB)
__host__ __device__ constexpr size_t rt_lds_bytes(int RG) { return 2 * RT_KB_BYTES + RT_A_RING * 4 * RG * 1024; }

// One 16-deep k-block of rt_mm: acc[g] += A_g[.., block] @ W[block, ..].  A fragments from the
// wave's ring slot `aslot` (lane l: row l % 16, columns 4 (l / 16) .. + 3 of the block), B
// fragments from the LDS weight buffer `buf` (this lane's first).  LAST: the transposed last
// block (k_pack_weight_kp) -- k-step e, lane group q takes column 4 e + q, i.e. element q of the
// piece lane 16 e + l % 16 copied -- and only its first `ns` k-steps (the others hold columns
// >= d only).
template <int NT, int RG, bool CLAMP>
__device__ __forceinline__ void rt_block(RAcc<NT> (&acc)[RG], const char* aslot, const f4* buf, bool LAST, int ns) {
  const int lane = threadIdx.x & 63;
  f4 a[RG];
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    if (!LAST) {
      a[g] = *reinterpret_cast<const f4*>(aslot + g * 1024 + lane * 16);
    } else {
      const float* t = reinterpret_cast<const float*>(aslot + g * 1024 + (lane & 15) * 16) + (lane >> 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[g][e] = t[64 * e];
    }
  }
  constexpr int JQ = (NT + 3) / 4;  // fragment quads a k-step reads
  f4 b[2][4];
#pragma unroll
  for (int jq = 0; jq < JQ; ++jq) b[0][jq] = buf[jq * 64];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (s >= ns) break;  // wave-uniform
    if (s + 1 < ns) {
#pragma unroll
      for (int jq = 0; jq < JQ; ++jq) b[(s + 1) & 1][jq] = buf[((s + 1) * 4 + jq) * 64];
    }
    // k-step s + 1's fragment reads stay ahead of k-step s's MFMAs (the scheduler would
    // otherwise sink each read to its first use and wait for it there)
    __builtin_amdgcn_sched_barrier(0);
    float as[RG];
#pragma unroll
    for (int g = 0; g < RG; ++g) as[g] = CLAMP ? clampf(a[g][s], -10.f, 10.f) : a[g][s];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g = 0; g < RG; ++g)
        acc[g].t[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(as[g], b[s & 1][t >> 2][t & 3], acc[g].t[t], 0, 0, 0);
  }
}

// acc[g] += A_g[16 rows x K] @ W for the wave's RG row groups: A row of lane l in group g =
// row arow[g] of the row-major matrix A (row l % 16 of the group), rows with !aok[g] read as 0,
// CLAMP: A clamped to +-10 (the time gate's operand); Wp packed by k_pack_weight_kp.  Both
// operands stream through LDS by DMA (buffer_load ... lds), nothing through registers: k-block
// kb + 1 of the weight (16 KB, a quarter per wave, double-buffered) and k-block kb + 2 of the
// wave's own A fragments (1 KB per group, each lane DMAs the 16 bytes it later reads: a 3-deep
// ring) are in flight while k-block kb's MFMAs run; every B fragment read feeds RG MFMAs.  The
// per-lane byte offsets are fixed for the whole product and the k-block advances the scalar
// offset only (no per-k-block address VALU); a masked row gets an offset past the resource's
// records, which the hardware reads as zeros.  Columns >= d of the last block read the next
// row's floats, which no k-step uses (the transposed last block: rt_block).  One raw barrier per
// k-block after a counted vmcnt (the A block two ahead may stay in flight across it;
// __syncthreads would drain it).  Every wave of the workgroup must call this with the same Wp
// and KB.  The last k-block runs only its k-steps that hold columns < d (rt_block).
constexpr uint32_t RT_OOB = 0xFFFF0000u;  // A offset of a masked row (+ any k-block: still past)
// one 16-B piece per lane, buffer -> LDS at `dst` (wave-uniform) + 16 lane
__device__ __forceinline__ void rt_dma16(__amdgpu_buffer_rsrc_t r, char* dst, uint32_t voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)dst, 16, voff, soff, 0, 0);
}
template <int NT, int RG, bool CLAMP>
__device__ __forceinline__ void rt_mm(RAcc<NT> (&acc)[RG], const float* A, const int (&arow)[RG], const bool (&aok)[RG],
                                      const float* __restrict__ Wp, int d, int KB, char* lds) {
  const int lane = threadIdx.x & 63, q = lane >> 4, w = wave_id();
  constexpr int A_SLOT = 4 * RG * 1024;
  char* wbuf = lds;
  char* abuf = lds + 2 * RT_KB_BYTES + w * RG * 1024;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Wp), (short)0, KB * RT_KB_BYTES, 0x00020000);
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), (short)0, (int)RT_OOB,
                                                                      0x00020000);
  const uint32_t wo = (uint32_t)(w * (RT_KB_BYTES / 4) + lane * 16);
  uint32_t ao[RG];
#pragma unroll
  for (int g = 0; g < RG; ++g) ao[g] = aok[g] ? ((uint32_t)arow[g] * (uint32_t)d + 4u * q) * 4u : RT_OOB;
  const int nlast = (d - 16 * (KB - 1) + 3) >> 2;  // k-steps of the last block with columns < d
  auto dma_w = [&](int kb) {  // this wave's quarter of k-block kb into buffer kb & 1
    char* dst = wbuf + (kb & 1) * RT_KB_BYTES + w * (RT_KB_BYTES / 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) rt_dma16(wr, dst + i * 1024, wo + i * 1024, kb * RT_KB_BYTES);
  };
  auto dma_a = [&](int kb) {  // lane l: A_g[row l % 16][16 kb + 4 (l / 16) ...] into ring slot kb % 3
#pragma unroll
    for (int g = 0; g < RG; ++g) rt_dma16(ar, abuf + (kb % RT_A_RING) * A_SLOT + g * 1024, ao[g], kb * 64);
  };
  dma_a(0);
  dma_w(0);
  if (KB > 1) dma_a(1);
  for (int kb = 0; kb < KB; ++kb) {
    // this wave's copies of k-block kb have landed (A of kb + 1, issued after them, may not);
    // after the barrier every wave's have, and every wave has read buffers kb - 1
    if (kb + 1 < KB) {
      if constexpr (RG == 1) asm volatile("s_waitcnt vmcnt(1)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (kb + 1 < KB) dma_w(kb + 1);
    if (kb + 2 < KB) dma_a(kb + 2);
    const char* aslot = abuf + (kb % RT_A_RING) * A_SLOT;
    const f4* buf = reinterpret_cast<const f4*>(wbuf + (kb & 1) * RT_KB_BYTES) + lane;
    const bool last = kb + 1 == KB;
    rt_block<NT, RG, CLAMP>(acc, aslot, buf, last, last ? nlast : 4);
  }
  // every wave has read the last buffers before a following call refills them
  asm volatile("s_barrier" ::: "memory");
}

// ---- per-row maps on the wave's 16 rows (lane l: rows 4 (l / 16) + r, column 16 t + l % 16)
template <int NT>
__device__ __forceinline__ void rt_sumsq(const RAcc<NT>& a, float n2[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) s += a.t[t][r] * a.t[t][r];
    n2[r] = row16_sum(s);
  }
}

template <int NT>
__device__ __forceinline__ void rt_scale(RAcc<NT>& a, const float f[4]) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) a.t[t][r] *= f[r];
}

// Row maps with the scaling deferred: m2 = |row|^2 and pf = the factor not yet multiplied into
// the row's elements, both for the lane's own row (own_row: lane l holds row l & 3 of its
// quarter).  A chain of maps (exp0 + project, project, log0, F.normalize, the radius) updates
// the two scalars only; rt_apply then multiplies the product of the chain's factors in, one
// pass over the row's elements instead of one per map (the step tail's chains of 6 and 4).
struct RtLazy {
  float m2, pf;
};
__device__ __forceinline__ void lz_scale(RtLazy& z, float f) {
  z.pf *= f;
  z.m2 *= f * f;
}
__device__ __forceinline__ void lz_project(RtLazy& z, const Curv& k) { lz_scale(z, project_factor(z.m2, k)); }
__device__ __forceinline__ void lz_log0(RtLazy& z, const Curv& k) { lz_scale(z, log0_factor(z.m2, k)); }
__device__ __forceinline__ void lz_exp0(RtLazy& z, const Curv& k) {  // exp0 + project
  float o;
  z.pf *= exp0_factor(z.m2, k, &o);
  z.m2 = o;
}
__device__ __forceinline__ void lz_normalize(RtLazy& z) {  // F.normalize, eps 1e-12
  lz_scale(z, frcp(fmaxf(fsqrt(z.m2), 1e-12f)));
}
template <int NT>
__device__ __forceinline__ void rt_apply(RAcc<NT>& a, RtLazy& z) {
  float f[4];
  spread_rows(z.pf, f);
  rt_scale(a, f);
  z.pf = 1.f;
}

// C-layout rows of a row-major matrix (columns >= d and rows past n_valid read 0)
template <int NT>
__device__ __forceinline__ void rt_load(RAcc<NT>& a, const float* __restrict__ M, const int crow[4], int n_valid,
                                        int d) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const bool ok = 4 * (lane >> 4) + r < n_valid;
    const int64_t base = (int64_t)crow[r] * d;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = 16 * t + (lane & 15);
      const float v = M[base + min(col, d - 1)];
      a.t[t][r] = (ok & (col < d)) ? v : 0.f;
    }
  }
}

template <int NT>
__device__ __forceinline__ void rt_store(const RAcc<NT>& a, float* __restrict__ M, const int crow[4], int n_valid,
                                         int d) {
  const int lane = threadIdx.x & 63;
  if (n_valid == 16 && d > 16 * (NT - 1)) {
    // (wave-uniform) all 16 rows valid and every tile but the last inside d: no masks, one row
    // address per row and the column tiles as immediate offsets (16 t floats)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float* row = M + (int64_t)crow[r] * d + (lane & 15);
#pragma unroll
      for (int t = 0; t < NT - 1; ++t) row[16 * t] = a.t[t][r];
      if (16 * (NT - 1) + (lane & 15) < d) row[16 * (NT - 1)] = a.t[NT - 1][r];
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (4 * (lane >> 4) + r >= n_valid) continue;
    float* row = M + (int64_t)crow[r] * d + (lane & 15);
#pragma unroll
    for (int t = 0; t < NT; ++t)  // a tile wholly inside d stores unmasked (a wave-uniform test)
      if (16 * t + 15 < d || 16 * t + (lane & 15) < d) row[16 * t] = a.t[t][r];
  }
}

// lane l: column 16 t + (l & 15) of the d-vector v for each column tile t, through a buffer
// resource of d floats: the tile is an immediate offset and columns >= d read 0 (no clamped
// address or select per load)
template <int NT>
__device__ __forceinline__ void rt_col(float out[NT], const float* __restrict__ v, int d) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(v), (short)0, d * 4, 0x00020000);
  const int vo = (int)(threadIdx.x & 15) * 4;
#pragma unroll
  for (int t = 0; t < NT; ++t) out[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo + 64 * t, 0, 0));
}

__device__ __forceinline__ void rt_store_radius(const float n2[4], float* __restrict__ rad, const int crow[4],
                                                int n_valid) {
  const int lane = threadIdx.x & 63;
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * (lane >> 4) + r < n_valid) rad[crow[r]] = row_radius(n2[r]);
  }
}

// The halo exchange's send block (regcn_layer_desc.send_*): row id i of the launch also goes to
// slots send_pos[send_ptr[i - send_lo] ..] -- its |h| and, after log0, its x row -- so no gather
// kernel re-reads the rows after the tail (parallel.exchange_halo).  Rows outside the block's
// id range have no slots.
__device__ __forceinline__ void rt_send_span(const LayerArgs& p, int rid, int& s0, int& s1) {
  const int64_t li = (int64_t)rid - p.send_lo;
  const bool in = li >= 0 && li < p.send_n;
  s0 = in ? p.send_ptr[li] : 0;
  s1 = in ? p.send_ptr[li + 1] : 0;
}

__device__ __forceinline__ void rt_send_radius(const LayerArgs& p, const float n2[4], const int crow[4], int n_valid) {
  const int lane = threadIdx.x & 63;
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (4 * (lane >> 4) + r >= n_valid) continue;
      int s0, s1;
      rt_send_span(p, crow[r], s0, s1);
      const float v = row_radius(n2[r]);  // = rt_store_radius's value
      for (int sl = s0; sl < s1; ++sl) p.send_r[p.send_pos[sl]] = v;
    }
  }
}

__device__ __forceinline__ int own_int(const int v[4]) {
  const bool b0 = threadIdx.x & 1, b1 = threadIdx.x & 2;
  const int lo = b0 ? v[1] : v[0], hi = b0 ? v[3] : v[2];
  return b1 ? hi : lo;
}

// The layer of the rows rows[64 b + 16 w ...] (wave w of workgroup b): v = clamp(agg @ W_n)
// (or clamp(agg): Lorentz; no clamps: euclid) + x @ (W_loop | W_evolve) -> clamp -> rrelu ->
// exp0; then the next layer's x / |h|, or the timestep (hyperbolic_model.py:829-869: project,
// layer norm, time gate, exp0, project, radius evolution / static radius).
// MODE: RT_LAYER; RT_GATE = RT_LAYER + the timestep's time-gate pre-activation clamp(x) @ W_g
// into gate_out (a cell's first layer: x is the timestep input); RT_STEP = the last layer with
// the timestep, its gate product in-kernel; RT_STEP_PRE = with the gate rows from RT_GATE (the
// blend reads them per column tile: no second accumulator set, half the registers).
enum { RT_LAYER = 0, RT_GATE = 1, RT_STEP = 2, RT_STEP_PRE = 3 };

// Stage layout of the step layer's blend operands and of the staged row stores: per column
// stage of RT_SC_COLS (80) and array, 16-B piece sc of row `row` sits at float
// 256 (sc >> 2) + 16 pi(row) + 4 (sc & 3), pi(row) = (row >> 2) + 4 (row & 3).  Lane l of the
// i-th 1-KB copy moves piece 4 i + (l & 3) of row rt_stage_row(l) (pi of it = l >> 2), so a
// copy is contiguous in LDS (global_load_lds puts lane l's 16 B at 16 l), a lane's row id is
// one shuffle per kernel, and the C-layout element (row 4 q + r, stage column 16 t + c) sits at
// 256 t + 64 r + 16 q + c = 256 t + 64 r + lane: conflict-free element reads and writes.  (A
// row-major stage divided the slot by the row width per piece -- ~20 VALU and a shuffle + LDS
// round trip per 16 B -- and its element accesses, rows 320 B apart, hit one bank 4 ways.)
__device__ __forceinline__ int rt_stage_row(int lane) {
  const int p = lane >> 2;
  return 4 * (p & 3) + (p >> 2);
}

// One 16-row group of a wave: its row ids (C layout), counts and A-operand row; stage_rid /
// stage_ok: the row this lane moves in the stage copies (rt_stage_row).
struct RtRows {
  int base, n_valid, arow_id, npos_w, stage_rid;
  bool a_valid, a_pos, stage_ok;
  int crow[4];
};

__device__ __forceinline__ RtRows rt_rows(const LayerArgs& p, int base) {
  const int lane = threadIdx.x & 63, q = lane >> 4, my_i = lane & 15;
  RtRows R;
  R.base = base;
  R.n_valid = max(0, min(16, p.V - base));  // p.V: the length of the row list
  R.arow_id = p.rows[min(base + min(my_i, max(R.n_valid - 1, 0)), p.V - 1)];
  R.a_valid = my_i < R.n_valid;
  R.a_pos = R.a_valid & (base + my_i < p.n_pos);
#pragma unroll
  for (int r = 0; r < 4; ++r) R.crow[r] = __shfl(R.arow_id, 4 * q + r);
  R.npos_w = min(max(p.n_pos - base, 0), R.n_valid);
  R.stage_rid = __shfl(R.arow_id, rt_stage_row(lane));
  R.stage_ok = rt_stage_row(lane) < R.n_valid;
  return R;
}

// The step layer's blend operands (x_prev and the gate rows) in column stages of RT_SC_COLS:
// each wave DMAs its 16 rows' columns [RT_SC_COLS s, ...) of both arrays into its own LDS
// region (the stage layout above; 16-B pieces, global_load_lds, <= 5 instructions per array),
// then reads them in C layout -- instead of 2 x NT x 4 scattered 4-B loads per lane.  The
// region is the products' LDS (free after rt_mm's final barrier): 4 waves x 2 arrays x 5 KB.
constexpr int RT_SC_COLS = 80, RT_SC_TILES = RT_SC_COLS / 16, RT_SC_BYTES = 16 * RT_SC_COLS * 4;
static_assert(4 * 2 * RT_SC_BYTES <= rt_lds_bytes(1), "blend staging must fit the tail's LDS");
static_assert(RT_SC_BYTES == RT_SC_TILES * 1024, "a stage is RT_SC_TILES 1-KB copies per array");

__device__ __forceinline__ void rt_stage_blend(const StepArgs& s, const RtRows& R, int d, int dpad, int stage,
                                               char* lds) {
  const int lane = threadIdx.x & 63, w = wave_id();
  // the stage spans the padded width (16 NT columns): columns >= d are staged as zeros, so the
  // blend reads every column of its tiles unmasked
  const int c0 = RT_SC_COLS * stage, ncols = min(RT_SC_COLS, dpad - c0), f4pr = ncols >> 2;
  const float* zrow = reinterpret_cast<const float*>(kZeroRow);
  char* base = lds + w * 2 * RT_SC_BYTES;
  const int64_t off = (int64_t)R.stage_rid * d + c0 + 4 * (lane & 3);
#pragma unroll
  for (int i = 0; i < RT_SC_TILES; ++i) {
    if (4 * i >= f4pr) break;  // (dpad and stage are compile-time: the stage's copies)
    const int sc = 4 * i + (lane & 3);
    const bool ok = R.stage_ok & (sc < f4pr) & (c0 + 4 * sc < d);
    __builtin_amdgcn_global_load_lds((const void*)(ok ? s.x_prev + off + 16 * i : zrow),
                                     (__attribute__((address_space(3))) void*)(base + i * 1024), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(ok ? s.tw + off + 16 * i : zrow),
                                     (__attribute__((address_space(3))) void*)(base + RT_SC_BYTES + i * 1024), 16, 0, 0);
  }
}

// C-layout rows stored through the wave's LDS region in the same 80-column stages (the stage
// layout): written there per element, read back as 16-B row pieces (one contiguous
// ds_read_b128 per copy), stored as whole 16-B vectors instead of NT x 4 scattered 4-B stores.
// In-order LDS within the wave: no barrier.  Pad columns are written (never stored).
// send: also into p's send block (every slot of the row, rt_send_span)
template <int NT>
__device__ __forceinline__ void rt_store_staged(const RAcc<NT>& a, float* __restrict__ M, const RtRows& R, int d,
                                                char* lds, const LayerArgs& p, bool send) {
  const int lane = threadIdx.x & 63;
  float* st = reinterpret_cast<float*>(lds + wave_id() * 2 * RT_SC_BYTES);
  constexpr int NS = (NT + RT_SC_TILES - 1) / RT_SC_TILES;
  float* mrow = M + (int64_t)R.stage_rid * d + 4 * (lane & 3);
  int s0 = 0, s1 = 0;
  if (send) rt_send_span(p, R.stage_rid, s0, s1);
#pragma unroll
  for (int stage = 0; stage < NS; ++stage) {
    const int c0 = RT_SC_COLS * stage;
    if (c0 >= d) break;
    const int f4pr = min(RT_SC_COLS, d - c0) >> 2;
    const int t0 = stage * RT_SC_TILES;
#pragma unroll
    for (int t = t0; t < min(NT, t0 + RT_SC_TILES); ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) st[256 * (t - t0) + 64 * r + lane] = a.t[t][r];
    constexpr int NI = RT_SC_TILES;
    f4 val[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i)
      if (t0 + i < NT) val[i] = *reinterpret_cast<const f4*>(st + 256 * i + 4 * lane);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (t0 + i < NT && R.stage_ok && 4 * i + (lane & 3) < f4pr) {
        *reinterpret_cast<f4*>(mrow + c0 + 16 * i) = val[i];
        for (int sl = s0; sl < s1; ++sl)
          *reinterpret_cast<f4*>(p.send_x + (int64_t)p.send_pos[sl] * d + c0 + 16 * i + 4 * (lane & 3)) = val[i];
      }
    }
  }
}

// Everything after the products for one 16-row group: clamps, rrelu, exp0, then the next
// layer's x / |h| or the timestep.  `g` (RT_STEP) holds the in-kernel gate product.
template <int NT, int MODE>
__device__ __forceinline__ void rt_finish(const LayerArgs& p, RAcc<NT>& v, const RtRows& R, const RAcc<NT>* g,
                                          char* lds, RtStamps* sp = nullptr) {
  constexpr bool STEP = MODE >= RT_STEP;
  const int lane = threadIdx.x & 63, q = lane >> 4, d = p.d;
  const int* crow = R.crow;
  const int n_valid = R.n_valid;
  // the first blend stage's copies fly under the epilogue's row maps
  if constexpr (MODE == RT_STEP_PRE) rt_stage_blend(p.step, R, d, 16 * NT, 0, lds);
  // the clamp as bounds (+-inf: none, Euclid) -- a runtime test per element would be a select
  const float cb = p.euclid ? __builtin_inff() : 10.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) v.t[t] = leaky4(clamp4(v.t[t], -cb, cb));
  float n2[4];
  RtLazy z{0.f, 1.f};
  if (!p.euclid || p.r_next) {
    rt_sumsq<NT>(v, n2);
    z.m2 = own_row(n2);
  }
  if (!p.euclid) lz_exp0(z, p.k);

  if constexpr (!STEP) {
    if (p.h_out) {
      if (!p.euclid) rt_apply<NT>(v, z);
      rt_store<NT>(v, p.h_out, crow, n_valid, d);
    }
    spread_rows(z.m2, n2);
    if (p.r_next) rt_store_radius(n2, p.r_next, crow, n_valid);
    if (p.send_x) rt_send_radius(p, n2, crow, n_valid);
    if (p.x_next) {
      if (!p.euclid) {
        lz_log0(z, p.k);
        rt_apply<NT>(v, z);
      }
      // staged like the step layer's rows (element stores: 2,062 vs 2,052 us at config 5,
      // profiles/r6_stage_layout_ab.jsonl)
      rt_store_staged<NT>(v, p.x_next, R, d, lds, p, p.send_x != nullptr);
    }
  } else {
    const StepArgs& s = p.step;
    const Curv k = s.k;
    // the radius step's operands, loaded now: their latency (r_static is an HBM row read) would
    // otherwise sit between the blend and the stores
    const float rs = s.r_static[own_int(crow)];
    const float br = s.residual ? *s.b_r : 0.f;
    float wr[NT], bg[NT];
    if (s.residual) rt_col<NT>(wr, s.w_r, d);
    rt_col<NT>(bg, s.b_g, d);  // (the blend's gate bias: in flight under the row maps too)
    lz_project(z, k);
    if (s.layer_norm) {
      lz_log0(z, k);
      lz_normalize(z);
      lz_exp0(z, k);
    }
    lz_log0(z, k);
    rt_apply<NT>(v, z);
    if (sp) sp->mark(1);
    if constexpr (MODE == RT_STEP_PRE) {
      const float* xs = reinterpret_cast<const float*>(lds + wave_id() * 2 * RT_SC_BYTES);
      const float* zs = xs + RT_SC_BYTES / 4;
      // sigmoid(z + b) = 1 / (1 + 2^(z (-log2 e) + b (-log2 e)))
      float nbg[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) nbg[t] = bg[t] * -FM_LOG2E;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int stage = t / RT_SC_TILES;
        if (t % RT_SC_TILES == 0) {
          if (stage > 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the last stage
            rt_stage_blend(s, R, d, 16 * NT, stage, lds);
          }
          if (sp) sp->mark(3);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stage's copies have landed
          if (sp) sp->mark(2);
        }
        // rows past n_valid and columns >= d were staged as zeros (pad columns: v, x_prev and the
        // gate row all 0 there, so the blend keeps them 0; such rows are never stored)
        const int tt = t - RT_SC_TILES * stage;  // the stage layout: element at 256 tt + 64 r + lane
        const f4 c4 = clamp4(v.t[t], -10.f, 10.f);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xp = xs[256 * tt + 64 * r + lane];
          const float zt = zs[256 * tt + 64 * r + lane];
          const float pr = clampf(xp, -10.f, 10.f);
          const float gg = frcp(1.f + __builtin_amdgcn_exp2f(fmaf(zt, -FM_LOG2E, nbg[t])));
          v.t[t][r] = fmaf(gg, c4[r] - pr, pr);  // gg c4 + (1 - gg) pr
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int col = 16 * t + (lane & 15), colc = min(col, d - 1);
        const f4 c4 = clamp4(v.t[t], -10.f, 10.f);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = (4 * q + r < n_valid) & (col < d);
          const float xp = s.x_prev[(int64_t)crow[r] * d + colc];
          const float pr = fminf(fmaxf(ok ? xp : 0.f, -10.f), 10.f);
          const float gg = sigmoidf(g->t[t][r] + bg[t]);
          v.t[t][r] = gg * c4[r] + (1.f - gg) * pr;
        }
      }
    }
    if (sp) sp->mark(3);
    rt_sumsq<NT>(v, n2);
    z.m2 = own_row(n2);
    lz_exp0(z, k);
    lz_project(z, k);  // hyperbolic_model.py:860
    // radius: per-row scalars once per lane, for its own row r = lane & 3 (own_row)
    const float n2o = z.m2;
    float newr = rs;
    if (s.residual) {
      float lf[4], dl[4];
      // w_r . log0(v pf) = (pf log0 factor) (w_r . v): the row's factor applied to the dot
      spread_rows(z.pf * log0_factor(n2o, s.k_rad), lf);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) acc = fmaf(wr[t], v.t[t][r], acc);
        dl[r] = row16_sum(acc) * lf[r];
      }
      const float delta = fminf(fmaxf(own_row(dl) + br, -s.eps_r), s.eps_r);
      const float dyn = row_radius(n2o);
      newr = (s.beta * rs + (1.f - s.beta) * dyn) + delta;
    }
    const Curv kr = s.residual ? s.k_rad : s.k;
    lz_scale(z, fdiv(fminf(fmaxf(newr, REGCN_EPS), kr.rmax), row_radius(n2o)));
    if (sp) sp->mark(4);
    if (s.h_out) {
      rt_apply<NT>(v, z);
      rt_store_staged<NT>(v, s.h_out, R, d, lds, p, false);
    }
    spread_rows(z.m2, n2);
    if (s.r_out) rt_store_radius(n2, s.r_out, crow, n_valid);
    if (p.send_x) rt_send_radius(p, n2, crow, n_valid);
    if (sp) sp->mark(5);
    if (s.x_out) {
      lz_log0(z, k);
      rt_apply<NT>(v, z);
      rt_store_staged<NT>(v, s.x_out, R, d, lds, p, p.send_x != nullptr);
    }
    if (sp) sp->mark(6);
  }
}

// The layer of the rows rows[64 RG b + 16 (RG w + g) ...] (wave w of workgroup b, group g): v =
// clamp(agg @ W_n) (or clamp(agg): Lorentz; no clamps: euclid) + x @ (W_loop | W_evolve) ->
// clamp -> rrelu -> exp0; then the next layer's x / |h|, or the timestep
// (hyperbolic_model.py:829-869: project, layer norm, time gate, exp0, project, radius
// evolution / static radius).  MODE: RT_LAYER; RT_GATE = RT_LAYER + the timestep's time-gate
// pre-activation clamp(x) @ W_g into gate_out (a cell's first layer: x is the timestep input);
// RT_STEP = the last layer with the timestep, its gate product in-kernel (RG = 1 only);
// RT_STEP_PRE = with the gate rows from RT_GATE (the blend reads them per column tile).
template <int NT, int MODE, int RG>
__device__ __forceinline__ void rowtail_body(const LayerArgs& p, int row0) {
  static_assert(MODE != RT_STEP || RG == 1, "the in-kernel gate product runs on one row group");
  extern __shared__ char rt_lds[];
  RtStamps st;
  st.start();
  const int w = wave_id();
  const int wg0 = row0 + blockIdx.x * RT_ROWS * RG;
  const int d = p.d, KB = (d + 15) >> 4;
  RtRows R[RG];
#pragma unroll
  for (int g = 0; g < RG; ++g) R[g] = rt_rows(p, wg0 + 16 * (RG * w + g));
  // the passes are the workgroup's (every wave takes part in each weight's LDS stream)
  const int n_wg = min(RT_ROWS * RG, p.V - wg0);
  const int npos_wg = min(max(p.n_pos - wg0, 0), n_wg);
  int arow[RG];
  bool valid[RG];
#pragma unroll
  for (int g = 0; g < RG; ++g) arow[g] = R[g].arow_id, valid[g] = R[g].a_valid;

  RAcc<NT> v[RG];
  if constexpr (MODE == RT_GATE) {  // the timestep's gate pre-activation, stored as is
#pragma unroll
    for (int g = 0; g < RG; ++g) v[g].zero();
    rt_mm<NT, RG, true>(v, p.x, arow, valid, p.w_gate, d, KB, rt_lds);
#pragma unroll
    for (int g = 0; g < RG; ++g) rt_store_staged<NT>(v[g], p.gate_out, R[g], d, rt_lds, p, false);
    __syncthreads();  // the waves' staging regions overlap the next product's first copies
  }
#pragma unroll
  for (int g = 0; g < RG; ++g) v[g].zero();
  // The products into v, one call site (one copy of the MFMA loop, one accumulator set):
  // pass 0 = agg @ W_n (in-edge rows), then x @ W_loop / x @ W_evolve -- both in the one
  // workgroup where the in-edge rows end (rows masked), one of them everywhere else.
  const bool p1 = npos_wg > 0 && p.agg != nullptr;
  if (p1 && !p.w_n) {  // Lorentz: the centroid rows as is
#pragma unroll
    for (int g = 0; g < RG; ++g) rt_load<NT>(v[g], p.agg, R[g].crow, R[g].npos_w, d);
  }
  const bool mixed = npos_wg > 0 && npos_wg < n_wg;
  const int first = (p1 && p.w_n) ? 0 : 1;
  const int last = p.w_loop ? (mixed ? 3 : 2) : 1;
  for (int pass = first; pass < last; ++pass) {
    if (pass == 1 && p1 && !p.euclid) {
#pragma unroll
      for (int g = 0; g < RG; ++g)
#pragma unroll
        for (int t = 0; t < NT; ++t) v[g].t[t] = clamp4(v[g].t[t], -10.f, 10.f);
    }
    bool ok[RG];
#pragma unroll
    for (int g = 0; g < RG; ++g)
      ok[g] = pass == 0 ? R[g].a_pos : (mixed ? (pass == 1 ? R[g].a_pos : R[g].a_valid & !R[g].a_pos) : R[g].a_valid);
    const float* W = pass == 0 ? p.w_n : (pass == 1 && npos_wg > 0 ? p.w_loop : p.w_evolve);
    rt_mm<NT, RG, false>(v, pass == 0 ? p.agg : p.x, arow, ok, W, d, KB, rt_lds);
  }
  if (((first == 0 && last == 1) || (first == 1 && last == 1 && p1)) && !p.euclid) {
    // agg @ W_n without a self loop, or Lorentz rows without one
#pragma unroll
    for (int g = 0; g < RG; ++g)
#pragma unroll
      for (int t = 0; t < NT; ++t) v[g].t[t] = clamp4(v[g].t[t], -10.f, 10.f);
  }
  if constexpr (MODE == RT_STEP) {  // the time gate pre-activation clamp(x_prev) @ W_g
    RAcc<NT> gt[1];
    gt[0].zero();
    const int xr[1] = {R[0].arow_id};
    const bool okp[1] = {R[0].a_valid};
    rt_mm<NT, 1, true>(gt, p.step.x_prev, xr, okp, p.step.w_g, d, KB, rt_lds);
    rt_finish<NT, MODE>(p, v[0], R[0], &gt[0], rt_lds);
  } else {
    st.mark(0);
#pragma unroll
    for (int g = 0; g < RG; ++g)
      rt_finish<NT, MODE>(p, v[g], R[g], nullptr, rt_lds, (kRtStamps && MODE == RT_STEP_PRE) ? &st : nullptr);
    if constexpr (MODE == RT_STEP_PRE) st.write(p.trace);
  }
}

template <int NT, int MODE, int RG>
__global__ __launch_bounds__(NTHR) void k_rowtail(LayerArgs p, int row0) {
  rowtail_body<NT, MODE, RG>(p, row0);
}

// two row groups per wave at two waves per SIMD
template <int NT, int MODE>
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(2))) void k_rowtail2(LayerArgs p, int row0) {
  rowtail_body<NT, MODE, 2>(p, row0);
}

// the timestep variant with the gate rows precomputed at three waves per SIMD (the compiler
// otherwise keeps ~170 VGPRs of blend loads in flight and the kernel runs at two)
template <int NT, int MODE>
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(3))) void k_rowtail3(LayerArgs p, int row0) {
  rowtail_body<NT, MODE, 1>(p, row0);
}

// ----------------------------------------------------------------------------- launchers
template <int AGG, int S>
static void launch_gather(const LayerArgs& a, float* out, int t0, int t1, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((k_gather_agg<AGG, S>), dim3(t1 - t0), dim3(NTHR), lds, st, a, out, t0);
}

// Row groups per wave of the layer tails (d > 128): 2 (default) = every B fragment feeds two
// MFMAs at 2 waves / SIMD; REGCN_ROWTAIL_RG=1: one group at 3 waves / SIMD.  Config 5
// (profiles/r4_rowtail_rg_kernel_stats.csv): first-layer tail 2.41 vs 2.55 ms; the step
// layer's tail is the same either way (1.99 ms) and keeps its one-group kernel.
static int rowtail_rg() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("REGCN_ROWTAIL_RG");
    v = e ? atoi(e) : 2;
  }
  return v;
}

// Rows from which a launch takes two groups per wave (REGCN_RT_RG2_MIN_ROWS overrides: a rank's
// chunk tails that run two at a time on two streams fill the chip with fewer rows each).
static int rt_rg2_min_rows() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("REGCN_RT_RG2_MIN_ROWS");
    v = e ? atoi(e) : 256 * 1024;
  }
  return v;
}

// REGCN_STEP_RG=2: the step layer's tail with two row groups per wave too (A/B; default one)
static int step_rg() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("REGCN_STEP_RG");
    v = e ? atoi(e) : 1;
  }
  return v;
}

template <int NT>
static int launch_tail(const LayerArgs& a, int r0, int r1, hipStream_t st) {
  // two groups only when the launch still fills the chip with 128-row workgroups (a rank's
  // slice of an owner-partitioned snapshot runs one group per wave: more, shorter workgroups)
  const int rg = (NT > 8 && rowtail_rg() == 2 && r1 - r0 >= rt_rg2_min_rows()) ? 2 : 1;
  const unsigned grid = (unsigned)((r1 - r0 + RT_ROWS * rg - 1) / (RT_ROWS * rg));
  const size_t lds = rt_lds_bytes(rg);
  if (kRtStamps && a.fuse_step && a.step.tw) const_cast<LayerArgs&>(a).trace = g_trace;
  if (a.fuse_step && a.step.tw && rg == 2 && step_rg() == 2) {
    hipLaunchKernelGGL((k_rowtail2<NT, RT_STEP_PRE>), dim3(grid), dim3(NTHR), lds, st, a, r0);
  } else if (a.fuse_step && a.step.tw) {
    hipLaunchKernelGGL((k_rowtail3<NT, RT_STEP_PRE>), dim3((r1 - r0 + RT_ROWS - 1) / RT_ROWS), dim3(NTHR),
                       rt_lds_bytes(1), st, a, r0);
  } else if (a.fuse_step) {
    hipLaunchKernelGGL((k_rowtail<NT, RT_STEP, 1>), dim3((r1 - r0 + RT_ROWS - 1) / RT_ROWS), dim3(NTHR),
                       rt_lds_bytes(1), st, a, r0);
  } else if (a.gate_out) {
    if (rg == 2) hipLaunchKernelGGL((k_rowtail2<NT, RT_GATE>), dim3(grid), dim3(NTHR), lds, st, a, r0);
    else hipLaunchKernelGGL((k_rowtail<NT, RT_GATE, 1>), dim3(grid), dim3(NTHR), lds, st, a, r0);
  } else {
    if (rg == 2) hipLaunchKernelGGL((k_rowtail2<NT, RT_LAYER>), dim3(grid), dim3(NTHR), lds, st, a, r0);
    else hipLaunchKernelGGL((k_rowtail<NT, RT_LAYER, 1>), dim3(grid), dim3(NTHR), lds, st, a, r0);
  }
  return 0;
}

// which == 1: the gather over tiles [lo, hi); which == 2: the tail over rows[lo, hi) (hi <= a.V);
// which == 3: both, all tiles and rows.
int layer_rowtail_part(const LayerArgs& a, float* agg, int which, int lo, int hi, hipStream_t st);

int layer_rowtail(const LayerArgs& a, float* agg, hipStream_t st) {
  return layer_rowtail_part(a, agg, 3, 0, 0, st);
}

int layer_rowtail_part(const LayerArgs& a, float* agg, int which, int lo, int hi, hipStream_t st) {
  const int mode = a.agg_mode;
  if (a.d <= 0 || a.d > MAX_D || (a.d & 3)) return set_error(REGCN_EINVAL, "rowtail needs d %% 4 == 0, d <= 256");
  // the products read x / agg / x_prev rows through 32-bit buffer offsets (rt_mm)
  if ((int64_t)a.V * a.d * 4 >= (int64_t)RT_OOB) return set_error(REGCN_ENOTSUP, "rowtail tables must stay under 4 GB");
  // a non-step layer may skip h (h_out NULL) when its consumer reads x_next and r_next only
  if (!a.x || !a.rows || (!a.h_out && !a.fuse_step && !a.x_next)) return set_error(REGCN_EINVAL, "null pointer");
  if ((a.w_loop == nullptr) != (a.w_evolve == nullptr)) return set_error(REGCN_EINVAL, "self-loop weights must come in pairs");
  if (a.prev_t || a.drop_mask) return set_error(REGCN_EINVAL, "rowtail has no skip gate / dropout mask (use regcn_layer_f32)");
  if (a.n_pos < 0 || a.n_pos > a.V) return set_error(REGCN_EINVAL, "bad n_pos");
  if (mode != AGG_NONE && mode != AGG_UNION && mode != AGG_EUCLID && mode != AGG_LORENTZ)
    return set_error(REGCN_EINVAL, "unknown aggregation mode %d", mode);
  if (a.n_pos > 0 && !agg) return set_error(REGCN_EINVAL, "rowtail needs the agg buffer");
  if (which < 1 || which > 3) return set_error(REGCN_EINVAL, "bad rowtail part");
  if ((mode == AGG_UNION || mode == AGG_EUCLID) && !a.w_n && a.n_pos > 0)
    return set_error(REGCN_EINVAL, "union / euclid rowtail needs w_n");
  if ((mode == AGG_UNION || mode == AGG_LORENTZ) && a.euclid) return set_error(REGCN_EINVAL, "hyperbolic gather with euclid tail");
  if ((a.gate_out == nullptr) != (a.w_gate == nullptr)) return set_error(REGCN_EINVAL, "gate_w and gate_out come in pairs");
  if (a.gate_out && a.fuse_step) return set_error(REGCN_EINVAL, "gate_out is for a cell's first layer, not the step layer");
  if (a.fuse_step) {
    const StepArgs& s = a.step;
    if (a.euclid) return set_error(REGCN_EINVAL, "the fused timestep is hyperbolic only");
    // the timestep may skip h (h_out NULL) when x_out is written (predict's earlier timesteps)
    if (!s.x_prev || !s.w_g || !s.b_g || !s.r_static || (!s.h_out && !s.x_out))
      return set_error(REGCN_EINVAL, "null timestep pointer");
    if (s.residual && (!s.w_r || !s.b_r)) return set_error(REGCN_EINVAL, "residual radius needs w_r and b_r");
  }
  if (a.V == 0) return 0;
  int t0 = 0, t1 = a.n_pos_tiles, r0 = 0, r1 = a.V;
  if (which == 1) {
    if (lo < 0 || hi > a.n_pos_tiles || lo > hi) return set_error(REGCN_EINVAL, "bad tile range");
    t0 = lo;
    t1 = hi;
  } else if (which == 2) {
    if (lo < 0 || hi > a.V || lo > hi) return set_error(REGCN_EINVAL, "bad row range");
    r0 = lo;
    r1 = hi;
  }
  if ((which & 1) && mode != AGG_NONE && t1 > t0) {
    if (!a.rowptr || !a.col_src || !a.col_type || !a.rel || !a.tiles || !a.item_ptr)
      return set_error(REGCN_EINVAL, "gather needs CSR, rel, tiles and item lists");
    if (mode == AGG_UNION && !a.radius) return set_error(REGCN_EINVAL, "union gather needs radius");
    if (mode != AGG_LORENTZ && !a.norm) return set_error(REGCN_EINVAL, "gather needs norm");
    if (mode == AGG_LORENTZ && (!a.w_rel || a.nb <= 0 || a.d % a.nb))
      return set_error(REGCN_EINVAL, "lorentz gather needs weights and d %% num_bases == 0");
    LayerArgs g = a;
    g.agg = agg;  // hub rows: read back (skipped) by the finish
    if ((mode == AGG_UNION || mode == AGG_EUCLID) && a.crel_tiles > 0 && t0 < a.crel_tiles) {
      if (!a.crel_item_src || !a.crel_item_tl || !a.rel_t) return set_error(REGCN_EINVAL, "crel needs its items and rel_t");
      if (a.n_types <= 0 || a.n_types > CREL_MAX_TYPES)
        return set_error(REGCN_ENOTSUP, "crel takes 1..%d relation types (got %d)", CREL_MAX_TYPES, a.n_types);
      if (a.crel_tiles > a.n_pos_tiles) return set_error(REGCN_EINVAL, "crel_tiles > n_pos_tiles");
      const int tc = std::min(t1, a.crel_tiles);
      LayerArgs c = g;
      c.item_src = a.crel_item_src;
      c.item_tl = a.crel_item_tl;
      const size_t lds_c = crel_lds_bytes(a.d, a.n_types);
      const bool eb32 = crel_eb() == 32;
      if (mode == AGG_UNION) {
        if (!a.radius) return set_error(REGCN_EINVAL, "union gather needs radius");
        if (eb32) hipLaunchKernelGGL((k_gather_crel<AGG_UNION, 32>), dim3(tc - t0), dim3(NTHR), lds_c, st, c, agg, t0);
        else hipLaunchKernelGGL((k_gather_crel<AGG_UNION, 16>), dim3(tc - t0), dim3(NTHR), lds_c, st, c, agg, t0);
      } else {
        if (eb32) hipLaunchKernelGGL((k_gather_crel<AGG_EUCLID, 32>), dim3(tc - t0), dim3(NTHR), lds_c, st, c, agg, t0);
        else hipLaunchKernelGGL((k_gather_crel<AGG_EUCLID, 16>), dim3(tc - t0), dim3(NTHR), lds_c, st, c, agg, t0);
      }
      const int rc = check_launch("k_gather_crel");
      if (rc) return rc;
      t0 = tc;
    }
    const int s = mode == AGG_LORENTZ ? a.d / a.nb : 1;
    const bool gen = mode == AGG_LORENTZ && s != 1 && s != 2 && s != 4;
    const size_t lds = (size_t)(((TM + NWAVE - 1) * tile_lda(a.d) + 32) + (gen ? NWAVE * MAX_D : 0)) * 4;
    if (t1 > t0) switch (mode) {
      case AGG_UNION: launch_gather<AGG_UNION, 1>(g, agg, t0, t1, lds, st); break;
      case AGG_EUCLID: launch_gather<AGG_EUCLID, 1>(g, agg, t0, t1, lds, st); break;
      default:
        if (s == 1) launch_gather<AGG_LORENTZ, 1>(g, agg, t0, t1, lds, st);
        else if (s == 2) launch_gather<AGG_LORENTZ, 2>(g, agg, t0, t1, lds, st);
        else if (s == 4) launch_gather<AGG_LORENTZ, 4>(g, agg, t0, t1, lds, st);
        else launch_gather<AGG_LORENTZ, 0>(g, agg, t0, t1, lds, st);
    }
    const int rc = check_launch("k_gather_agg");
    if (rc) return rc;
  }
  if (!(which & 2) || r1 <= r0) return 0;
  LayerArgs t = a;
  t.agg = agg;
  t.V = r1;
  if (mode == AGG_LORENTZ) t.w_n = nullptr;  // the centroid rows are the aggregation itself
  const int nt = (a.d + 15) / 16;
  if (nt <= 4) launch_tail<4>(t, r0, r1, st);
  else if (nt <= 8) launch_tail<8>(t, r0, r1, st);
  else if (nt <= 13) launch_tail<13>(t, r0, r1, st);
  else launch_tail<16>(t, r0, r1, st);
  return check_launch("k_rowtail");
}

}  // namespace regcn
