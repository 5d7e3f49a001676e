// CSR gather / segment-reduce kernels.
//
// Work decomposition.  The host (regcn_amd/graph.py) sorts a snapshot's edges by
// destination (stable, so ties keep the reference's edge order) and cuts every
// destination's edge list into chunks of at most `chunk_edges` edges:
//     chunk = {row, e_begin, e_end, slot}
// slot < 0: the row fits one chunk and the wave writes the finished row.
// slot >= 0: the wave writes a raw partial sum into partial[slot]; a fix-up
// kernel then sums each long row's partials in chunk order and finishes it.
// No atomics: results are bitwise reproducible run to run.
//
// One 64-lane wave per chunk; lane l owns columns [4l, 4l+4) (float4), so each
// gathered 800-B row (d = 200) is one coalesced wave load.  Edge indices of up
// to 64 edges are fetched cooperatively (one per lane) and broadcast with
// readlane; the row loads of 4 edges are issued before they are consumed.
//
// HBM roofline (Union, per layer): E*(4d + 12) + V*(4d + 12) algorithmic bytes
// (src row + col_src + col_type + radius_src per edge; output row + row
// metadata per node); relation rows and Lorentz blocks are L2-resident.
#include "common.h"
#include "gather.h"
#include "regcn_internal.h"

namespace regcn {

// ------------------------------------------------------------------------------ mean
// MEAN: acc = sum_e x[idx_e];  out = acc / count  (hyperbolic_model.py:802-812), one wave
// per chunk, 8 gathered rows in flight, unconditional loads (clamped column).
template <int MODE>
__global__ __launch_bounds__(256) void k_gather_sum(
    const float* __restrict__ x, const float* __restrict__ radius, const float* __restrict__ rel,
    const int* __restrict__ col_src, const int* __restrict__ col_type, const float* __restrict__ rowscale,
    const Chunk* __restrict__ chunks, int n_chunks, float gamma, int d, float* __restrict__ partial,
    int pstride, float* __restrict__ out) {
  static_assert(MODE == AGG_MEAN, "union / euclid: k_union_runs");
  const int lane = threadIdx.x & 63;
  const int col = lane * 4;
  const uint32_t off = (uint32_t)min(col, d - 4) * 4u;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int ci = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); ci < n_chunks; ci += nw) {
    const Chunk ch = chunks[ci];
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int e0 = ch.beg; e0 < ch.end; e0 += 64) {
      const int n = min(64, ch.end - e0);
      const int my_s = col_src[e0 + min(lane, n - 1)];
      int j = 0;
      for (; j + 8 <= n; j += 8) {
        f4 xs[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) xs[u] = row_load4(x + (int64_t)rl(my_s, j + u) * d, off);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += xs[u];
      }
      for (; j < n; ++j) acc += row_load4(x + (int64_t)rl(my_s, j) * d, off);
    }
    if (ch.slot < 0) store4(out + (int64_t)ch.row * d, col, d, acc / rowscale[ch.row]);
    else store4(partial + (int64_t)ch.slot * pstride, col, d, acc);
  }
}

// One 64-edge batch of a chunk in source order (lane = edge, my_s its source): a head lane
// starts a run of equal sources (cut at the batch end); its row is gathered once with weight
// count * w.  8 distinct rows in flight; a short last group repeats its first row with weight 0.
template <bool EUCLID>
__device__ __forceinline__ void src_runs_batch(const float* __restrict__ x, const float* __restrict__ radius,
                                               int my_s, float r_dst, float gamma, int d, uint32_t off, int lane,
                                               int n, uint64_t upto, f4& acc) {
  const float my_w = EUCLID ? 1.f : expf(-gamma * fabsf(radius[my_s] - r_dst));
  const int prev_s = __shfl_up(my_s, 1);
  const uint64_t hm = __ballot(lane < n && (lane == 0 || my_s != prev_s));
  const uint64_t after = hm & ~upto;
  const int nxt = after ? __builtin_ctzll(after) : n;
  const float wc = my_w * (float)(nxt - lane);  // count * w on a head lane
  uint64_t m = hm;
  while (m) {
    const int h0 = __builtin_ctzll(m);
    int hs[8];
    float wv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool ok = m != 0;
      hs[u] = ok ? __builtin_ctzll(m) : h0;
      wv[u] = ok ? rlf(wc, hs[u]) : 0.f;
      if (ok) m &= m - 1;
    }
    f4 xs[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) xs[u] = row_load4(x + (int64_t)rl(my_s, hs[u]) * d, off);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += wv[u] * xs[u];
  }
}

// UNION / EUCLID with relation-type runs.  By linearity
//   sum_e w_e (x[src_e] + rel[t_e]) = sum_e w_e x[src_e] + sum_runs (sum_{e in run} w_e) rel[t_run]
// over the maximal runs of equal type in the chunk's edge order.  A hub row's edges in
// row/type order (graph.row_type_cols: the fused layers' heavy rows) are a few long runs,
// so the relation rows are read once per run instead of once per edge: the per-edge load
// stream is the gathered source row alone (8 rows in flight per wave).  Any edge order is
// valid (CSR order: runs of about one edge, relation rows loaded 4 at a time).
// Per 64-edge batch, lane = edge: run heads by ballot, a segmented lane scan of the
// weights, then each closed run's relation row once; the batch's last run stays open
// into the next batch.  Deterministic (fixed lane and run order, no atomics).
//
// SRC_RUNS (col_src_s = the same rows' edges in source order, graph.row_src_cols): the
// source half runs over source runs instead.  w_e depends on (src, dst) only, so a row's
// duplicate sources (the same neighbour under several relations, or a repeated triple) sum
// to count * w * x[src]: one gathered row per distinct source of the batch.  The type
// pass then reads only (col_src, col_type) and radius[src] per edge (12 B, no rows).  Both
// orders permute each row's CSR span, so a chunk [beg, end) covers a different edge subset
// in each, and the row's chunks together still cover every edge exactly once per half.
template <bool EUCLID, bool SRC_RUNS>
__global__ __launch_bounds__(256) void k_union_runs(
    const float* __restrict__ x, const float* __restrict__ radius, const float* __restrict__ rel,
    const int* __restrict__ col_src, const int* __restrict__ col_type, const int* __restrict__ col_src_s,
    const float* __restrict__ rowscale, const Chunk* __restrict__ chunks, int n_chunks, float gamma, int d,
    float* __restrict__ partial, int pstride, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int col = lane * 4;
  // clamped column: lanes past d re-read the row's last quad (same cache lines, never
  // stored), so every row load is unconditional
  const uint32_t off = (uint32_t)min(col, d - 4) * 4u;
  const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);  // lanes 0..lane
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int ci = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); ci < n_chunks; ci += nw) {
    const Chunk ch = chunks[ci];
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    const float r_dst = EUCLID ? 0.f : radius[ch.row];
    int run_t = -1;     // the open run (wave-uniform)
    float run_w = 0.f;
    for (int e0 = ch.beg; e0 < ch.end; e0 += 64) {
      const int n = min(64, ch.end - e0);
      const int ei = e0 + min(lane, n - 1);
      const int my_s = col_src[ei];
      const int my_t = col_type[ei];
      // SRC_RUNS: the same batch positions in source order, loaded together with the type
      // order's indices so both passes' index -> radius round trips overlap
      const int my_ss = SRC_RUNS ? col_src_s[ei] : 0;
      const float my_w = EUCLID ? 1.f : expf(-gamma * fabsf(radius[my_s] - r_dst));
      if constexpr (SRC_RUNS) src_runs_batch<EUCLID>(x, radius, my_ss, r_dst, gamma, d, off, lane, n, upto, acc);
      // gathered source rows (SRC_RUNS: src_runs_batch above)
      int j = SRC_RUNS ? n : 0;
      for (; j + 8 <= n; j += 8) {
        f4 xs[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) xs[u] = row_load4(x + (int64_t)rl(my_s, j + u) * d, off);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (EUCLID) acc += xs[u];
          else acc += rlf(my_w, j + u) * xs[u];
        }
      }
      for (; j < n; ++j) {
        const f4 xs = row_load4(x + (int64_t)rl(my_s, j) * d, off);
        if (EUCLID) acc += xs;
        else acc += rlf(my_w, j) * xs;
      }
      // runs: a head starts a run (lane 0 compares with the open run's type)
      int prev_t = __shfl_up(my_t, 1);
      if (lane == 0) prev_t = run_t;
      const uint64_t hm = __ballot(lane < n && my_t != prev_t);
      const uint64_t below = hm & upto;
      const int start = below ? 63 - __builtin_clzll(below) : 0;
      float v = lane < n ? my_w : 0.f;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float u = __shfl_up(v, o);
        if (lane - o >= start) v += u;
      }
      // lane 0 starts a new run: the open run ended with the previous batch
      if ((hm & 1ull) && run_t >= 0) acc += run_w * row_load4(rel + (int64_t)run_t * d, off);
      float cw = (hm & 1ull) ? 0.f : run_w;  // otherwise the first closed run continues it
      uint64_t m = hm & ~1ull;                // each head > 0 closes the run ending just before it
      while (m) {
        const int h0 = __builtin_ctzll(m);
        m &= m - 1;
        const bool ok1 = m != 0;
        const int h1 = ok1 ? __builtin_ctzll(m) : h0;
        if (ok1) m &= m - 1;
        const bool ok2 = m != 0;
        const int h2 = ok2 ? __builtin_ctzll(m) : h0;
        if (ok2) m &= m - 1;
        const bool ok3 = m != 0;
        const int h3 = ok3 ? __builtin_ctzll(m) : h0;
        if (ok3) m &= m - 1;
        const float w0 = rlf(v, h0 - 1) + cw;
        cw = 0.f;
        const float w1 = ok1 ? rlf(v, h1 - 1) : 0.f;
        const float w2 = ok2 ? rlf(v, h2 - 1) : 0.f;
        const float w3 = ok3 ? rlf(v, h3 - 1) : 0.f;
        const f4 a0 = row_load4(rel + (int64_t)rl(my_t, h0 - 1) * d, off);
        const f4 a1 = row_load4(rel + (int64_t)rl(my_t, h1 - 1) * d, off);
        const f4 a2 = row_load4(rel + (int64_t)rl(my_t, h2 - 1) * d, off);
        const f4 a3 = row_load4(rel + (int64_t)rl(my_t, h3 - 1) * d, off);
        acc += w0 * a0;
        acc += w1 * a1;
        acc += w2 * a2;
        acc += w3 * a3;
      }
      const float wl = rlf(v, n - 1);
      if (hm == 0ull) {
        run_w += wl;  // the whole batch continues the open run
      } else {
        run_t = rl(my_t, n - 1);
        run_w = wl;
      }
    }
    if (run_t >= 0) acc += run_w * row_load4(rel + (int64_t)run_t * d, off);
    if (ch.slot < 0) store4(out + (int64_t)ch.row * d, col, d, acc * rowscale[ch.row]);
    else store4(partial + (int64_t)ch.slot * pstride, col, d, acc);
  }
}

// ---------------------------------------------------------------------------- fix-ups
// A fix-up {row, sbeg, send, out} sums partial slots [sbeg, send) in slot order.  out = 0:
// the finishing kernels below complete `row` from the sum.  out > 0: a first-level group
// (graph.py cuts a hub row's slots into groups of <= 64, so no single wave walks thousands
// of slots): k_fixup_groups writes the raw sum into partial slot out - 1, which the row's
// own (second-level) fix-up then reads.  The group pass runs first, in its own launch.
__device__ __forceinline__ f4 slot_sum4(const float* __restrict__ partial, int pstride, int sbeg, int send, int c) {
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  int s = sbeg;
  for (; s + 4 <= send; s += 4) {  // 4 independent loads in flight, summed in slot order
    const f4 v0 = *reinterpret_cast<const f4*>(partial + (int64_t)s * pstride + c);
    const f4 v1 = *reinterpret_cast<const f4*>(partial + (int64_t)(s + 1) * pstride + c);
    const f4 v2 = *reinterpret_cast<const f4*>(partial + (int64_t)(s + 2) * pstride + c);
    const f4 v3 = *reinterpret_cast<const f4*>(partial + (int64_t)(s + 3) * pstride + c);
    acc += v0;
    acc += v1;
    acc += v2;
    acc += v3;
  }
  for (; s < send; ++s) acc += *reinterpret_cast<const f4*>(partial + (int64_t)s * pstride + c);
  return acc;
}

__device__ __forceinline__ float slot_sum1(const float* __restrict__ partial, int pstride, int sbeg, int send, int c) {
  float acc = 0.f;
  for (int s = sbeg; s < send; ++s) acc += partial[(int64_t)s * pstride + c];
  return acc;
}

// First-level groups: raw sums of the first `width` columns (d, or d + 1 with the Lorentz
// time coordinate at column d), float4 up to width & ~3, then scalar.
__global__ __launch_bounds__(256) void k_fixup_groups(float* __restrict__ partial, int pstride,
                                                      const Fixup* __restrict__ fx, int n_fix, int width) {
  const int d = width & ~3;
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n_fix; i += nw) {
    const Fixup f = fx[i];
    if (f.pad <= 0) continue;
    float* dst = partial + (int64_t)(f.pad - 1) * pstride;
    for (int c = lane * 4; c < d; c += 256) *reinterpret_cast<f4*>(dst + c) = slot_sum4(partial, pstride, f.sbeg, f.send, c);
    for (int c = d + lane; c < width; c += 64) dst[c] = slot_sum1(partial, pstride, f.sbeg, f.send, c);
  }
}

static inline unsigned grid_for(int n_items);

static int launch_groups(float* partial, int pstride, const void* fixups, int n_fix, int width, hipStream_t st) {
  hipLaunchKernelGGL(k_fixup_groups, dim3(grid_for(n_fix)), dim3(256), 0, st, partial, pstride,
                     (const Fixup*)fixups, n_fix, width);
  return check_launch("k_fixup_groups");
}

template <int MODE>
__global__ __launch_bounds__(256) void k_gather_fixup(const float* __restrict__ partial, int pstride,
                                                      const Fixup* __restrict__ fx, int n_fix,
                                                      const float* __restrict__ rowscale, int d,
                                                      float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int col = lane * 4;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n_fix; i += nw) {
    const Fixup f = fx[i];
    if (f.pad > 0) continue;  // a first-level group (k_fixup_groups)
    const f4 acc = slot_sum4(partial, pstride, f.sbeg, f.send, min(col, d - 4));
    f4 v = (MODE == AGG_MEAN) ? acc / rowscale[f.row] : acc * rowscale[f.row];
    store4(out + (int64_t)f.row * d, col, d, v);
  }
}

// Raw partial sums of a shard (multi-GPU, edge partition): out[row] = sum of its chunk
// partials, all `width` columns (d, or d + 1 with the Lorentz time coordinate), unfinished,
// so the all-reduce of out across ranks is a plain sum.
__global__ __launch_bounds__(256) void k_partial_sum(const float* __restrict__ partial, int pstride,
                                                     const Fixup* __restrict__ fx, int n_fix, int width,
                                                     float* __restrict__ out, int ostride) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n_fix; i += nw) {
    const Fixup f = fx[i];
    if (f.pad > 0) continue;  // a first-level group (k_fixup_groups)
    for (int c = lane; c < width; c += 64) out[(int64_t)f.row * ostride + c] = slot_sum1(partial, pstride, f.sbeg, f.send, c);
  }
}

// ------------------------------------------------------------------------------ Lorentz
// Messages and centroid: gather.h (hyperbolic_layers.py:589-625).
// S in {1, 2, 4}: blocks held in registers, 8 (S = 4: 4) edges in flight per wave
// (independent loads and reductions, accumulation in edge order).  S == 0: any s, x row staged in LDS.
template <int S>
__global__ __launch_bounds__(256) void k_lorentz_sum(
    const float* __restrict__ x, const float* __restrict__ rel, const float* __restrict__ W,
    const int* __restrict__ col_src, const int* __restrict__ col_type, const Chunk* __restrict__ chunks,
    int n_chunks, int nb, int s_gen, Curv k, int d, float* __restrict__ partial, int pstride,
    float* __restrict__ out) {
  __shared__ float xsh_all[S == 0 ? 4 : 1][S == 0 ? 256 : 1];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int col = lane * 4;
  const bool active = col < d;
  const int wstride = nb * (d / nb) * (d / nb);
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int ci = blockIdx.x * (blockDim.x >> 6) + wv; ci < n_chunks; ci += nw) {
    const Chunk ch = chunks[ci];
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    float acc0 = 0.f;
    for (int e0 = ch.beg; e0 < ch.end; e0 += 64) {
      const int n = min(64, ch.end - e0);
      int my_s = 0, my_t = 0;
      if (lane < n) {
        my_s = col_src[e0 + lane];
        my_t = col_type[e0 + lane];
      }
      int j = 0;
      if constexpr (S > 0) {
        // EB edges per batch, all loads unconditional: wave-uniform row base (SGPR pair) +
        // one per-lane byte offset, so the loads need no per-lane address arithmetic; lanes
        // past d load the last real columns again and are masked out of |m|^2 (their acc is
        // zeroed before the finish).  |m_u|^2 of the batch come from one transposing
        // reduction (batch_sums) and the per-edge scalars of the Lorentz point (exp0 factor,
        // time coordinate, scale) are computed lane-parallel, edge u in lane batch_lane(u).
        constexpr int EB = S == 4 ? 4 : 8;
        const uint32_t xoff = (uint32_t)min(col, d - 4) * 4u, woff = xoff * S;
        const float amask = active ? 1.f : 0.f;
        // A batch inside one relation-type run (the row/type edge order makes a hub row's
        // edges a few long runs) loads the run's block weights and relation row once for its
        // EB edges: 0.8 KB + 2.4 KB / EB per edge from L2 instead of 3.2 KB (vector-memory
        // request rate, not HBM, bounded it).  Same arithmetic per edge as the general path.
        for (; j + EB <= n; j += EB) {
          f4 xs[EB], m[EB];
          const int t_first = rl(my_t, j);
          const uint64_t want = ((1ull << EB) - 1ull) << j;
          if ((__ballot(my_t == t_first) & want) == want) {  // wave-uniform
            WFrag<S> wr;
            wr.load_row(W + (int64_t)t_first * wstride, woff);
            const f4 rr = row_load4(rel + (int64_t)t_first * d, xoff);
#pragma unroll
            for (int u = 0; u < EB; ++u) xs[u] = row_load4(x + (int64_t)rl(my_s, j + u) * d, xoff);
#pragma unroll
            for (int u = 0; u < EB; ++u) m[u] = wr.apply(xs[u]) + rr;
          } else {
            f4 rv[EB];
            WFrag<S> wf[EB];
#pragma unroll
            for (int u = 0; u < EB; ++u) {
              const int src = rl(my_s, j + u), typ = rl(my_t, j + u);
              xs[u] = row_load4(x + (int64_t)src * d, xoff);
              rv[u] = row_load4(rel + (int64_t)typ * d, xoff);
              wf[u].load_row(W + (int64_t)typ * wstride, woff);
            }
#pragma unroll
            for (int u = 0; u < EB; ++u) m[u] = wf[u].apply(xs[u]) + rv[u];
          }
          float q[EB];
#pragma unroll
          for (int u = 0; u < EB; ++u) q[u] = dot4(m[u], m[u]) * amask;
          const float n2l = batch_sums<EB>(q, lane);
          float p2;  // lorentz_accum (gather.h), lane-parallel over the batch
          const float f = exp0_factor(n2l, k, &p2);
          const float den = fmaxf(1.f - k.c * p2, REGCN_EPS);
          const float a0 = (1.f + k.c * p2) / (k.sqrt_c * den);
          const float sc = 2.f * f / den;
#pragma unroll
          for (int u = 0; u < EB; ++u) {
            acc0 += rlane(a0, batch_lane<EB>(u));
            acc += m[u] * rlane(sc, batch_lane<EB>(u));
          }
        }
        if (!active) acc = f4{0.f, 0.f, 0.f, 0.f};
      }
      for (; j < n; ++j) {
        const int src = rl(my_s, j), typ = rl(my_t, j);
        const float* Wt = W + (int64_t)typ * wstride;
        f4 xs = load4(x + (int64_t)src * d, col, d);
        f4 m = {0.f, 0.f, 0.f, 0.f};
        if constexpr (S > 0) {
          if (active) {
            WFrag<S> wf;
            wf.load(Wt, col);
            m = wf.apply(xs);
          }
        } else {
          m = block_general4(xsh_all[S == 0 ? wv : 0], xs, Wt, s_gen, col, active);
        }
        m += load4(rel + (int64_t)typ * d, col, d);
        lorentz_accum(m, wave_sum(dot4(m, m)), k, acc0, acc);
      }
    }
    if (ch.slot < 0) {
      store4(out + (int64_t)ch.row * d, col, d, lorentz_finish(acc0, acc, k));
    } else {
      float* p = partial + (int64_t)ch.slot * pstride;
      store4(p, col, d, acc);
      if (lane == 0) p[d] = acc0;
    }
  }
}

__global__ __launch_bounds__(256) void k_lorentz_fixup(const float* __restrict__ partial, int pstride,
                                                       const Fixup* __restrict__ fx, int n_fix, Curv k,
                                                       int d, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int col = lane * 4;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n_fix; i += nw) {
    const Fixup f = fx[i];
    if (f.pad > 0) continue;  // a first-level group (k_fixup_groups)
    f4 acc = slot_sum4(partial, pstride, f.sbeg, f.send, min(col, d - 4));
    if (col >= d) acc = f4{0.f, 0.f, 0.f, 0.f};
    const float acc0 = slot_sum1(partial, pstride, f.sbeg, f.send, d);
    store4(out + (int64_t)f.row * d, col, d, lorentz_finish(acc0, acc, k));
  }
}

static inline unsigned grid_for(int n_items) {
  long b = ((long)n_items + 3) / 4;
  if (b > 16384) b = 16384;
  return (unsigned)(b < 1 ? 1 : b);
}

int gather_sum(int mode, const float* x, const float* radius, const float* rel, const int* col_src,
               const int* col_type, const float* rowscale, const void* chunks, int n_chunks,
               const void* fixups, int n_fix, float gamma, int d, float* partial, int pstride, float* out,
               hipStream_t st, const int* col_src_s) {
  if (d <= 0 || d > 256 || (d & 3)) return set_error(REGCN_EINVAL, "aggregation needs d %% 4 == 0 and d <= 256 (d=%d)", d);
  if (!x || !col_src || !rowscale || !out) return set_error(REGCN_EINVAL, "null pointer");
  if (mode != AGG_MEAN && (!col_type || !rel)) return set_error(REGCN_EINVAL, "null pointer");
  if (col_src_s && mode == AGG_MEAN) return set_error(REGCN_EINVAL, "source runs apply to the union aggregations only");
  if (mode == AGG_UNION && !radius) return set_error(REGCN_EINVAL, "union aggregation needs radius");
  if (n_fix > 0 && !partial) return set_error(REGCN_EINVAL, "partial workspace required");
  const Chunk* ch = (const Chunk*)chunks;
  const Fixup* fx = (const Fixup*)fixups;
  if (n_chunks > 0) {
    // the mean and the source-run hub pass run every chunk in one pass (one wave each, no
    // grid-stride): chunk i sits on workgroup i / 4, XCD (i / 4) % 8, in dispatch order
    // (graph.py blocked_span_chunks deals a block's chunks to one XCD)
    const long gm = ((long)n_chunks + 3) / 4;
    dim3 g((mode == AGG_MEAN || col_src_s) && gm <= 0x7fffffffL ? (unsigned)gm : grid_for(n_chunks)), b(256);
    if (mode == AGG_UNION && col_src_s)
      hipLaunchKernelGGL((k_union_runs<false, true>), g, b, 0, st, x, radius, rel, col_src, col_type, col_src_s,
                         rowscale, ch, n_chunks, gamma, d, partial, pstride, out);
    else if (mode == AGG_UNION)
      hipLaunchKernelGGL((k_union_runs<false, false>), g, b, 0, st, x, radius, rel, col_src, col_type, nullptr,
                         rowscale, ch, n_chunks, gamma, d, partial, pstride, out);
    else if (mode == AGG_EUCLID && col_src_s)
      hipLaunchKernelGGL((k_union_runs<true, true>), g, b, 0, st, x, radius, rel, col_src, col_type, col_src_s,
                         rowscale, ch, n_chunks, gamma, d, partial, pstride, out);
    else if (mode == AGG_EUCLID)
      hipLaunchKernelGGL((k_union_runs<true, false>), g, b, 0, st, x, radius, rel, col_src, col_type, nullptr,
                         rowscale, ch, n_chunks, gamma, d, partial, pstride, out);
    else if (mode == AGG_MEAN)
      hipLaunchKernelGGL(k_gather_sum<AGG_MEAN>, g, b, 0, st, x, radius, rel, col_src, col_type, rowscale, ch,
                         n_chunks, gamma, d, partial, pstride, out);
    else
      return set_error(REGCN_EINVAL, "unknown aggregation mode %d", mode);
    int rc = check_launch("k_gather_sum");
    if (rc) return rc;
  }
  if (n_fix > 0) {
    int rc = launch_groups(partial, pstride, fixups, n_fix, d, st);
    if (rc) return rc;
    dim3 g(grid_for(n_fix)), b(256);
    if (mode == AGG_MEAN)
      hipLaunchKernelGGL(k_gather_fixup<AGG_MEAN>, g, b, 0, st, partial, pstride, fx, n_fix, rowscale, d, out);
    else
      hipLaunchKernelGGL(k_gather_fixup<AGG_UNION>, g, b, 0, st, partial, pstride, fx, n_fix, rowscale, d, out);
    return check_launch("k_gather_fixup");
  }
  return 0;
}

int partial_sum(float* partial, int pstride, const void* fixups, int n_fix, int width, float* out, int ostride,
                hipStream_t st) {
  if (n_fix == 0) return 0;
  if (!partial || !fixups || !out) return set_error(REGCN_EINVAL, "null pointer");
  if (width <= 0 || width > pstride || width > ostride) return set_error(REGCN_EINVAL, "bad partial-sum width");
  int rc = launch_groups(partial, pstride, fixups, n_fix, width, st);  // group slots: scratch
  if (rc) return rc;
  dim3 g(grid_for(n_fix)), b(256);
  hipLaunchKernelGGL(k_partial_sum, g, b, 0, st, partial, pstride, (const Fixup*)fixups, n_fix, width, out, ostride);
  return check_launch("k_partial_sum");
}

int lorentz_sum(const float* x, const float* rel, const float* W, const int* col_src, const int* col_type,
                const void* chunks, int n_chunks, const void* fixups, int n_fix, int nb, float c, int d,
                float* partial, int pstride, float* out, hipStream_t st) {
  if (d <= 0 || d > 256 || (d & 3)) return set_error(REGCN_EINVAL, "aggregation needs d %% 4 == 0 and d <= 256 (d=%d)", d);
  if (nb <= 0 || d % nb) return set_error(REGCN_EINVAL, "d=%d not divisible by num_bases=%d", d, nb);
  if (!x || !rel || !W || !col_src || !col_type || !out) return set_error(REGCN_EINVAL, "null pointer");
  if (n_fix > 0 && (!partial || pstride < d + 1)) return set_error(REGCN_EINVAL, "partial workspace required");
  const int s = d / nb;
  Curv k = make_curv(c);
  const Chunk* ch = (const Chunk*)chunks;
  if (n_chunks > 0) {
    dim3 g(grid_for(n_chunks)), b(256);
    if (s == 1)
      hipLaunchKernelGGL(k_lorentz_sum<1>, g, b, 0, st, x, rel, W, col_src, col_type, ch, n_chunks, nb, s, k, d,
                         partial, pstride, out);
    else if (s == 2)
      hipLaunchKernelGGL(k_lorentz_sum<2>, g, b, 0, st, x, rel, W, col_src, col_type, ch, n_chunks, nb, s, k, d,
                         partial, pstride, out);
    else if (s == 4)
      hipLaunchKernelGGL(k_lorentz_sum<4>, g, b, 0, st, x, rel, W, col_src, col_type, ch, n_chunks, nb, s, k, d,
                         partial, pstride, out);
    else
      hipLaunchKernelGGL(k_lorentz_sum<0>, g, b, 0, st, x, rel, W, col_src, col_type, ch, n_chunks, nb, s, k, d,
                         partial, pstride, out);
    int rc = check_launch("k_lorentz_sum");
    if (rc) return rc;
  }
  if (n_fix > 0) {
    int rc = launch_groups(partial, pstride, fixups, n_fix, d + 1, st);
    if (rc) return rc;
    dim3 g(grid_for(n_fix)), b(256);
    hipLaunchKernelGGL(k_lorentz_fixup, g, b, 0, st, partial, pstride, (const Fixup*)fixups, n_fix, k, d, out);
    return check_launch("k_lorentz_fixup");
  }
  return 0;
}

}  // namespace regcn
