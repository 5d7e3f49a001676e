// Device pieces of the fused layer kernels, shared by layer.hip (one launch per layer) and
// timestep.hip (the per-timestep phase launches): LDS layout, timestep epilogue, the inline
// CSR gather of a destination tile and its finish.  See layer.hip's header for the design.
#pragma once
#include "common.h"
#include "gather.h"
#include "regcn_internal.h"
#include "rowtile.h"

namespace regcn {
// per wave count (rowtile.h): units built with different REGCN_ROWTILE_WAVES never share a definition
inline namespace REGCN_RT_CAT(rowtile_w, REGCN_ROWTILE_WAVES) {

// partial slots of the gather (TM + NWAVE - 1), reused for the three operand tiles after it
constexpr int PART_ROWS = (TM + NWAVE - 1) > 3 * TM ? (TM + NWAVE - 1) : 3 * TM;

struct LdsLayout {
  int lda;
  int part, X, red, ints, xsh, total_bytes;  // float offsets; total in bytes
};

// Partial / operand rows one k_layer launch needs: the gather's TM + NWAVE - 1 partial slots,
// reused after the finish for the aggregate tile, the skip operand (P1) and the timestep
// operand (P2) -- only the ones the launch has, so a plain layer's tile fits more workgroups
// per CU (LDS: 5 per CU without skip / timestep, 4 with one of them, 3 with both).
__host__ __device__ inline int layer_part_rows(bool skip, bool step) {
  const int ops = TM * (1 + (skip ? 1 : 0) + (step ? 1 : 0));
  return ops > TM + NWAVE - 1 ? ops : TM + NWAVE - 1;
}

__host__ __device__ inline LdsLayout lds_layout(int d, bool gen_s, int part_rows = PART_ROWS) {
  LdsLayout L;
  L.lda = tile_lda(d);
  L.part = 0;
  L.X = part_rows * L.lda;
  L.red = L.X + TM * L.lda;
  L.ints = L.red + RED_FLOATS;
  L.xsh = L.ints + 32;  // trow[16], tmask[NWAVE] (+pad)
  L.total_bytes = (L.xsh + (gen_s ? NWAVE * MAX_D : 0)) * 4;
  return L;
}

__device__ __forceinline__ void frag_to_tile(const Frag& a, float* T, int lda, int n_valid, int d) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = frag_row(r);
    float* row = T + i * lda;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int col = frag_col(j);
      if (col < d) row[col] = i < n_valid ? a.t[j][r] : 0.f;
    }
  }
}

// ---------------------------------------------------------------------- timestep epilogue
// x_lds / p2_lds (optional): the output tangent rows and their +-10 clamp also into LDS tiles
// (the next timestep's operands when a kernel runs several timesteps; they may alias P: P's
// last read precedes the radius reduction's barrier).
// tw: the time-gate pre-activation clamp(x_prev) @ W_g (taken by reference: a pointer to a
// local Frag compared against null pins it in scratch memory, private null being nonzero).
// h_out / x_out / r_out: the output rows (p's own, or per-timestep ones of a chain: passed
// apart, since a local copy of StepArgs would live in scratch).
// ANA (--run-analysis, k_timestep only): also the time gate per element into p.gate_out and,
// with the residual evolution, per row {clipped delta, dynamic radius, base radius} into
// p.stat_out[0 / V / 2V + row] (hyperbolic_model.py:852-856, hyperbolic_ops.py:426-434).
template <bool ANA = false>
__device__ __forceinline__ void step_epilogue_out(RowRed& rr, Frag& ct, float n2[4], const float* P, int lda,
                                                  const int* trow, int n_valid, const StepArgs& p, const Frag& tw,
                                                  float* h_out, float* x_out, float* r_out, int64_t* trace = nullptr,
                                                  float* x_lds = nullptr, float* p2_lds = nullptr) {
  auto stamp = [&](int k) {  // profiling: phase stamps 14, 15 (trace_mark)
    if (trace && threadIdx.x == 0) trace[blockIdx.x * 16 + k] = (int64_t)__builtin_amdgcn_s_memrealtime();
  };
  stamp(14);
  project_known(ct, n2, p.k);
  if (p.layer_norm) {
    log0_known(ct, n2, p.k);
    normalize_known(ct, n2);
    exp0_known(ct, n2, p.k);
  }
  log0_known(ct, n2, p.k);
  Frag pt;
  frag_from_tile(pt, P, lda, p.d);
  float bg[TPW];
  col_load(bg, p.b_g, p.d);
  Frag gate;  // ANA only
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const f4 c4 = clamp4(ct.t[j], -10.f, 10.f);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float g = sigmoidf(tw.t[j][r] + bg[j]);
      if constexpr (ANA) gate.t[j][r] = g;
      ct.t[j][r] = g * c4[r] + (1.f - g) * pt.t[j][r];
    }
  }
  if constexpr (ANA) frag_store(gate, p.gate_out, trow, n_valid, p.d);
  rr.sumsq(ct, n2);
  exp0_known(ct, n2, p.k);
  project_known(ct, n2, p.k);  // hyperbolic_model.py:860
  stamp(15);
  // radius: per-row scalars once per lane, for its own row (rowtile.h own_row/spread_rows)
  const int ri = frag_row(threadIdx.x & 3);
  const float rs = p.r_static[trow[ri < n_valid ? ri : 0]];
  const float n2o = own_row(n2);
  float newr = rs;
  if (p.residual) {
    float wr[TPW], dl[4], lf[4];
    col_load(wr, p.w_r, p.d);
    spread_rows(log0_factor(n2o, p.k_rad), lf);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < TPW; ++j) s += wr[j] * (ct.t[j][r] * lf[r]);
      dl[r] = s;
    }
    rr.allreduce(dl);
    const float delta = fminf(fmaxf(own_row(dl) + *p.b_r, -p.eps_r), p.eps_r);
    const float dyn = row_radius(n2o);
    newr = (p.beta * rs + (1.f - p.beta) * dyn) + delta;
    if constexpr (ANA) {
      if (p.stat_out && (threadIdx.x & 15) < 4 && wave_id() == 0 && ri < n_valid) {
        const int64_t row = trow[ri];
        p.stat_out[row] = delta;
        p.stat_out[(int64_t)p.V + row] = dyn;
        p.stat_out[2 * (int64_t)p.V + row] = p.beta * rs + (1.f - p.beta) * dyn;
      }
    }
  }
  const Curv kr = p.residual ? p.k_rad : p.k;  // by value: a pointer select would pin a local StepArgs in scratch
  float f[4];
  spread_rows(fdiv(fminf(fmaxf(newr, REGCN_EPS), kr.rmax), row_radius(n2o)), f);
  scale_known(ct, n2, f);
  frag_store(ct, h_out, trow, n_valid, p.d);
  if (r_out) store_radius(n2, r_out, trow, n_valid);
  if (x_out || x_lds) {
    log0_known(ct, n2, p.k);
    if (x_out) frag_store(ct, x_out, trow, n_valid, p.d);
    if (x_lds) {
      frag_to_tile(ct, x_lds, lda, n_valid, p.d);
#pragma unroll
      for (int j = 0; j < TPW; ++j) ct.t[j] = clamp4(ct.t[j], -10.f, 10.f);
      frag_to_tile(ct, p2_lds, lda, n_valid, p.d);
    }
  }
}

__device__ __forceinline__ void step_epilogue_tw(RowRed& rr, Frag& ct, float n2[4], const float* P, int lda,
                                                 const int* trow, int n_valid, const StepArgs& p, const Frag& tw,
                                                 int64_t* trace = nullptr) {
  step_epilogue_out(rr, ct, n2, P, lda, trow, n_valid, p, tw, p.h_out, p.x_out, p.r_out, trace);
}

// The timestep epilogue computing the time-gate GEMM itself (tw_pre == nullptr) or taking the
// caller's.
template <bool ANA = false>
__device__ __forceinline__ void step_epilogue(RowRed& rr, Frag& ct, float n2[4], const float* P, int lda,
                                              const int* trow, int n_valid, const StepArgs& p,
                                              int64_t* trace = nullptr, const Frag* tw_pre = nullptr) {
  if (tw_pre) return step_epilogue_tw(rr, ct, n2, P, lda, trow, n_valid, p, *tw_pre, trace);
  Frag tw;
  tw.zero();
  mfma_tile(tw, P, lda, p.w_g, p.d, p.d);
  if constexpr (ANA)
    step_epilogue_out<true>(rr, ct, n2, P, lda, trow, n_valid, p, tw, p.h_out, p.x_out, p.r_out, trace);
  else
    step_epilogue_tw(rr, ct, n2, P, lda, trow, n_valid, p, tw, trace);
}

// Profiling hook: wall-clock phase stamps (100 MHz) of wave 0, 16 slots per workgroup.
__device__ __forceinline__ void trace_mark(const LayerArgs& p, int k) {
  if (p.trace && threadIdx.x == 0) p.trace[blockIdx.x * 16 + k] = (int64_t)__builtin_amdgcn_s_memrealtime();
}

// --------------------------------------------------------------------------- inline gather
// Flattened, segmented gather of the tile's in-edges (see file header).  Items come from
// the host-built per-tile list (item_src, item_tl = type << 4 | local row), so an edge's
// row loads depend on one coalesced index load only.  Wave w reduces items [ib, ie), EB
// edges in flight (all loads unconditional, clamped addresses); each row it touches gets
// one partial row in slot i + w (+ the Lorentz time coordinate at column d) and a bit in
// tmask[w].
template <int AGG, int S>
__device__ __forceinline__ void tile_gather(const LayerArgs& p, float* part, int lda, const int* trow, int tile,
                                            int* tmask, float* xsh) {
  constexpr int EB = (AGG == AGG_LORENTZ && (S == 4 || S == 0)) ? 4 : 8;
  const int lane = threadIdx.x & 63, w = wave_id();
  const int d = p.d;
  const int col = lane * 4, colc = min(col, d - 4);
  const bool active = col < d;
  const int i0 = p.item_ptr[tile], n_items = p.item_ptr[tile + 1] - i0;
  const int ib = i0 + (n_items * w) / NWAVE, ie = i0 + (n_items * (w + 1)) / NWAVE;
  const int s_gen = (AGG == AGG_LORENTZ) ? d / p.nb : 1;
  const int wstride = (AGG == AGG_LORENTZ) ? p.nb * s_gen * s_gen : 0;
  const Curv k = p.k;
  const f4 zero = {0.f, 0.f, 0.f, 0.f};
  int cur = -1;
  unsigned mask = 0;
  f4 acc = zero;
  float acc0 = 0.f;
  auto flush = [&]() {
    if (cur >= 0) {
      float* dst = part + (cur + w) * lda;
      if (active) {
        dst[col] = acc.x;
        dst[col + 1] = acc.y;
        dst[col + 2] = acc.z;
        dst[col + 3] = acc.w;
      }
      if (AGG == AGG_LORENTZ && lane == 0) dst[d] = acc0;
      mask |= 1u << cur;
    }
  };
  auto take = [&](int li) {
    if (li != cur) {
      flush();
      cur = li;
      acc = zero;
      acc0 = 0.f;
    }
  };
  const uint32_t xoff = (uint32_t)colc * 4u, woff = xoff * (S > 0 ? S : 1);
  auto row4 = [&](const float* base, int row) {  // unconditional clamped row fragment, zero past d
    const f4 v = row_load4(base + (int64_t)row * d, xoff);
    return active ? v : zero;
  };
  // Batched loads: lanes past d keep their duplicate of the last real columns (a flush stores
  // active lanes only; the Lorentz |m|^2 masks them), so no per-load select.
  auto row4u = [&](const float* base, int row) { return row_load4(base + (int64_t)row * d, xoff); };
  const float amask = active ? 1.f : 0.f;
  trace_mark(p, 8);
  for (int t0 = ib; t0 < ie; t0 += 64) {
    const int n = min(64, ie - t0);
    const int t = t0 + min(lane, n - 1);
    const int my_s = p.item_src[t];
    const int tl = p.item_tl[t];
    const int my_t = tl >> 4, my_i = tl & 15;
    float my_w = 1.f;
    if (AGG == AGG_UNION) my_w = expf(-p.gamma * fabsf(p.radius[my_s] - p.radius[trow[my_i]]));
    if (t0 == ib) {
      __builtin_amdgcn_s_waitcnt(0);
      trace_mark(p, 9);
    }
    // Batches of EB edges; the last batch of a window is partial: its missing edges read
    // lane n-1's (valid) indices, so every load of the batch is in flight at once, and
    // contribute nothing (wave-uniform guard).  A tile's few edges cost one round trip,
    // not one per edge.
    int j = 0;
    if constexpr (AGG == AGG_UNION || AGG == AGG_EUCLID) {
      // With item_src_runs the items are in (row, source) order: a run of equal (row, source)
      // in this window gathers the source row once, at its head, with weight count * w; the
      // other items' x loads go through an empty buffer resource (no memory request, zero) and
      // the relation rows stay per item.  Without it every item is its own head (count 1).
      uint64_t hx = ~0ull;
      float wx = my_w;
      if (p.item_src_runs) {
        const int ps = __shfl_up(my_s, 1), pi = __shfl_up(my_i, 1);
        hx = __ballot(lane < n && (lane == 0 || my_s != ps || my_i != pi));
        const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
        const uint64_t after = hx & ~upto;
        wx = my_w * (float)((after ? __builtin_ctzll(after) : n) - lane);
      }
      for (; j < n; j += EB) {
        const int nv = n - j;
        f4 xs[EB], rv[EB];
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          const int nrec = ((hx >> ((j + u) & 63)) & 1ull) ? 0x7FFFFFFF : 0;
          xs[u] = row_load4_n(p.x + (int64_t)rl(my_s, j + u) * d, xoff, nrec);
          rv[u] = row4u(p.rel, rl(my_t, j + u));
        }
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          if (u < nv) {
            take(rl(my_i, j + u));
            if (AGG == AGG_EUCLID) acc += rlf(wx, j + u) * xs[u] + rv[u];
            else acc += rlf(wx, j + u) * xs[u] + rlf(my_w, j + u) * rv[u];
          }
        }
      }
    } else if constexpr (AGG == AGG_LORENTZ) {
      if constexpr (S > 0) {
        for (; j < n; j += EB) {
          const int nv = n - j;
          f4 xs[EB], rv[EB];
          WFrag<S> wf[EB];
#pragma unroll
          for (int u = 0; u < EB; ++u) {
            const int src = rl(my_s, j + u), typ = rl(my_t, j + u);
            xs[u] = row4u(p.x, src);
            rv[u] = row4u(p.rel, typ);
            wf[u].load_row(p.w_rel + (int64_t)typ * wstride, woff);
          }
          f4 m[EB];
          float q[EB];
#pragma unroll
          for (int u = 0; u < EB; ++u) {
            m[u] = wf[u].apply(xs[u]) + rv[u];
            q[u] = dot4(m[u], m[u]) * amask;
          }
          const float n2l = batch_sums<EB>(q, lane);  // |m_u|^2 in lane batch_lane(u)
          // the per-edge scalars of the Lorentz point, once per batch with lane = edge
          float p2;
          const float f = exp0_factor(n2l, k, &p2);
          const float den = fmaxf(1.f - k.c * p2, REGCN_EPS);
          const float a0 = (1.f + k.c * p2) / (k.sqrt_c * den);
          const float sc = 2.f * f / den;
#pragma unroll
          for (int u = 0; u < EB; ++u) {
            if (u < nv) {
              take(rl(my_i, j + u));
              acc0 += rlane(a0, batch_lane<EB>(u));
              acc += m[u] * rlane(sc, batch_lane<EB>(u));
            }
          }
          if (j == 0 && t0 == ib) trace_mark(p, 10);
        }
      }
      for (; j < n; ++j) {  // general block size s (S == 0)
        const int src = rl(my_s, j), typ = rl(my_t, j);
        const float* Wt = p.w_rel + (int64_t)typ * wstride;
        const f4 xs = row4(p.x, src);
        f4 m = zero;
        if constexpr (S > 0) {
          WFrag<S> wf;
          wf.load(Wt, colc);
          m = active ? wf.apply(xs) : zero;
        } else {
          m = block_general4(xsh + w * MAX_D, xs, Wt, s_gen, col, active);
        }
        m += row4(p.rel, typ);
        take(rl(my_i, j));
        lorentz_accum(m, wave_sum(dot4(m, m)), k, acc0, acc);
      }
    }
  }
  trace_mark(p, 11);
  flush();
  if (lane == 0) tmask[w] = (int)mask;
}

// Combine the wave partials of row i (wave w does rows w, w + NWAVE) and finish it:
// Lorentz centroid -> log0, or norm-scaled sum; rows over budget read the pre-aggregated
// row.  Row w + NWAVE q of the tile ends in out[q] (heavy[q]: pre[q] holds its pre-aggregated
// row instead).
template <int AGG>
__device__ __forceinline__ void tile_finish_rows(const LayerArgs& p, const float* part, int lda, const int* trow,
                                                 int count, const int* tmask, int rdeg, float rnorm,
                                                 f4 out[TM / NWAVE], f4 pre[TM / NWAVE], bool heavy[TM / NWAVE]) {
  const int lane = threadIdx.x & 63, w = wave_id();
  const int d = p.d;
  const int col = lane * 4, colc = min(col, d - 4);
  const bool active = col < d;
  const f4 zero = {0.f, 0.f, 0.f, 0.f};
  // the wave's rows side by side: independent loads and reductions
  constexpr int RPW = TM / NWAVE;  // rows per wave
  f4 acc[RPW];
  float acc0[RPW];
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int i = w + NWAVE * q;
    const int row = trow[i < count ? i : 0];
    heavy[q] = i < count && __builtin_amdgcn_readlane(rdeg, i) > p.budget;
    pre[q] = zero;
    if (heavy[q]) {  // pre-aggregated by the chunked kernels
      const f4 v = *reinterpret_cast<const f4*>(p.agg + (int64_t)row * d + colc);
      pre[q] = active ? v : zero;
    }
    acc[q] = zero;
    acc0[q] = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < NWAVE; ++w2) {
      if ((tmask[w2] >> i) & 1) {  // slot i + w2 written by wave w2 (wave-uniform branch)
        const float* src = part + (i + w2) * lda;
        const f4 v = *reinterpret_cast<const f4*>(src + colc);  // rows 16-B aligned (tile_lda)
        acc[q] += active ? v : zero;
        if (AGG == AGG_LORENTZ) acc0[q] += src[d];
      }
    }
  }
  if constexpr (AGG == AGG_LORENTZ) {
    // Centroid -> Poincare -> log0 of the wave's RPW rows with the per-row scalar chain run
    // once, lane-parallel (row q in lane batch_lane<RPW>(q)): |acc_q|^2 from one transposing
    // reduction, y_q = acc_q / (sc (1 + c0 sqrt_c)) so |y_q|^2 = |acc_q|^2 / (sc den)^2 needs
    // no second reduction, and out_q = acc_q * (one factor).  gather.h lorentz_finish, batched.
    // a batch of RB >= RPW values (4 or 8; with 8 waves a wave has 2 rows: zero padded)
    constexpr int RB = RPW < 4 ? 4 : RPW;
    static_assert(RB == 4 || RB == 8, "batched finish needs 4 or 8 rows per wave");
    float ss[RB];
#pragma unroll
    for (int q = 0; q < RB; ++q) ss[q] = q < RPW ? dot4(acc[q < RPW ? q : 0], acc[q < RPW ? q : 0]) : 0.f;
    const float s2 = batch_sums<RB>(ss, lane);
    const int my_q = batch_row<RB>(lane);
    float a0 = acc0[0];
#pragma unroll
    for (int q = 1; q < RPW; ++q) a0 = my_q == q ? acc0[q] : a0;
    const float ip = -a0 * a0 + s2;
    const float sc = sqrtf(fmaxf(-ip * p.k.c, REGCN_EPS));
    const float den = fmaxf(1.f + (a0 / sc) * p.k.sqrt_c, REGCN_EPS);
    const float inv = 1.f / (sc * den);
    const float fac = inv * log0_factor(s2 * inv * inv, p.k);
#pragma unroll
    for (int q = 0; q < RPW; ++q) out[q] = acc[q] * rlane(fac, batch_lane<RB>(q));
  } else {
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int i = w + NWAVE * q;
      out[q] = acc[q] * rlane(rnorm, i);
    }
  }
}

// tile_finish_rows, the result overwriting slot i (the A operand / agg fragment source).
template <int AGG>
__device__ __forceinline__ void tile_finish(const LayerArgs& p, float* part, int lda, const int* trow, int count,
                                            const int* tmask, int rdeg, float rnorm) {
  const int lane = threadIdx.x & 63, w = wave_id();
  const int col = lane * 4;
  const bool active = col < p.d;
  const f4 zero = {0.f, 0.f, 0.f, 0.f};
  constexpr int RPW = TM / NWAVE;
  f4 out[RPW], pre[RPW];
  bool heavy[RPW];
  tile_finish_rows<AGG>(p, part, lda, trow, count, tmask, rdeg, rnorm, out, pre, heavy);
  __syncthreads();  // every partial slot is read before any slot is overwritten
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int i = w + NWAVE * q;
    f4 a = heavy[q] ? pre[q] : out[q];
    if (i >= count) a = zero;
    float* dst = part + i * lda;
    if (active) {
      dst[col] = a.x;
      dst[col + 1] = a.y;
      dst[col + 2] = a.z;
      dst[col + 3] = a.w;
    }
  }
}

}  // inline namespace
}  // namespace regcn
