// Fused message-passing layer (+ timestep) kernels.
//
// One workgroup = NWAVE = 4 waves = one tile of up to 16 destination rows with all d columns:
//   1. CSR gather: the tile's in-edges are flattened into one item list and split into NWAVE
//      contiguous ranges, one per wave; each wave keeps 4-8 edges in flight and does a
//      segmented (per-row) reduction into LDS partial rows, so a tile's hub and its
//      single-edge rows cost the same wall time.  Items are row-sorted, so wave w touches
//      a row range starting at or after the last row of wave w - 1: partial slot i + w
//      (row i, wave w) never collides, and TM + NWAVE - 1 slots hold every partial.  Partials are
//      combined in wave order (deterministic, no atomics).  Rows with in-degree > budget
//      were pre-aggregated by the chunked kernels (aggregate.hip) and are read back.
//   2. Self-loop / neighbour GEMMs on fp32 MFMA (rowtile.h) from LDS tiles.
//   3. Epilogue in registers: clamp, rrelu, dropout mask, exp0 -> h; then either the next
//      layer's prologue (x = log0 h, r = |h|) or the whole timestep (time gate GEMM, radius
//      evolution) -- the layer output never round-trips through HBM.
// Tiles come from the host (graph.py): in-degree-sorted rows packed greedily under an
// edge budget, so no tile's gather is much longer than another's; zero in-degree rows
// follow in plain 16-row tiles (self-evolve weight only).
//
// Reference: UnionRGCNLayer / LorentzRGCNLayer forward (hyperbolic_layers.py:242-323,
// :627-694), rgcn/layers.py:226-279 (euclid), timestep hyperbolic_model.py:829-869.
#include "layer_parts.h"

namespace regcn {

// ==================================================================================== layer
// 4 waves per SIMD (VGPRs <= 128: a few spilled registers on the cold paths) and the LDS
// rows of layer_part_rows: 4-5 workgroups per CU instead of 3, so more tiles' gathers are in
// flight while others run their MFMA products.
template <int AGG, int S, bool STEP>
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(4))) void k_layer(LayerArgs p) {
  extern __shared__ float lds[];
  const bool skip_op = p.prev_t != nullptr;
  const LdsLayout L = lds_layout(p.d, AGG == AGG_LORENTZ && S == 0, layer_part_rows(skip_op, STEP));
  const int lda = L.lda;
  float* part = lds + L.part;
  float* X = lds + L.X;
  int* trow = reinterpret_cast<int*>(lds + L.ints);
  int* tmask = trow + TM;
  RowRed rr{lds + L.red, 0};
  float* P1 = part + TM * lda;                        // skip-connection operand
  float* P2 = part + (skip_op ? 2 : 1) * TM * lda;    // timestep: clamp(x_prev)

  auto mark = [&](int k) {
    trace_mark(p, k);
  };
  mark(0);
  if (p.trace && threadIdx.x == 0) p.trace[blockIdx.x * 16 + 6] = (int64_t)__builtin_amdgcn_s_memtime();
  const int n_pos_tiles = p.tiles ? p.n_pos_tiles : (p.n_pos + TM - 1) / TM;
  const bool pos = (int)blockIdx.x < n_pos_tiles;
  int start, count;
  if (pos) {
    if (p.tiles) {
      start = p.tiles[2 * blockIdx.x];
      count = p.tiles[2 * blockIdx.x + 1];
    } else {
      start = blockIdx.x * TM;
      count = min(TM, p.n_pos - start);
    }
  } else {
    start = p.n_pos + (blockIdx.x - n_pos_tiles) * TM;
    count = min(TM, p.V - start);
  }
  const bool inline_gather = pos && AGG != AGG_NONE;
  if (threadIdx.x < TM) trow[threadIdx.x] = p.rows[start + ((int)threadIdx.x < count ? threadIdx.x : 0)];
  __syncthreads();
  mark(1);
  // Per-row facts the finish needs (lane i < TM: tile row i), issued now so their latency
  // hides under the gather rather than stalling the finish.
  int rdeg = 0;
  float rnorm = 1.f;
  if constexpr (AGG != AGG_NONE) {
    const int lrow = trow[min((int)(threadIdx.x & 63), TM - 1)];
    rdeg = p.rowptr[lrow + 1] - p.rowptr[lrow];
    if (AGG != AGG_LORENTZ) rnorm = p.norm[lrow];
  }

  // ---- operands: self-loop rows; pre-aggregated rows (AGG_NONE); gather.  The first
  // GEMM's B ring is issued before the A tiles (it depends on nothing), except on tiles
  // that gather inline, where it would sit in registers across the gather.
  const float* wsel = pos ? p.w_loop : p.w_evolve;
  const float* wfirst = (pos && p.w_n) ? p.w_n : wsel;
  // With the timestep fused, the time-gate GEMM (clamp(x_prev) @ W_g) depends only on staged
  // rows: it runs in the self-loop GEMM's k-loop (two MFMA chains, two B streams in flight)
  // instead of as a third serial GEMM in the epilogue.
  const bool gate_with_loop = STEP && wsel != nullptr;
  const bool prefetch = wfirst && !(gate_with_loop && wfirst == wsel);
  BRing br;
  if (!inline_gather && prefetch) br.load(wfirst, p.d);
  // inline gather: the self-loop rows stream into LDS while the gather's first indices load
  if (inline_gather) stage_rows_async(X, lda, p.x, trow, p.d);
  else stage_rows<false>(X, lda, p.x, trow, p.d, count);
  if (pos && AGG == AGG_NONE) stage_rows<false>(part, lda, p.agg, trow, p.d, count);
  if (!inline_gather) {
    if (STEP) stage_rows<true>(P2, lda, p.step.x_prev, trow, p.d, count);
    if (p.prev_t) stage_rows<false>(P1, lda, p.prev_t, trow, p.d, count);
  }
  if (inline_gather) {
    if constexpr (AGG != AGG_NONE) {
      tile_gather<AGG, S>(p, part, lda, trow, blockIdx.x, tmask, lds + L.xsh);
      __syncthreads();
      trace_mark(p, 12);
      tile_finish<AGG>(p, part, lda, trow, count, tmask, rdeg, rnorm);
      trace_mark(p, 13);
    }
    if (STEP) stage_rows<true>(P2, lda, p.step.x_prev, trow, p.d, count);
    if (p.prev_t) stage_rows<false>(P1, lda, p.prev_t, trow, p.d, count);
    if (prefetch) br.load(wfirst, p.d);
  }
  __syncthreads();
  mark(2);

  // ---- v = clamp(agg [@ W_n]) + x @ (W_loop | W_evolve)
  Frag v;
  v.zero();
  if (pos) {
    if (p.w_n) mfma_tile_pf(v, part, lda, p.w_n, p.d, br, p.d);
    else frag_from_tile(v, part, lda, p.d);
    if (!p.euclid) {
#pragma unroll
      for (int j = 0; j < TPW; ++j) v.t[j] = clamp4(v.t[j], -10.f, 10.f);
    }
  }
  // the self-loop message x @ W in its own accumulator, then added: the reference's order
  // (node_repr = clamp(agg) + loop_message, hyperbolic_layers.py:296-310, :672-683), and the
  // same bits as the phase launches (timestep.hip), which compute it in an earlier launch
  Frag tw;
  if (gate_with_loop) {
    Frag acc[2];
    acc[0].zero();
    acc[1].zero();
    const float* Ts[2] = {X, P2};
    const float* Ws[2] = {wsel, p.step.w_g};
    mfma_tiles<2, RING>(acc, Ts, Ws, lda, p.d, p.d);
#pragma unroll
    for (int j = 0; j < TPW; ++j) v.t[j] += acc[0].t[j];
    tw = acc[1];
  } else if (wsel) {
    Frag lp;
    lp.zero();
    if (wfirst == wsel && !(pos && p.w_n)) mfma_tile_pf(lp, X, lda, wsel, p.d, br, p.d);
    else mfma_tile(lp, X, lda, wsel, p.d, p.d);
#pragma unroll
    for (int j = 0; j < TPW; ++j) v.t[j] += lp.t[j];
  }
  mark(3);
  if (p.prev_t) {  // v = g v + (1 - g) prev_t, g = sigmoid(prev_t @ W_skip + b)
    Frag g;
    g.zero();
    mfma_tile(g, P1, lda, p.w_skip, p.d, p.d);
    Frag pt;
    frag_from_tile(pt, P1, lda, p.d);
    float b[TPW];
    col_load(b, p.b_skip, p.d);
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gt = sigmoidf(g.t[j][r] + b[j]);
        v.t[j][r] = gt * v.t[j][r] + (1.f - gt) * pt.t[j][r];
      }
  }
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    if (!p.euclid) v.t[j] = clamp4(v.t[j], -10.f, 10.f);
    v.t[j] = leaky4(v.t[j]);
  }
  if (p.drop_mask) {
    Frag m;
    frag_load(m, p.drop_mask, trow, count, p.d);
#pragma unroll
    for (int j = 0; j < TPW; ++j) v.t[j] *= m.t[j];
  }
  float n2[4];  // |row|^2 of v, carried through the row maps (rowtile.h)
  if (!p.euclid || p.r_next) rr.sumsq(v, n2);
  if (!p.euclid) exp0_known(v, n2, p.k);
  mark(4);

  if constexpr (STEP) {
    if (gate_with_loop) step_epilogue_tw(rr, v, n2, P2, lda, trow, count, p.step, tw, p.trace);
    else step_epilogue(rr, v, n2, P2, lda, trow, count, p.step, p.trace);
  } else {
    frag_store(v, p.h_out, trow, count, p.d);
    if (p.r_next) store_radius(n2, p.r_next, trow, count);
    if (p.x_next && !p.euclid) log0_known(v, n2, p.k);
    if (p.x_next) frag_store(v, p.x_next, trow, count, p.d);
  }
  mark(5);
  if (p.trace && threadIdx.x == 0) p.trace[blockIdx.x * 16 + 7] = (int64_t)__builtin_amdgcn_s_memtime();
}

// ================================================================================ timestep
template <bool ANA>
__global__ __launch_bounds__(NTHR) void k_timestep(StepArgs p) {
  extern __shared__ float lds[];
  const int lda = tile_lda(p.d);
  float* P = lds;
  RowRed rr{lds + TM * lda, 0};
  int* trow = reinterpret_cast<int*>(lds + TM * lda + RED_FLOATS);
  const int r0 = blockIdx.x * TM;
  const int n_valid = min(TM, p.V - r0);
  if (threadIdx.x < TM) trow[threadIdx.x] = r0 + (threadIdx.x < n_valid ? threadIdx.x : 0);
  __syncthreads();
  stage_rows<true>(P, lda, p.x_prev, trow, p.d, n_valid);
  Frag ct;
  frag_load(ct, p.hc, trow, n_valid, p.d);
  __syncthreads();
  float n2[4];
  rr.sumsq(ct, n2);
  step_epilogue<ANA>(rr, ct, n2, P, lda, trow, n_valid, p);
}

// ============================================================================ pack weights
// Wp[s][jq][lane][e] = W[4s + lane/16][16(4jq + e) + lane%16] (zero outside d_in x d_out).
__global__ void k_pack_weight(const float* __restrict__ W, int d_in, int d_out, float* __restrict__ Wp) {
  const int S = (d_in + 3) >> 2;
  const int total = S * 4 * 64 * 4;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int e = idx & 3, lane = (idx >> 2) & 63, jq = (idx >> 8) & 3, s = idx >> 10;
    const int k = 4 * s + (lane >> 4), n = 16 * (4 * jq + e) + (lane & 15);
    Wp[idx] = (k < d_in && n < d_out) ? W[(int64_t)k * d_out + n] : 0.f;
  }
}

// ============================================================================ launchers
template <int AGG, int S>
static void launch_layer(const LayerArgs& a, dim3 grid, size_t lds, hipStream_t st) {
  if (a.fuse_step)
    hipLaunchKernelGGL((k_layer<AGG, S, true>), grid, dim3(NTHR), lds, st, a);
  else
    hipLaunchKernelGGL((k_layer<AGG, S, false>), grid, dim3(NTHR), lds, st, a);
}

int layer(const LayerArgs& a, hipStream_t st) {
  if (a.d <= 0 || a.d > MAX_D || (a.d & 3)) return set_error(REGCN_EINVAL, "layer needs d %% 4 == 0, d <= 256 (d=%d)", a.d);
  if (!a.x || !a.rows || (!a.h_out && !a.fuse_step)) return set_error(REGCN_EINVAL, "null pointer");
  if ((a.w_loop == nullptr) != (a.w_evolve == nullptr)) return set_error(REGCN_EINVAL, "self-loop weights must come in pairs");
  if (a.prev_t && (!a.w_skip || !a.b_skip)) return set_error(REGCN_EINVAL, "skip needs weight and bias");
  if (a.n_pos < 0 || a.n_pos > a.V) return set_error(REGCN_EINVAL, "bad n_pos");
  const int mode = a.agg_mode;
  if (mode != AGG_NONE && mode != AGG_UNION && mode != AGG_EUCLID && mode != AGG_LORENTZ)
    return set_error(REGCN_EINVAL, "unknown aggregation mode %d", mode);
  if (mode == AGG_NONE && a.n_pos > 0 && !a.agg) return set_error(REGCN_EINVAL, "AGG_NONE needs agg rows");
  if (mode != AGG_NONE) {
    if (!a.rowptr || !a.col_src || !a.col_type || !a.rel) return set_error(REGCN_EINVAL, "gather needs CSR + rel");
    if (mode == AGG_UNION && !a.radius) return set_error(REGCN_EINVAL, "union gather needs radius");
    if (mode != AGG_LORENTZ && !a.norm) return set_error(REGCN_EINVAL, "gather needs norm");
    if (mode == AGG_LORENTZ && (!a.w_rel || a.nb <= 0 || a.d % a.nb))
      return set_error(REGCN_EINVAL, "lorentz gather needs weights and d %% num_bases == 0");
    if (!a.tiles || !a.item_ptr || a.n_pos_tiles < 0)
      return set_error(REGCN_EINVAL, "inline gather needs tiles and item lists");
  }
  if ((mode == AGG_UNION || mode == AGG_LORENTZ) && a.euclid) return set_error(REGCN_EINVAL, "hyperbolic gather with euclid tail");
  if (a.fuse_step) {
    const StepArgs& s = a.step;
    if (a.euclid) return set_error(REGCN_EINVAL, "the fused timestep is hyperbolic only");
    if (!s.x_prev || !s.w_g || !s.b_g || !s.r_static || !s.h_out) return set_error(REGCN_EINVAL, "null timestep pointer");
    if (s.residual && (!s.w_r || !s.b_r)) return set_error(REGCN_EINVAL, "residual radius needs w_r and b_r");
    if (s.d != a.d || s.V != a.V) return set_error(REGCN_EINVAL, "timestep shape mismatch");
  }
  if (a.V == 0) return 0;
  const int n_pos_tiles = (a.tiles && mode != AGG_NONE) ? a.n_pos_tiles : (a.n_pos + TM - 1) / TM;
  LayerArgs b = a;
  if (mode == AGG_NONE) b.tiles = nullptr;
  b.n_pos_tiles = n_pos_tiles;
  const unsigned grid = (unsigned)(n_pos_tiles + (a.V - a.n_pos + TM - 1) / TM);
  const int s = mode == AGG_LORENTZ ? a.d / a.nb : 1;
  const bool gen = mode == AGG_LORENTZ && s != 1 && s != 2 && s != 4;
  const size_t lds = (size_t)lds_layout(a.d, gen, layer_part_rows(a.prev_t != nullptr, a.fuse_step != 0)).total_bytes;
  switch (mode) {
    case AGG_NONE: launch_layer<AGG_NONE, 1>(b, dim3(grid), lds, st); break;
    case AGG_UNION: launch_layer<AGG_UNION, 1>(b, dim3(grid), lds, st); break;
    case AGG_EUCLID: launch_layer<AGG_EUCLID, 1>(b, dim3(grid), lds, st); break;
    default:
      if (s == 1) launch_layer<AGG_LORENTZ, 1>(b, dim3(grid), lds, st);
      else if (s == 2) launch_layer<AGG_LORENTZ, 2>(b, dim3(grid), lds, st);
      else if (s == 4) launch_layer<AGG_LORENTZ, 4>(b, dim3(grid), lds, st);
      else launch_layer<AGG_LORENTZ, 0>(b, dim3(grid), lds, st);
  }
  return check_launch("k_layer");
}

int timestep(const StepArgs& a, hipStream_t st, bool analysis) {
  if (a.d <= 0 || a.d > MAX_D || (a.d & 3)) return set_error(REGCN_EINVAL, "timestep needs d %% 4 == 0, d <= 256");
  if (!a.hc || !a.x_prev || !a.w_g || !a.b_g || !a.r_static || !a.h_out) return set_error(REGCN_EINVAL, "null pointer");
  if (a.residual && (!a.w_r || !a.b_r)) return set_error(REGCN_EINVAL, "residual radius needs w_r and b_r");
  if (analysis && !a.gate_out) return set_error(REGCN_EINVAL, "analysis needs gate_out");
  if (a.V == 0) return 0;
  const unsigned grid = (unsigned)((a.V + TM - 1) / TM);
  const size_t lds = (size_t)(TM * tile_lda(a.d) + RED_FLOATS + TM) * 4;
  if (analysis) hipLaunchKernelGGL(k_timestep<true>, dim3(grid), dim3(NTHR), lds, st, a);
  else hipLaunchKernelGGL(k_timestep<false>, dim3(grid), dim3(NTHR), lds, st, a);
  return check_launch("k_timestep");
}

size_t packed_weight_floats(int d_in) { return (size_t)((d_in + 3) / 4) * 4 * 64 * 4; }

int pack_weight(const float* W, int d_in, int d_out, float* Wp, hipStream_t st) {
  if (!W || !Wp) return set_error(REGCN_EINVAL, "null pointer");
  if (d_in <= 0 || d_out <= 0 || d_out > MAX_D) return set_error(REGCN_EINVAL, "pack_weight needs d_out <= 256");
  const int total = (int)packed_weight_floats(d_in);
  hipLaunchKernelGGL(k_pack_weight, dim3((total + 255) / 256), dim3(256), 0, st, W, d_in, d_out, Wp);
  return check_launch("k_pack_weight");
}

}  // namespace regcn
