// One timestep of the recurrent encoder in three phase launches on one stream
// (hyperbolic_model.py:797-884 with a 2-layer cell).
//
// The per-layer launches (layer.hip) put a tile's whole layer behind its gather: on a small
// snapshot (ICEWS: ~20 in-edge tiles beside ~430 tiles of rows without in-edges) the launch
// time is the in-edge tiles' latency chain gather -> finish -> GEMMs -> epilogue.  Work that
// does not depend on a gather moves to an earlier launch, and work of rows without in-edges
// (their layers are row-local maps) rides in whichever launch has room:
//
//   A  relation GRU, x-half (k_gru_x blocks: relation means over r_to_e + W_ih^x)
//      in-edge rows:  s1 = x0 @ W_loop[0],  tw = clamp(x0) @ W_g      (two MFMA chains)
//      other rows:    layer 0: x1 = log0(exp0(rrelu(clamp(x0 @ W_evolve[0]))))
//   B  in-edge tiles: layer-0 gather (messages need h_0 from A) -> finish ->
//                     v = clamp(agg [@ W_n[0]]) + s1 -> x1, r1;  then s1 = x1 @ W_loop[1]
//                     (layer 1's self-loop message, off phase C's critical path)
//      other rows:    layer 1: h2 = exp0(rrelu(clamp(x1 @ W_evolve[1] [skip on x0]))), |h2|^2
//      relation GRU pre-half of the NEXT timestep (k_gru_pre blocks: needs h_0 from A)
//   C  in-edge tiles: layer-1 gather (x1, r1 from B) -> finish ->
//                     v = clamp(agg [@ W_n[1]]) + s1 [skip] -> timestep epilogue
//                     with the gate pre-activation tw from A
//      other rows:    timestep epilogue on h2 with tw = clamp(x0) @ W_g
//
// Each row's op sequence and MFMA k-order equal the per-layer launches' (the self-loop
// message is accumulated on its own and then added in both, the reference order), so the
// outputs are bit-identical to regcn_layer_f32 x 2 with fuse_step.  Scratch between the
// phases (V x d each: s1, tw, x1, h2; V: r1, n2) stays in HBM / the Infinity Cache.  Phase A
// holds the relation GRU, the head of every timestep's critical path, with little beside it.
#include "layer_parts.h"
#include "gru_parts.h"

namespace regcn {

// profiling (regcn_set_trace): TRACE_SLOTS stamps per workgroup, 0 = start, TRACE_SLOTS - 1 =
// end, intermediate stamps 1 .. TRACE_SLOTS - 2 (wave 0)
constexpr int TRACE_SLOTS = 8;
__device__ __forceinline__ void mid_stamp(const PhaseArgs& p, int k) {
  if (p.trace && threadIdx.x == 0) p.trace[TRACE_SLOTS * blockIdx.x + k] = (int64_t)__builtin_amdgcn_s_memrealtime();
}

// Rows [start, start + count) of the snapshot's row list into trow; returns count.
__device__ __forceinline__ int load_trow(int* trow, const int* rows, int start, int count) {
  if (threadIdx.x < TM) trow[threadIdx.x] = rows[start + ((int)threadIdx.x < count ? threadIdx.x : 0)];
  __syncthreads();
  return count;
}

__device__ __forceinline__ bool row_hot(const int* rowptr, int v) { return rowptr[v + 1] > rowptr[v]; }

// Tile b of the rows without in-edges that run at this timestep.  Plain mode: rows[n_pos:V].
// Memo mode: entries [16 b, 16 b + 16) of the earlier snapshots' in-edge rows, concatenated;
// entry v of snapshot t' runs iff v has no in-edge now nor at any snapshot after t' (so a
// row runs once, for its last earlier snapshot), compacted by a ballot in every wave.
// Returns the tile's row count (0: nothing to run; uniform over the workgroup).
__device__ __forceinline__ int zero_tile_rows(const PhaseArgs& p, int b, int* trow) {
  const LayerArgs& l = p.L[0];
  if (!p.memo_h) {
    const int start = b * TM, zn = l.V - l.n_pos;
    if (start >= zn) return 0;
    return load_trow(trow, l.rows + l.n_pos, start, min(TM, zn - start));
  }
  const int lane = threadIdx.x & 63;
  int v = 0;
  bool ok = false;
  if (lane < TM) {
    int e = b * TM + lane, tp = -1;
    for (int i = 0; i < p.n_prev; ++i) {
      if (e < p.prev_n_pos[i]) {
        tp = i;
        break;
      }
      e -= p.prev_n_pos[i];
    }
    if (tp >= 0) {
      v = p.prev_rows[tp][e];
      ok = !row_hot(l.rowptr, v);
      for (int i = tp + 1; i < p.n_prev && ok; ++i) ok = !row_hot(p.prev_rowptr[i], v);
    }
  }
  const uint64_t m = __ballot(ok);
  if (ok && wave_id() == 0) trow[__popcll(m & ((1ull << lane) - 1ull))] = v;
  __syncthreads();
  return __popcll(m);
}

// Phase A, memo mode: this timestep's output rows start as the memoised pristine state
// (the running rows overwrite theirs in phase C).  Bandwidth work at the lowest priority.
__device__ __forceinline__ void copy_block(const PhaseArgs& p, int b) {
  __builtin_amdgcn_s_setprio(0);
  const int64_t n4 = (int64_t)p.L[0].V * p.d / 4, stride = (int64_t)p.n_copy * NTHR;
  const f4* hs = reinterpret_cast<const f4*>(p.memo_h);
  const f4* xs = reinterpret_cast<const f4*>(p.memo_x);
  f4* hd = reinterpret_cast<f4*>(p.step.h_out);
  f4* xd = reinterpret_cast<f4*>(p.step.x_out);
  for (int64_t i = (int64_t)b * NTHR + threadIdx.x; i < n4; i += stride) {
    const f4 h = hs[i], x = xs[i];
    hd[i] = h;
    xd[i] = x;
  }
  for (int64_t i = (int64_t)b * NTHR + threadIdx.x; i < p.L[0].V; i += stride) p.step.r_out[i] = p.memo_r[i];
}

__device__ __forceinline__ void store_rows_scalar(const float n2[4], float* __restrict__ out, const int* rows,
                                                  int n_valid) {
  if ((threadIdx.x & 15) == 0 && wave_id() == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = frag_row(r);
      if (i < n_valid) out[rows[i]] = n2[r];
    }
  }
}

__device__ __forceinline__ void load_rows_scalar(float n2[4], const float* __restrict__ in, const int* rows,
                                                 int n_valid) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = frag_row(r);
    const float v = in[rows[i < n_valid ? i : 0]];
    n2[r] = i < n_valid ? v : 0.f;
  }
}

__device__ __forceinline__ void rrelu_clamp(Frag& v) {
#pragma unroll
  for (int j = 0; j < TPW; ++j) v.t[j] = leaky4(clamp4(v.t[j], -10.f, 10.f));
}

// v = g v + (1 - g) P, g = sigmoid(P @ W_skip + b)  (hyperbolic_layers.py:678-681)
__device__ __forceinline__ void skip_gate(Frag& v, const float* P, int lda, const float* w_skip, const float* b_skip,
                                          int d) {
  Frag g;
  g.zero();
  mfma_tile(g, P, lda, w_skip, d, d);
  Frag pt;
  frag_from_tile(pt, P, lda, d);
  float b[TPW];
  col_load(b, b_skip, d);
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float gt = sigmoidf(g.t[j][r] + b[j]);
      v.t[j][r] = gt * v.t[j][r] + (1.f - gt) * pt.t[j][r];
    }
}

// ------------------------------------------------------------------------------- phase A
// In-edge rows (plain 16-row tiles over rows[:n_pos]): the two GEMMs that need only x0, one
// per workgroup (block 2 t: s1 = x0 @ W_loop[0]; block 2 t + 1: tw = clamp(x_prev) @ W_g), so
// the phase's critical path is one GEMM deep.
__device__ __forceinline__ void a_pos_rows(const PhaseArgs& p, int b, float* lds) {
  const int lda = tile_lda(p.d);
  float* X = lds;
  int* trow = reinterpret_cast<int*>(lds + TM * lda);
  const bool gate = (b & 1) || !p.L[0].w_loop;
  const int start = (b >> 1) * TM;
  const int count = load_trow(trow, p.L[0].rows, start, min(TM, p.L[0].n_pos - start));
  BRing br;
  br.load(gate ? p.step.w_g : p.L[0].w_loop, p.d);
  if (gate) stage_rows<true>(X, lda, p.step.x_prev, trow, p.d, count);
  else stage_rows<false>(X, lda, p.L[0].x, trow, p.d, count);
  __syncthreads();
  Frag acc;
  acc.zero();
  mfma_tile_pf(acc, X, lda, gate ? p.step.w_g : p.L[0].w_loop, p.d, br, p.d);
  frag_store(acc, gate ? p.tw : p.s1, trow, count, p.d);
}

// ------------------------------------------------------------------ in-edge tiles, B and C
// LDS of an in-edge tile: `part_rows` rows for the gather partials (TM + NWAVE - 1) and,
// after the finish, the operand tiles; the cross-wave reduction scratch; the row ids.
// Sized per phase so the launch's occupancy is not set by a layout it does not use.
struct GLds {
  int lda, part, red, ints, xsh, total_bytes;
};
__host__ __device__ inline GLds glds(int d, bool gen_s, int part_rows) {
  GLds L;
  L.lda = tile_lda(d);
  L.part = 0;
  L.red = part_rows * L.lda;
  L.ints = L.red + RED_FLOATS;
  L.xsh = L.ints + 32;  // trow[16], tmask[NWAVE] (+pad)
  L.total_bytes = (L.xsh + (gen_s ? NWAVE * MAX_D : 0)) * 4;
  return L;
}
constexpr int GATHER_ROWS = TM + NWAVE - 1;
__host__ __device__ inline int c_part_rows(bool skip) { return skip ? 3 * TM : 2 * TM; }

// A tile's rows of a row-major matrix held in registers between the load and the LDS
// store (stage_rows split in two), so the load latency hides under other work.
struct RowRegs {
  static constexpr int IT = TM * (MAX_D / 4) / NTHR;
  f4 v[IT];
  __device__ __forceinline__ void load(const float* __restrict__ A, const int* rows, int d, int n_valid) {
    const int q4 = d >> 2, n = TM * q4;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = min((int)threadIdx.x + it * NTHR, n - 1);
      const int i = idx / q4, c = (idx - i * q4) * 4;
      v[it] = *reinterpret_cast<const f4*>(A + (int64_t)rows[i < n_valid ? i : 0] * d + c);
    }
  }
  template <bool CLAMP10>
  __device__ __forceinline__ void store(float* T, int lda, int d, int n_valid) const {
    const int q4 = d >> 2, n = TM * q4;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = threadIdx.x + it * NTHR;
      if (idx >= n) break;
      const int i = idx / q4, c = (idx - i * q4) * 4;
      f4 x = v[it];
      if (CLAMP10) x = clamp4(x, -10.f, 10.f);
      if (i >= n_valid) x = f4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f4*>(T + i * lda + c) = x;
    }
  }
};

// The rows of destination tile `tile` into trow, plus each lane's row degree / norm for the
// finish; returns the row count.
struct TileRows {
  int count, rdeg;
  float rnorm;
};
template <int AGG>
__device__ __forceinline__ TileRows tile_rows(const LayerArgs& l, int tile, int* trow) {
  TileRows t;
  const int start = l.tiles[2 * tile];
  t.count = load_trow(trow, l.rows, start, l.tiles[2 * tile + 1]);
  const int lrow = trow[min((int)(threadIdx.x & 63), TM - 1)];
  t.rdeg = l.rowptr[lrow + 1] - l.rowptr[lrow];
  t.rnorm = AGG != AGG_LORENTZ ? l.norm[lrow] : 1.f;
  return t;
}

// Gather + finish of destination tile `tile` for layer l (layer.hip k_layer's pos path).
template <int AGG, int S>
__device__ __forceinline__ void gather_finish(const PhaseArgs& p, const LayerArgs& l, int tile, float* lds,
                                              const GLds& L, int* trow, const TileRows& t) {
  float* part = lds + L.part;
  int* tmask = trow + TM;
  mid_stamp(p, 1);
  tile_gather<AGG, S>(l, part, L.lda, trow, tile, tmask, lds + L.xsh);
  mid_stamp(p, 2);
  __syncthreads();
  tile_finish<AGG>(l, part, L.lda, trow, t.count, tmask, t.rdeg, t.rnorm);
  mid_stamp(p, 3);
}

template <int AGG, int S>
__device__ __forceinline__ int gather_tile(const PhaseArgs& p, const LayerArgs& l, int tile, float* lds, const GLds& L,
                                           int* trow) {
  const TileRows t = tile_rows<AGG>(l, tile, trow);
  gather_finish<AGG, S>(p, l, tile, lds, L, trow, t);
  return t.count;
}

// v = clamp(agg [@ W_n]) from the finished tile in `part`; the B ring of W_n (if any) is
// loaded by the caller behind the gather.
__device__ __forceinline__ void agg_term(Frag& v, const LayerArgs& l, const float* part, int lda, BRing& br) {
  v.zero();
  if (l.w_n) mfma_tile_pf(v, part, lda, l.w_n, l.d, br, l.d);
  else frag_from_tile(v, part, lda, l.d);
#pragma unroll
  for (int j = 0; j < TPW; ++j) v.t[j] = clamp4(v.t[j], -10.f, 10.f);
}

template <int AGG, int S>
__device__ __forceinline__ void b_pos_tile(const PhaseArgs& p, int tile, float* lds) {
  const LayerArgs& l = p.L[0];
  const GLds L = glds(p.d, AGG == AGG_LORENTZ && S == 0, GATHER_ROWS);
  int* trow = reinterpret_cast<int*>(lds + L.ints);
  RowRed rr{lds + L.red, 0};
  const TileRows tr = tile_rows<AGG>(l, tile, trow);
  const int count = tr.count;
  Frag lp;  // the self-loop message from phase A, in flight under the gather
  if (l.w_loop) frag_load(lp, p.s1, trow, count, p.d);
  gather_finish<AGG, S>(p, l, tile, lds, L, trow, tr);
  BRing br;
  if (l.w_n) br.load(l.w_n, p.d);
  __syncthreads();
  Frag v;
  agg_term(v, l, lds + L.part, L.lda, br);
  if (l.w_loop) {
#pragma unroll
    for (int j = 0; j < TPW; ++j) v.t[j] += lp.t[j];
  }
  rrelu_clamp(v);
  float n2[4];
  rr.sumsq(v, n2);
  mid_stamp(p, 4);
  exp0_known(v, n2, l.k);
  store_radius(n2, p.r1, trow, count);
  log0_known(v, n2, l.k);
  frag_store(v, p.x1, trow, count, p.d);
  mid_stamp(p, 5);
  // layer 1's self-loop message x1 @ W_loop[1] of these rows: it needs no gather, so it
  // leaves phase C's critical path for this one (into s1: this tile read its s1 rows above)
  const LayerArgs& l1 = p.L[1];
  if (l1.w_loop) {
    BRing br1;
    br1.load(l1.w_loop, p.d);
    float* X = lds + L.part;  // the finished tile is consumed
    frag_to_tile(v, X, L.lda, count, p.d);
    __syncthreads();
    Frag lp;
    lp.zero();
    mfma_tile_pf(lp, X, L.lda, l1.w_loop, p.d, br1, p.d);
    mid_stamp(p, 6);
    frag_store(lp, p.s1, trow, count, p.d);
  }
}

template <int AGG, int S>
__device__ __forceinline__ void c_pos_tile(const PhaseArgs& p, int tile, float* lds) {
  const LayerArgs& l = p.L[1];
  const bool skip = l.prev_t != nullptr;
  const GLds L = glds(p.d, AGG == AGG_LORENTZ && S == 0, c_part_rows(skip));
  const int lda = L.lda;
  float* part = lds + L.part;
  float* P2 = part + TM * lda;      // clamp(x0): the timestep gate operand
  float* P1 = part + 2 * TM * lda;  // skip operand: the cell input x0
  int* trow = reinterpret_cast<int*>(lds + L.ints);
  RowRed rr{lds + L.red, 0};
  const TileRows tr = tile_rows<AGG>(l, tile, trow);
  const int count = tr.count;
  // operand rows in flight under the gather: x_prev (gate blend), tw (gate pre-activation,
  // phase A), s1 = x1 @ W_loop[1] (phase B), the skip operand
  RowRegs r2, r1;
  r2.load(p.step.x_prev, trow, p.d, count);
  if (skip) r1.load(l.prev_t, trow, p.d, count);
  Frag tw, lp;
  frag_load(tw, p.tw, trow, count, p.d);
  if (l.w_loop) frag_load(lp, p.s1, trow, count, p.d);
  gather_finish<AGG, S>(p, l, tile, lds, L, trow, tr);
  BRing br;
  if (l.w_n) br.load(l.w_n, p.d);
  __syncthreads();
  Frag v;
  agg_term(v, l, part, lda, br);
  __syncthreads();  // the finished tile is consumed: its rows take the operands
  mid_stamp(p, 4);
  r2.store<true>(P2, lda, p.d, count);
  if (skip) r1.store<false>(P1, lda, p.d, count);
  __syncthreads();
  if (l.w_loop) {
#pragma unroll
    for (int j = 0; j < TPW; ++j) v.t[j] += lp.t[j];
  }
  if (skip) skip_gate(v, P1, lda, l.w_skip, l.b_skip, p.d);
  mid_stamp(p, 5);
  rrelu_clamp(v);
  float n2[4];
  rr.sumsq(v, n2);
  exp0_known(v, n2, l.k);
  step_epilogue_tw(rr, v, n2, P2, lda, trow, count, p.step, tw);
}

// ------------------------------------------------------------ rows without in-edges, B, C
// Layers 0 and 1 of a tile of rows without in-edges (k_layer's zero-tile paths), the
// layer-0 output kept in LDS -> h2 (Poincare rows) and |h2|^2 as the epilogue carries it.
__device__ __forceinline__ void a_zero_rows(const PhaseArgs& p, int b, float* lds) {
  const LayerArgs& l0 = p.L[0];
  const int lda = tile_lda(p.d);
  float* X = lds;  // x0
  RowRed rr{lds + TM * lda, 0};
  int* trow = reinterpret_cast<int*>(lds + TM * lda + RED_FLOATS);
  const int count = zero_tile_rows(p, b, trow);
  if (!count) return;
  BRing br;
  if (l0.w_evolve) br.load(l0.w_evolve, p.d);
  stage_rows<false>(X, lda, l0.x, trow, p.d, count);
  __syncthreads();
  Frag v;
  v.zero();
  if (l0.w_evolve) {
    Frag lp;
    lp.zero();
    mfma_tile_pf(lp, X, lda, l0.w_evolve, p.d, br, p.d);
#pragma unroll
    for (int j = 0; j < TPW; ++j) v.t[j] += lp.t[j];
  }
  rrelu_clamp(v);
  float n2[4];
  rr.sumsq(v, n2);
  exp0_known(v, n2, l0.k);
  log0_known(v, n2, l0.k);
  frag_store(v, p.x1, trow, count, p.d);
}

// Layer 1 of a tile of rows without in-edges (their layer 0 ran in phase A: x1 in HBM)
// -> h2 (Poincare rows) and |h2|^2 as the epilogue carries it.
__device__ __forceinline__ void b_zero_rows(const PhaseArgs& p, int b, float* lds) {
  const LayerArgs& l = p.L[1];
  const int lda = tile_lda(p.d);
  float* X = lds;                // the skip operand: the cell input x0
  float* X1 = lds + TM * lda;    // layer-0 output x1
  RowRed rr{lds + 2 * TM * lda, 0};
  int* trow = reinterpret_cast<int*>(lds + 2 * TM * lda + RED_FLOATS);
  const int count = zero_tile_rows(p, b, trow);
  if (!count) return;
  mid_stamp(p, 1);
  BRing br;
  if (l.w_evolve) br.load(l.w_evolve, p.d);
  stage_rows<false>(X1, lda, p.x1, trow, p.d, count);
  if (l.prev_t) stage_rows<false>(X, lda, p.L[0].x, trow, p.d, count);
  __syncthreads();
  mid_stamp(p, 2);
  Frag v;
  v.zero();
  if (l.w_evolve) {
    Frag lp;
    lp.zero();
    mfma_tile_pf(lp, X1, lda, l.w_evolve, p.d, br, p.d);
#pragma unroll
    for (int j = 0; j < TPW; ++j) v.t[j] += lp.t[j];
  }
  if (l.prev_t) skip_gate(v, X, lda, l.w_skip, l.b_skip, p.d);
  rrelu_clamp(v);
  float n2[4];
  rr.sumsq(v, n2);
  exp0_known(v, n2, l.k);
  frag_store(v, p.h2, trow, count, p.d);
  store_rows_scalar(n2, p.n2, trow, count);
}

__device__ __forceinline__ void c_zero_rows(const PhaseArgs& p, int b, float* lds) {
  const int lda = tile_lda(p.d);
  float* P2 = lds;
  RowRed rr{lds + TM * lda, 0};
  int* trow = reinterpret_cast<int*>(lds + TM * lda + RED_FLOATS);
  const int count = zero_tile_rows(p, b, trow);
  if (!count) return;
  BRing br;
  br.load(p.step.w_g, p.d);
  stage_rows<true>(P2, lda, p.step.x_prev, trow, p.d, count);
  Frag v;
  frag_load(v, p.h2, trow, count, p.d);
  float n2[4];
  load_rows_scalar(n2, p.n2, trow, count);
  __syncthreads();
  mid_stamp(p, 1);
  Frag tw;
  tw.zero();
  mfma_tile_pf(tw, P2, lda, p.step.w_g, p.d, br, p.d);
  mid_stamp(p, 2);
  step_epilogue_tw(rr, v, n2, P2, lda, trow, count, p.step, tw);
}

// ---------------------------------------------------------------------------- the kernels
// Block order puts the longest chains first: the dispatcher hands out blocks in order.
struct PhaseStamp {  // profiling: a workgroup's start / end (100 MHz) when p.trace is set
  const PhaseArgs& p;
  __device__ __forceinline__ explicit PhaseStamp(const PhaseArgs& a) : p(a) {
    if (p.trace && threadIdx.x == 0) p.trace[TRACE_SLOTS * blockIdx.x] = (int64_t)__builtin_amdgcn_s_memrealtime();
  }
  __device__ __forceinline__ ~PhaseStamp() {
    if (p.trace) {
      __syncthreads();
      if (threadIdx.x == 0) p.trace[TRACE_SLOTS * blockIdx.x + TRACE_SLOTS - 1] = (int64_t)__builtin_amdgcn_s_memrealtime();
    }
  }
};

__global__ __launch_bounds__(NTHR) void k_phase_a(PhaseArgs p) {
  extern __shared__ float lds[];
  PhaseStamp stamp(p);
  int b = blockIdx.x;
  // every block of A is on the timestep's critical path; the dispatcher hands blocks out in
  // order, so the longest go first: rows without in-edges (layer 0, ~11 us at GDELT's late
  // timesteps), the relation GRU x-half (~10 us), the in-edge rows' GEMMs (~8 us), the memo
  // copy (~4 us).  (GDELT timestep 6 with the zero rows last: they started at 8.4 us behind
  // the GRU blocks and set the 25 us span, profiles/r6_phasetrace_gdelt.log.)
  __builtin_amdgcn_s_setprio(2);
  // (the zero-row segment is padded to a multiple of 8 blocks, so the GRU blocks' XCD grouping
  // -- blocks g and g + 8 on one XCD -- holds; the pads return at once)
  const int zpad = gru_blocks_padded(p.n_zero_rt);
  if (b < zpad) {
    if (b < p.n_zero_rt) a_zero_rows(p, b, lds);
    return;
  }
  b -= zpad;
  if (b < gru_blocks_padded(p.n_gru)) {
    int bx, by;
    if (gru_block_xcd(b, p.n_gru, p.gru_rt, bx, by)) gru_x_block(p.gru, bx, by, lds);
    return;
  }
  b -= gru_blocks_padded(p.n_gru);
  if (b < 2 * p.n_pos_rt) {
    if ((b & 1) == 0 && !p.L[0].w_loop) return;  // no self loop: the gate GEMM only
    return a_pos_rows(p, b, lds);
  }
  copy_block(p, b - 2 * p.n_pos_rt);
}

template <int AGG, int S>
__global__ __launch_bounds__(NTHR) void k_phase_b(PhaseArgs p) {
  extern __shared__ float lds[];
  PhaseStamp stamp(p);
  int b = blockIdx.x;
  // in-edge tiles carry the critical path; rows without in-edges and the next GRU pre-half
  // fill the SIMDs' idle issue slots at the default priority
  if (b < p.L[0].n_pos_tiles) {
    __builtin_amdgcn_s_setprio(2);
    return b_pos_tile<AGG, S>(p, b, lds);
  }
  b -= p.L[0].n_pos_tiles;
  if (b < p.n_zero_rt) return b_zero_rows(p, b, lds);
  b -= p.n_zero_rt;
  int bx, by;
  if (gru_block_xcd(b, p.n_gru, p.gru_rt, bx, by)) gru_pre_block(p.gru, bx, by, lds);
}

template <int AGG, int S>
__global__ __launch_bounds__(NTHR) void k_phase_c(PhaseArgs p) {
  extern __shared__ float lds[];
  PhaseStamp stamp(p);
  int b = blockIdx.x;
  if (b < p.L[1].n_pos_tiles) {
    __builtin_amdgcn_s_setprio(2);
    return c_pos_tile<AGG, S>(p, b, lds);
  }
  b -= p.L[1].n_pos_tiles;
  c_zero_rows(p, b, lds);
}

// ------------------------------------------------------------------------------ launchers
template <int AGG, int S>
static void launch_bc(const PhaseArgs& a, int phase, unsigned grid, size_t lds, hipStream_t st) {
  if (phase == 1) hipLaunchKernelGGL((k_phase_b<AGG, S>), dim3(grid), dim3(NTHR), lds, st, a);
  else hipLaunchKernelGGL((k_phase_c<AGG, S>), dim3(grid), dim3(NTHR), lds, st, a);
}

int timestep_phase(PhaseArgs a, int phase, hipStream_t st) {
  const LayerArgs& l0 = a.L[0];
  const int d = a.d;
  if (d <= 0 || d > MAX_D || (d & 3)) return set_error(REGCN_EINVAL, "phase needs d %% 4 == 0, d <= 256 (d=%d)", d);
  if (phase < 0 || phase > 2) return set_error(REGCN_EINVAL, "phase must be 0 (A), 1 (B) or 2 (C)");
  const int mode = l0.agg_mode;
  if (mode != AGG_UNION && mode != AGG_LORENTZ) return set_error(REGCN_EINVAL, "phases support the union and Lorentz layers");
  if (!l0.rows || !l0.x || !a.step.x_prev || !a.step.w_g || !a.step.h_out || !a.s1 || !a.tw || !a.x1 || !a.r1 ||
      !a.h2 || !a.n2)
    return set_error(REGCN_EINVAL, "null pointer");
  if (a.L[0].prev_t) return set_error(REGCN_EINVAL, "layer 0 has no skip connection");
  if (a.L[1].prev_t && (!a.L[1].w_skip || !a.L[1].b_skip)) return set_error(REGCN_EINVAL, "skip needs weight and bias");
  if (l0.n_pos > 0 && phase > 0) {  // the gathers (phase A reads no message operand)
    for (int i = 0; i < 2; ++i) {
      const LayerArgs& l = a.L[i];
      if (!l.rowptr || !l.rel || !l.tiles || !l.item_ptr) return set_error(REGCN_EINVAL, "gather needs CSR, tiles, rel");
      if (mode == AGG_UNION && (!l.radius || !l.norm)) return set_error(REGCN_EINVAL, "union gather needs radius, norm");
      if (mode == AGG_LORENTZ && (!l.w_rel || l.nb <= 0 || d % l.nb))
        return set_error(REGCN_EINVAL, "lorentz gather needs weights and d %% num_bases == 0");
    }
  }
  int n_zero = a.skip_zero_rows ? 0 : l0.V - l0.n_pos;
  if (a.memo_h) {
    n_zero = 0;
    for (int i = 0; i < a.n_prev; ++i) n_zero += a.prev_n_pos[i];
  }
  const int n_zero_rt = (n_zero + TM - 1) / TM;
  a.n_copy = a.memo_h ? std::min(128, (int)(((int64_t)l0.V * d / 4 + NTHR * 8 - 1) / (NTHR * 8))) : 0;
  a.n_zero_rt = n_zero_rt;
  a.trace = g_trace;
  a.n_pos_rt = (l0.n_pos + TM - 1) / TM;
  a.gru_rt = (a.gru.R2 + TM - 1) / TM;
  const int gru_blocks = a.gru_rt * (gru_dpad(d) / 16);
  const int s = mode == AGG_LORENTZ ? d / l0.nb : 1;
  const bool gen = mode == AGG_LORENTZ && s != 1 && s != 2 && s != 4;
  const bool skip = a.L[1].prev_t != nullptr;
  const size_t tile = (size_t)TM * tile_lda(d) * 4, small = (size_t)(RED_FLOATS + TM) * 4;
  size_t lds = 0;
  unsigned grid = 0;
  if (phase == 0) {
    a.n_gru = a.gru.h_out ? gru_blocks : 0;
    if (a.n_gru && (!a.gru.h_prev || !a.gru.w_ih_x || !a.gru.pre || (!a.gru.x_mean && !a.gru.rel_start)))
      return set_error(REGCN_EINVAL, "GRU x-phase operands missing");
    grid = (unsigned)(gru_blocks_padded(n_zero_rt) + gru_blocks_padded(a.n_gru) + 2 * a.n_pos_rt + a.n_copy);
    lds = std::max({2 * tile + TM * 4, tile + small, a.n_gru ? gru_x_lds_bytes(d) : 0});
    if (grid) hipLaunchKernelGGL(k_phase_a, dim3(grid), dim3(NTHR), lds, st, a);
    return grid ? check_launch("k_phase_a") : 0;
  }
  if (phase == 1) {
    a.n_gru = a.gru.pre ? gru_blocks : 0;
    if (a.n_gru && (!a.gru.emb_rel || !a.gru.h_prev || !a.gru.w_ih_e || !a.gru.w_hh || !a.gru.b_ih || !a.gru.b_hh))
      return set_error(REGCN_EINVAL, "GRU pre-phase operands missing");
    grid = (unsigned)(l0.n_pos_tiles + n_zero_rt + gru_blocks_padded(a.n_gru));
    lds = std::max({(size_t)glds(d, gen, GATHER_ROWS).total_bytes, 2 * tile + small,
                    a.n_gru ? gru_pre_lds_bytes(d) : 0});
  } else {
    grid = (unsigned)(a.L[1].n_pos_tiles + n_zero_rt);
    lds = std::max((size_t)glds(d, gen, c_part_rows(skip)).total_bytes, tile + small);
  }
  if (!grid) return 0;
  if (mode == AGG_UNION) launch_bc<AGG_UNION, 1>(a, phase, grid, lds, st);
  else if (s == 1) launch_bc<AGG_LORENTZ, 1>(a, phase, grid, lds, st);
  else if (s == 2) launch_bc<AGG_LORENTZ, 2>(a, phase, grid, lds, st);
  else if (s == 4) launch_bc<AGG_LORENTZ, 4>(a, phase, grid, lds, st);
  else launch_bc<AGG_LORENTZ, 0>(a, phase, grid, lds, st);
  return check_launch(phase == 1 ? "k_phase_b" : "k_phase_c");
}

}  // namespace regcn
