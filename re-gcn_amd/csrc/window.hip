// History-window scheduling of the recurrent encoder.
//
// A row without in-edges in a snapshot receives no message in any layer: its cell and
// timestep are row-local maps whose operands are parameters only (W_evolve, the skip gate,
// the time gate, the static radius).  A row with no in-edge in ANY snapshot of the window
// ("cold", set C) therefore evolves over all T timesteps independently of the graphs and of
// every other row, and nothing else reads it before the decoder: with doubled edges every
// message source is itself a row with in-edges at that timestep (rgcn/utils.py:116-118).
//
//   regcn_window_plan_i32   flags[v] = bit t for each snapshot t where v has in-edges; then,
//                           in row order, C = {v : flags = 0}, U = {v : flags != 0} and per t
//                           Z_t = {v in U : bit t clear} (the U rows without in-edges at t)
//   k_cold_chain            C rows: T x (layer 0, layer 1, timestep) in one launch, the rows
//                           held in LDS between layers and timesteps, every timestep's h, x,
//                           r written out (history_embs)
//
// The phase launches (timestep.hip) then cover the U rows only: in-edge tiles plus Z_t.
// Each row's op sequence equals the per-layer launches' (same device functions, same MFMA
// k-order), so the outputs are bit-identical to them.
#include "layer_parts.h"

namespace regcn {

// ---------------------------------------------------------------------------------- plan
// One workgroup: zero the flags, OR in bit t for each snapshot's in-edge rows, then compact
// C / U / Z_t in row order, 1024 rows per pass: per list a wave ballot gives each row its
// rank in the wave, per-wave counts in LDS give the wave offsets (a 16-entry scan per list).
constexpr int PLAN_THREADS = 1024, PLAN_WAVES = PLAN_THREADS / 64, PLAN_LISTS = 2 + REGCN_MAX_WINDOW;
__global__ __launch_bounds__(PLAN_THREADS) void k_plan(PlanArgs p) {
  __shared__ int wofs[PLAN_LISTS][PLAN_WAVES];
  __shared__ int base[PLAN_LISTS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nl = 2 + p.T;
  for (int v = tid; v < p.V; v += PLAN_THREADS) p.flags[v] = 0;
  if (tid < PLAN_LISTS) base[tid] = 0;
  __threadfence();
  __syncthreads();
  for (int t = 0; t < p.T; ++t)
    for (int i = tid; i < p.n_pos[t]; i += PLAN_THREADS) atomicOr(p.flags + p.pos_rows[t][i], 1 << t);
  __threadfence();
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int v0 = 0; v0 < p.V; v0 += PLAN_THREADS) {
    const int v = v0 + tid;
    const unsigned f = v < p.V ? (unsigned)__hip_atomic_load(p.flags + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    bool in[PLAN_LISTS];
    int pos[PLAN_LISTS];
#pragma unroll
    for (int L = 0; L < PLAN_LISTS; ++L) {
      in[L] = v < p.V && L < nl && (L == 0 ? f == 0u : L == 1 ? f != 0u : (f != 0u && !((f >> (L - 2)) & 1u)));
      const uint64_t m = __ballot(in[L]);
      pos[L] = __popcll(m & lt);
      if (lane == 0) wofs[L][w] = __popcll(m);
    }
    __syncthreads();
    if (tid < nl) {  // exclusive scan of the per-wave counts, after the running base
      int s = base[tid];
      for (int ww = 0; ww < PLAN_WAVES; ++ww) {
        const int c = wofs[tid][ww];
        wofs[tid][ww] = s;
        s += c;
      }
      base[tid] = s;
    }
    __syncthreads();
#pragma unroll
    for (int L = 0; L < PLAN_LISTS; ++L) {
      if (!in[L]) continue;
      int* out = L == 0 ? p.c_rows : L == 1 ? p.u_rows : p.z_rows + (int64_t)(L - 2) * p.z_stride;
      out[wofs[L][w] + pos[L]] = v;
    }
    __syncthreads();
  }
  if (tid < nl) p.counts[tid] = base[tid];
}

int window_plan(const PlanArgs& a, hipStream_t st) {
  if (a.T < 1 || a.T > REGCN_MAX_WINDOW) return set_error(REGCN_EINVAL, "window plan needs 1..%d snapshots", REGCN_MAX_WINDOW);
  if (!a.flags || !a.c_rows || !a.u_rows || !a.z_rows || !a.counts) return set_error(REGCN_EINVAL, "null pointer");
  int max_pos = 0;
  for (int t = 0; t < a.T; ++t) {
    if (a.n_pos[t] < 0 || a.n_pos[t] > a.V || (a.n_pos[t] && !a.pos_rows[t])) return set_error(REGCN_EINVAL, "bad snapshot rows");
    max_pos = std::max(max_pos, a.n_pos[t]);
  }
  if (a.z_stride < std::min(a.V, [&] { int s = 0; for (int t = 0; t < a.T; ++t) s += a.n_pos[t]; return s; }()))
    return set_error(REGCN_EINVAL, "z_stride below the U bound");
  (void)max_pos;
  hipLaunchKernelGGL(k_plan, dim3(1), dim3(PLAN_THREADS), 0, st, a);
  return check_launch("k_plan");
}

// ----------------------------------------------------------------------------- cold chain
// 16 C rows per workgroup through T timesteps.  LDS tiles: XI = the timestep input x,
// X1 = layer-0 output, P2 = clamp(x) (time-gate operand).  Per timestep exactly the
// per-layer zero-tile path: layer 0 (k_layer<., ., false> zero tile), layer 1 with the
// timestep (k_layer<., ., true> zero tile: loop and gate GEMMs in one k-loop).
// SEQ: layer 1's two GEMMs one after the other (one B ring: fewer registers, more resident
// workgroups for the throughput-bound per-timestep launch); same k-order, same bits.
// trace (profiling, regcn_set_trace): 8 stamps per workgroup, 0 = start, 7 = end, 1-6 after
// staging / layer-0 GEMM / layer-0 epilogue / layer-1 GEMMs / skip + activation / timestep.
template <bool SEQ>
__device__ __forceinline__ void chain_tile(const ChainArgs& p, int tile, int n_rows, float* lds,
                                           int64_t* trace = nullptr) {
  auto stamp = [&](int k) {
    if (trace && threadIdx.x == 0) trace[8 * blockIdx.x + k] = (int64_t)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  const int lda = tile_lda(p.d);
  float* XI = lds;
  float* X1 = lds + TM * lda;
  float* P2 = lds + 2 * TM * lda;
  RowRed rr{lds + 3 * TM * lda, 0};
  int* trow = reinterpret_cast<int*>(lds + 3 * TM * lda + RED_FLOATS);
  const int start = tile * TM;
  const int count = min(TM, n_rows - start);
  if (threadIdx.x < TM) trow[threadIdx.x] = p.rows[start + ((int)threadIdx.x < count ? threadIdx.x : 0)];
  __syncthreads();
  BRing br;
  if (p.w_evolve0) br.load(p.w_evolve0, p.d);
  stage_rows<false>(XI, lda, p.x0, trow, p.d, count);
  stage_rows<true>(P2, lda, p.x0, trow, p.d, count);
  __syncthreads();
  stamp(1);
  Frag tw;
  const int T = SEQ ? 1 : p.T;  // the per-timestep launch: one timestep, a static index
  for (int t = 0; t < T; ++t) {
    // ---- layer 0: v = x @ W_evolve[0]; rrelu(clamp); exp0; x1 = log0
    {
      Frag v;
      v.zero();
      if (p.w_evolve0) {
        Frag lp;
        lp.zero();
        if (t == 0) mfma_tile_pf(lp, XI, lda, p.w_evolve0, p.d, br, p.d);
        else mfma_tile(lp, XI, lda, p.w_evolve0, p.d, p.d);
#pragma unroll
        for (int j = 0; j < TPW; ++j) v.t[j] += lp.t[j];
      }
      stamp(2);
#pragma unroll
      for (int j = 0; j < TPW; ++j) v.t[j] = leaky4(clamp4(v.t[j], -10.f, 10.f));
      float n2[4];
      rr.sumsq(v, n2);
      exp0_known(v, n2, p.k);
      log0_known(v, n2, p.k);
      frag_to_tile(v, X1, lda, count, p.d);
      __syncthreads();
      stamp(3);
    }
    // ---- layer 1 + timestep: v = x1 @ W_evolve[1] beside tw = clamp(x) @ W_g; skip gate on
    // the cell input; rrelu(clamp); exp0; the timestep epilogue (outputs of timestep t, and
    // the next timestep's operands into XI / P2)
    {
      Frag v;
      v.zero();
      if (SEQ) {
        if (p.w_evolve1) {
          Frag lp;
          lp.zero();
          mfma_tile(lp, X1, lda, p.w_evolve1, p.d, p.d);
#pragma unroll
          for (int j = 0; j < TPW; ++j) v.t[j] += lp.t[j];
        }
        tw.zero();
        mfma_tile(tw, P2, lda, p.step.w_g, p.d, p.d);
      } else if (p.w_evolve1) {
        Frag acc[2];
        acc[0].zero();
        acc[1].zero();
        const float* Ts[2] = {X1, P2};
        const float* Ws[2] = {p.w_evolve1, p.step.w_g};
        mfma_tiles<2, RING>(acc, Ts, Ws, lda, p.d, p.d);
#pragma unroll
        for (int j = 0; j < TPW; ++j) v.t[j] += acc[0].t[j];
        tw = acc[1];
      } else {
        tw.zero();
        mfma_tile(tw, P2, lda, p.step.w_g, p.d, p.d);
      }
      stamp(4);
      if (p.w_skip1) {  // v = g v + (1 - g) x, g = sigmoid(x @ W_skip + b)
        Frag g;
        g.zero();
        mfma_tile(g, XI, lda, p.w_skip1, p.d, p.d);
        Frag pt;
        frag_from_tile(pt, XI, lda, p.d);
        float b[TPW];
        col_load(b, p.b_skip1, p.d);
#pragma unroll
        for (int j = 0; j < TPW; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gt = sigmoidf(g.t[j][r] + b[j]);
            v.t[j][r] = gt * v.t[j][r] + (1.f - gt) * pt.t[j][r];
          }
      }
#pragma unroll
      for (int j = 0; j < TPW; ++j) v.t[j] = leaky4(clamp4(v.t[j], -10.f, 10.f));
      float n2[4];
      rr.sumsq(v, n2);
      exp0_known(v, n2, p.k);
      stamp(5);
      const bool more = t + 1 < T;
      step_epilogue_out(rr, v, n2, P2, lda, trow, count, p.step, tw, p.h_out[t], p.x_out[t], p.r_out[t], nullptr,
                        more ? XI : nullptr, more ? P2 : nullptr);
      __syncthreads();
      stamp(7);
    }
  }
}

// One workgroup per tile (the tile count is on the device: a grid over the host's bound,
// the loop covers a bound beyond 64 workgroups per CU), at the lowest wave priority, so
// concurrent timestep phases' waves (raised priority) win the SIMDs' issue slots.
__global__ __launch_bounds__(NTHR) void k_cold_chain(ChainArgs p) {
  extern __shared__ float lds[];
  __builtin_amdgcn_s_setprio(0);
  const int n_rows = *p.n_rows;
  const int n_tiles = (n_rows + TM - 1) / TM;
  for (int tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    chain_tile<false>(p, tile, n_rows, lds);
    __syncthreads();  // the LDS tiles are reused by the next tile
  }
}

// ------------------------------------------------------------- one timestep, no in-edges
// The rows of one snapshot that receive no message (rows[n_pos:V]) through this timestep:
// layer 0, layer 1, the timestep epilogue in one tile pass (rows held in LDS between them),
// one workgroup per 16-row tile.  Launched on a side stream beside the phase launches, which
// then carry only the in-edge tiles and the relation GRU (regcn_phase_desc.skip_zero_rows):
// the phases keep their registers for the gather paths and these tiles keep theirs.
__global__ __launch_bounds__(NTHR) void k_zero_step(ChainArgs p, int n_rows, int64_t* trace) {
  extern __shared__ float lds[];
  chain_tile<true>(p, blockIdx.x, n_rows, lds, trace);
}

int cold_chain(const ChainArgs& a, int grid_bound, hipStream_t st) {
  if (a.d <= 0 || a.d > MAX_D || (a.d & 3)) return set_error(REGCN_EINVAL, "chain needs d %% 4 == 0, d <= 256 (d=%d)", a.d);
  if (a.T < 1 || a.T > REGCN_MAX_WINDOW) return set_error(REGCN_EINVAL, "chain needs 1..%d timesteps", REGCN_MAX_WINDOW);
  const StepArgs& s = a.step;
  if (!a.rows || !a.n_rows || !a.x0 || !s.w_g || !s.b_g || !s.r_static) return set_error(REGCN_EINVAL, "null pointer");
  if (s.residual && (!s.w_r || !s.b_r)) return set_error(REGCN_EINVAL, "residual radius needs w_r and b_r");
  if (a.w_skip1 && !a.b_skip1) return set_error(REGCN_EINVAL, "skip needs a bias");
  for (int t = 0; t < a.T; ++t)
    if (!a.h_out[t] || !a.x_out[t] || !a.r_out[t]) return set_error(REGCN_EINVAL, "null output of timestep %d", t);
  if (grid_bound <= 0) return 0;
  const size_t lds = (size_t)(3 * TM * tile_lda(a.d) + RED_FLOATS + TM) * 4;
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n_cu = 256;
  }
  // one workgroup per tile up to the bound (the device count may be smaller: the rest exit)
  const int grid = std::max(1, std::min((grid_bound + TM - 1) / TM, 64 * n_cu));
  hipLaunchKernelGGL(k_cold_chain, dim3((unsigned)grid), dim3(NTHR), lds, st, a);
  return check_launch("k_cold_chain");
}

int zero_step(const ChainArgs& a, int n_rows, hipStream_t st) {
  if (a.d <= 0 || a.d > MAX_D || (a.d & 3)) return set_error(REGCN_EINVAL, "zero step needs d %% 4 == 0, d <= 256 (d=%d)", a.d);
  if (a.T != 1) return set_error(REGCN_EINVAL, "zero step runs one timestep (T=%d)", a.T);
  const StepArgs& s = a.step;
  if (n_rows < 0) return set_error(REGCN_EINVAL, "negative row count");
  if (n_rows && (!a.rows || !a.x0 || !s.w_g || !s.b_g || !s.r_static)) return set_error(REGCN_EINVAL, "null pointer");
  if (s.residual && (!s.w_r || !s.b_r)) return set_error(REGCN_EINVAL, "residual radius needs w_r and b_r");
  if (a.w_skip1 && !a.b_skip1) return set_error(REGCN_EINVAL, "skip needs a bias");
  if (!a.h_out[0] || !a.x_out[0] || !a.r_out[0]) return set_error(REGCN_EINVAL, "null output");
  if (!n_rows) return 0;
  const size_t lds = (size_t)(3 * TM * tile_lda(a.d) + RED_FLOATS + TM) * 4;
  hipLaunchKernelGGL(k_zero_step, dim3((unsigned)((n_rows + TM - 1) / TM)), dim3(NTHR), lds, st, a, n_rows, g_trace);
  return check_launch("k_zero_step");
}

}  // namespace regcn
