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
__global__ void k_plan_flags(PlanArgs p) {
  const int t = blockIdx.y;
  const int n = p.n_pos[t];
  const int* rows = p.pos_rows[t];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    atomicOr(p.flags + rows[i], 1 << t);
}

// One workgroup: each thread takes a contiguous run of rows, counts its C / U / Z_t rows,
// a block-wide exclusive scan places the runs, then each thread writes its rows in order.
constexpr int PLAN_THREADS = 1024;
__global__ __launch_bounds__(PLAN_THREADS) void k_plan_lists(PlanArgs p) {
  __shared__ int scan[PLAN_THREADS];
  __shared__ int tot;
  const int tid = threadIdx.x;
  const int per = (p.V + PLAN_THREADS - 1) / PLAN_THREADS;
  const int beg = min(p.V, tid * per), end = min(p.V, beg + per);
  // lists: 0 = C, 1 = U, 2 + t = Z_t
  for (int list = 0; list < 2 + p.T; ++list) {
    int cnt = 0;
    for (int v = beg; v < end; ++v) {
      const unsigned f = (unsigned)p.flags[v];
      cnt += list == 0 ? f == 0 : list == 1 ? f != 0 : (f != 0 && !((f >> (list - 2)) & 1u));
    }
    scan[tid] = cnt;
    __syncthreads();
    for (int off = 1; off < PLAN_THREADS; off <<= 1) {  // inclusive Hillis-Steele scan
      const int add = tid >= off ? scan[tid - off] : 0;
      __syncthreads();
      scan[tid] += add;
      __syncthreads();
    }
    int pos = scan[tid] - cnt;
    if (tid == PLAN_THREADS - 1) tot = scan[tid];
    int* out = list == 0 ? p.c_rows : list == 1 ? p.u_rows : p.z_rows + (int64_t)(list - 2) * p.z_stride;
    for (int v = beg; v < end; ++v) {
      const unsigned f = (unsigned)p.flags[v];
      const bool in = list == 0 ? f == 0 : list == 1 ? f != 0 : (f != 0 && !((f >> (list - 2)) & 1u));
      if (in) out[pos++] = v;
    }
    __syncthreads();
    if (tid == 0) p.counts[list] = tot;
    __syncthreads();
  }
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
  hipMemsetAsync(a.flags, 0, (size_t)a.V * sizeof(int), st);
  if (max_pos) hipLaunchKernelGGL(k_plan_flags, dim3((max_pos + 255) / 256, a.T), dim3(256), 0, st, a);
  hipLaunchKernelGGL(k_plan_lists, dim3(1), dim3(PLAN_THREADS), 0, st, a);
  return check_launch("k_plan_lists");
}

// ----------------------------------------------------------------------------- cold chain
// 16 C rows per workgroup through T timesteps.  LDS tiles: XI = the timestep input x,
// X1 = layer-0 output, P2 = clamp(x) (time-gate operand).  Per timestep exactly the
// per-layer zero-tile path: layer 0 (k_layer<., ., false> zero tile), layer 1 with the
// timestep (k_layer<., ., true> zero tile: loop and gate GEMMs in one k-loop).
__global__ __launch_bounds__(NTHR) void k_cold_chain(ChainArgs p) {
  extern __shared__ float lds[];
  const int lda = tile_lda(p.d);
  float* XI = lds;
  float* X1 = lds + TM * lda;
  float* P2 = lds + 2 * TM * lda;
  RowRed rr{lds + 3 * TM * lda, 0};
  int* trow = reinterpret_cast<int*>(lds + 3 * TM * lda + RED_FLOATS);
  const int n_rows = *p.n_rows;
  const int start = blockIdx.x * TM;
  if (start >= n_rows) return;  // grid sized by the host's bound; the plan's count is on the device
  const int count = min(TM, n_rows - start);
  if (threadIdx.x < TM) trow[threadIdx.x] = p.rows[start + ((int)threadIdx.x < count ? threadIdx.x : 0)];
  __syncthreads();
  BRing br;
  if (p.w_evolve0) br.load(p.w_evolve0, p.d);
  stage_rows<false>(XI, lda, p.x0, trow, p.d, count);
  stage_rows<true>(P2, lda, p.x0, trow, p.d, count);
  __syncthreads();
  for (int t = 0; t < p.T; ++t) {
    // ---- layer 0: v = x @ W_evolve[0]; rrelu(clamp); exp0; x1 = log0
    {
      Frag v;
      v.zero();
      if (p.w_evolve0) {
        Frag lp;
        lp.zero();
        if (t == 0) mfma_tile_pf(lp, XI, lda, p.w_evolve0, p.d, br);
        else mfma_tile(lp, XI, lda, p.w_evolve0, p.d);
#pragma unroll
        for (int j = 0; j < TPW; ++j) v.t[j] += lp.t[j];
      }
#pragma unroll
      for (int j = 0; j < TPW; ++j) v.t[j] = leaky4(clamp4(v.t[j], -10.f, 10.f));
      float n2[4];
      rr.sumsq(v, n2);
      exp0_known(v, n2, p.k);
      log0_known(v, n2, p.k);
      frag_to_tile(v, X1, lda, count, p.d);
      __syncthreads();
    }
    // ---- layer 1 + timestep: v = x1 @ W_evolve[1] beside tw = clamp(x) @ W_g; skip gate on
    // the cell input; rrelu(clamp); exp0; the timestep epilogue (outputs of timestep t, and
    // the next timestep's operands into XI / P2)
    {
      Frag v, tw;
      v.zero();
      if (p.w_evolve1) {
        Frag acc[2];
        acc[0].zero();
        acc[1].zero();
        const float* Ts[2] = {X1, P2};
        const float* Ws[2] = {p.w_evolve1, p.step.w_g};
        mfma_tiles<2, RING>(acc, Ts, Ws, lda, p.d);
#pragma unroll
        for (int j = 0; j < TPW; ++j) v.t[j] += acc[0].t[j];
        tw = acc[1];
      } else {
        tw.zero();
        mfma_tile(tw, P2, lda, p.step.w_g, p.d);
      }
      if (p.w_skip1) {  // v = g v + (1 - g) x, g = sigmoid(x @ W_skip + b)
        Frag g;
        g.zero();
        mfma_tile(g, XI, lda, p.w_skip1, p.d);
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
      StepArgs st = p.step;
      st.h_out = p.h_out[t];
      st.x_out = p.x_out[t];
      st.r_out = p.r_out[t];
      const bool more = t + 1 < p.T;
      step_epilogue(rr, v, n2, P2, lda, trow, count, st, nullptr, &tw, more ? XI : nullptr, more ? P2 : nullptr);
      __syncthreads();
    }
  }
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
  hipLaunchKernelGGL(k_cold_chain, dim3((unsigned)((grid_bound + TM - 1) / TM)), dim3(NTHR), lds, st, a);
  return check_launch("k_cold_chain");
}

}  // namespace regcn
