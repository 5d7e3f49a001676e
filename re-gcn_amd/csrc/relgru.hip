// Relation evolution of one timestep in one launch:
//   x_mean[r] = mean_{e in span(r)} x[e]               (hyperbolic_model.py:802-812)
//   h0'       = GRUCell([emb_rel | x_mean], h0)         (hyperbolic_model.py:813-818)
// torch.nn.GRUCell semantics, gate order (r, z, n):
//   r = s(Wir x + bir + Whr h + bhr), z = s(Wiz x + biz + Whz h + bhz)
//   n = tanh(Win x + bin + r (Whn h + bhn)),  h' = (1 - z) n + z h
//
// Decomposition: a workgroup owns 16 relation rows x ONE 16-column tile of the output;
// its 6 waves split the K = 3d reduction: four take equal ranges of the 2d input columns
// (W_ih: r, z, n_in tiles), two of the d hidden columns (W_hh: r, z, n_h), so each wave
// runs d/8 k-steps of 3 v_mfma_f32_16x16x4_f32; the partials are summed through LDS and the
// gate epilogue runs on the sum.  Grid = ceil(R2/16) x ceil(d/16): ~380 workgroups at
// R2 = 460, d = 200, each with a 25-step MFMA chain per wave.  The first 16 k-steps of B
// fragments are issued before the A rows are staged (they do not depend on them).
// The A rows [emb_rel | x_mean | h0] are staged once per workgroup; x_mean is either
// gathered in-kernel from the r_to_e spans (short spans, the per-snapshot case) or read
// from a precomputed buffer (regcn_segment_mean_f32, long spans).
//
// Weights are packed per 16-column tile and 16-deep k-block (regcn_pack_linear_f32):
//   Wp[g][b][jt][lane][e] = W[g*d + 16 jt + lane%16][16 b + 4 (lane/16) + e]
// (W row-major out x in, as nn.Linear / nn.GRUCell store it): one dwordx4 per lane, gate
// and k-block.
#include "common.h"
#include "gather.h"
#include "regcn_internal.h"
#include "rowtile.h"
#include "gru_parts.h"

namespace regcn {

// K split: W_ih (2d inputs) over IH_WAVES waves, W_hh (d) over HH_WAVES, so no wave
// straddles the two packs and the waves' MFMA chains are about equally long.
constexpr int IH_WAVES = 4, HH_WAVES = 2;
constexpr int GW = IH_WAVES + HH_WAVES;  // waves per workgroup (waves 0-3 finish C registers 0-3)
constexpr int GTHR = 64 * GW;

// A tile row stride: >= 3d + 16 (a zero tail for the last k-block of W_hh) and = 8 (mod 16),
// which makes the ds_read_b128 fragment reads below bank-conflict free.
__host__ __device__ inline int gru_lda(int d) {
  const int n = 3 * d + 16;
  return n + ((8 - n % 16) + 16) % 16;
}

// k-block order: MFMA sub-step e of k-block b reads k = 16 b + 4 (lane >> 4) + e, so each
// lane's A (LDS) and B (packed) operands for a whole block are one contiguous float4.
__global__ __launch_bounds__(GTHR) void k_rel_gru(RelGruArgs p) {
  extern __shared__ float lds[];
  const int d = p.d, lda = gru_lda(d);
  float* A = lds;                      // TM x lda: [emb_rel | x_mean | h0 | 0]
  f4* red = reinterpret_cast<f4*>(lds + TM * lda);  // [GW][4 acc][64 lanes]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r0 = blockIdx.x * TM, jt = blockIdx.y;
  const int n_valid = min(TM, p.R2 - r0);
  const int col = lane * 4;
  auto stamp = [&](int k) {  // profiling (regcn_set_trace)
    if (p.trace && threadIdx.x == 0)
      p.trace[(blockIdx.y * gridDim.x + blockIdx.x) * 16 + k] = (int64_t)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  // ---- this wave's k-blocks and the first GR4 blocks of B fragments (3 gates), issued
  // before the staging below: they do not depend on it.  Packs: Wp[g][b][jt][lane][e].
  const int B_in = (2 * d + 15) >> 4, B_h = (d + 15) >> 4;
  const int NT = (d + 15) >> 4;
  const bool hh = w >= IH_WAVES;
  const int wi = hh ? w - IH_WAVES : w, nw = hh ? HH_WAVES : IH_WAVES, Bg = hh ? B_h : B_in;
  const int beg = (Bg * wi) / nw, end = (Bg * (wi + 1)) / nw;
  const f4* bb = reinterpret_cast<const f4*>(hh ? p.w_hh : p.w_ih) + (int64_t)jt * 64 + lane;
  const int64_t gs = (int64_t)Bg * NT * 64;  // gate stride (float4 units)
  auto clamp_blk = [&](int b) { return max(min(b, end - 1), 0); };  // unconditional loads
  f4 br[GR4], bz[GR4], bn[GR4], ra[GR4];
#pragma unroll
  for (int i = 0; i < GR4; ++i) {
    const f4* b = bb + (int64_t)clamp_blk(beg + i) * NT * 64;
    br[i] = b[0];
    bz[i] = b[gs];
    bn[i] = b[2 * gs];
  }

  // ---- stage the 16 A rows (wave w: rows w, w + GW, ...) and zero the tail columns
  for (int t = threadIdx.x; t < TM * 16; t += GTHR) A[(t >> 4) * lda + 3 * d + (t & 15)] = 0.f;
  for (int i = w; i < TM; i += GW) {
    const int row = r0 + min(i, n_valid - 1);
    f4 e = load4(p.emb_rel + (int64_t)row * d, col, d);
    f4 h = load4(p.h_prev + (int64_t)row * d, col, d);
    f4 m = {0.f, 0.f, 0.f, 0.f};
    if (p.x_mean) {
      m = load4(p.x_mean + (int64_t)row * d, col, d);
    } else {
      const int beg = p.rel_start[row];
      const float cntf = p.rel_count[row];
      const int cnt = (int)cntf;
      f4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int e0 = 0; e0 < cnt; e0 += 64) {
        const int n = min(64, cnt - e0);
        const int my = lane < n ? p.rel_idx[beg + e0 + lane] : 0;
        int j = 0;
        for (; j + 4 <= n; j += 4) {
          f4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = load4(p.x + (int64_t)rl(my, j + u) * d, col, d);
#pragma unroll
          for (int u = 0; u < 4; ++u) acc += v[u];
        }
        for (; j < n; ++j) acc += load4(p.x + (int64_t)rl(my, j) * d, col, d);
      }
      if (cnt > 0) m = acc / cntf;
    }
    if (i >= n_valid) {
      e = f4{0.f, 0.f, 0.f, 0.f};
      m = e;
      h = e;
    }
    float* dst = A + i * lda;
    if (col < d) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dst[col + q] = e[q];
        dst[d + col + q] = m[q];
        dst[2 * d + col + q] = h[q];
      }
    }
  }
  __syncthreads();
  stamp(1);

  // ---- MFMA over k-blocks [beg, end): r, z and the n gate's input (W_ih waves) or hidden
  // (W_hh waves) part; A and B operands ride in rings GR4 blocks ahead of their MFMAs.
  f4 ar = {0.f, 0.f, 0.f, 0.f}, az = ar, an = ar;
  const float* arow = A + (lane & 15) * lda + 4 * (lane >> 4) + (hh ? 2 * d : 0);
#pragma unroll
  for (int i = 0; i < GR4; ++i) ra[i] = *reinterpret_cast<const f4*>(arow + 16 * clamp_blk(beg + i));
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
  const f4 z4 = {0.f, 0.f, 0.f, 0.f};
  const f4 ai = hh ? z4 : an, ah = hh ? an : z4;
  red[(w * 4 + 0) * 64 + lane] = ar;
  red[(w * 4 + 1) * 64 + lane] = az;
  red[(w * 4 + 2) * 64 + lane] = ai;
  red[(w * 4 + 3) * 64 + lane] = ah;
  stamp(2);
  __syncthreads();
  stamp(3);

  // ---- wave w < 4 finishes C register q = w: row 4 (lane >> 4) + w, column 16 jt + lane % 16
  if (w >= 4) {
    stamp(4);
    return;
  }
  const int q = w;
  float v[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    float t = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < GW; ++w2) t += red[(w2 * 4 + a) * 64 + lane][q];
    v[a] = t;
  }
  const int i = 4 * (lane >> 4) + q;
  const int n = 16 * jt + (lane & 15);
  if (i < n_valid && n < d) {
    const float r = sigmoidf(v[0] + p.b_ih[n] + p.b_hh[n]);
    const float z = sigmoidf(v[1] + p.b_ih[d + n] + p.b_hh[d + n]);
    const float nn = ftanh(v[2] + p.b_ih[2 * d + n] + r * (v[3] + p.b_hh[2 * d + n]));
    const float h = A[i * lda + 2 * d + n];
    p.h_out[(int64_t)(r0 + i) * d + n] = (1.f - z) * nn + z * h;
  }
  stamp(4);
}

// ============================================================ two-phase relation GRU (gru_parts.h)
__global__ __launch_bounds__(64 * PRE_WAVES) void k_gru_pre(RelGru2Args p) {
  extern __shared__ float lds[];
  gru_pre_block(p, blockIdx.x, blockIdx.y, lds);
}

__global__ __launch_bounds__(64 * X_WAVES) void k_gru_x(RelGru2Args p) {
  extern __shared__ float lds[];
  gru_x_block(p, blockIdx.x, blockIdx.y, lds);
}

int rel_gru_pre(const RelGru2Args& a, hipStream_t st) {
  if (a.d <= 0 || a.d > MAX_D || (a.d & 3)) return set_error(REGCN_EINVAL, "relation GRU needs d %% 4 == 0, d <= 256");
  if (!a.emb_rel || !a.h_prev || !a.w_ih_e || !a.w_hh || !a.b_ih || !a.b_hh || !a.pre)
    return set_error(REGCN_EINVAL, "null pointer");
  if (a.R2 == 0) return 0;
  dim3 grid((unsigned)((a.R2 + TM - 1) / TM), (unsigned)(gru_dpad(a.d) / 16));
  const size_t lds = gru_pre_lds_bytes(a.d);
  hipLaunchKernelGGL(k_gru_pre, grid, dim3(64 * PRE_WAVES), lds, st, a);
  return check_launch("k_gru_pre");
}

int rel_gru_x(const RelGru2Args& a, hipStream_t st) {
  if (a.d <= 0 || a.d > MAX_D || (a.d & 3)) return set_error(REGCN_EINVAL, "relation GRU needs d %% 4 == 0, d <= 256");
  if (!a.h_prev || !a.w_ih_x || !a.pre || !a.h_out) return set_error(REGCN_EINVAL, "null pointer");
  if (!a.x_mean && (!a.x || !a.rel_start || !a.rel_count))
    return set_error(REGCN_EINVAL, "relation GRU needs x_mean or the r_to_e spans");
  if (a.R2 == 0) return 0;
  dim3 grid((unsigned)((a.R2 + TM - 1) / TM), (unsigned)(gru_dpad(a.d) / 16));
  const size_t lds = gru_x_lds_bytes(a.d);
  hipLaunchKernelGGL(k_gru_x, grid, dim3(64 * X_WAVES), lds, st, a);
  return check_launch("k_gru_x");
}

// Wp[g][b][jt][lane][e] = W[g*n_out + 16 jt + lane%16][16 b + 4 (lane/16) + e]  (zero padded)
__global__ void k_pack_linear(const float* __restrict__ W, int n_gates, int n_out, int n_in, float* __restrict__ Wp) {
  const int NB = (n_in + 15) >> 4, NT = (n_out + 15) >> 4;
  const int per_gate = NB * NT * 64 * 4;
  const int total = n_gates * per_gate;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int g = idx / per_gate, rem = idx - g * per_gate;
    const int e = rem & 3, lane = (rem >> 2) & 63, t = rem >> 8;
    const int jt = t % NT, b = t / NT;
    const int o = 16 * jt + (lane & 15), k = 16 * b + 4 * (lane >> 4) + e;
    Wp[idx] = (o < n_out && k < n_in) ? W[((int64_t)g * n_out + o) * n_in + k] : 0.f;
  }
}

size_t packed_linear_floats(int n_gates, int n_out, int n_in) {
  return (size_t)n_gates * ((n_in + 15) / 16) * ((n_out + 15) / 16) * 64 * 4;
}

int pack_linear(const float* W, int n_gates, int n_out, int n_in, float* Wp, hipStream_t st) {
  if (!W || !Wp) return set_error(REGCN_EINVAL, "null pointer");
  if (n_gates <= 0 || n_out <= 0 || n_in <= 0) return set_error(REGCN_EINVAL, "bad pack_linear shape");
  const size_t total = packed_linear_floats(n_gates, n_out, n_in);
  const unsigned blocks = (unsigned)std::min<size_t>((total + 255) / 256, 65535);
  hipLaunchKernelGGL(k_pack_linear, dim3(blocks), dim3(256), 0, st, W, n_gates, n_out, n_in, Wp);
  return check_launch("k_pack_linear");
}

int rel_gru(const RelGruArgs& a, hipStream_t st) {
  if (a.d <= 0 || a.d > MAX_D || (a.d & 3)) return set_error(REGCN_EINVAL, "relation GRU needs d %% 4 == 0, d <= 256");
  if (!a.emb_rel || !a.h_prev || !a.w_ih || !a.w_hh || !a.b_ih || !a.b_hh || !a.h_out)
    return set_error(REGCN_EINVAL, "null pointer");
  if (!a.x_mean && (!a.x || !a.rel_start || !a.rel_count))
    return set_error(REGCN_EINVAL, "relation GRU needs x_mean or the r_to_e spans");
  if (a.R2 == 0) return 0;
  RelGruArgs b = a;
  b.trace = g_trace;
  dim3 grid((unsigned)((a.R2 + TM - 1) / TM), (unsigned)((a.d + 15) / 16));
  const size_t lds = (size_t)TM * gru_lda(a.d) * 4 + (size_t)GW * 4 * 64 * 16;
  hipLaunchKernelGGL(k_rel_gru, grid, dim3(GTHR), lds, st, b);
  return check_launch("k_rel_gru");
}

}  // namespace regcn
