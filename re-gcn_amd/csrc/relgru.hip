// Relation evolution of one timestep in one launch:
//   x_mean[r] = mean_{e in span(r)} x[e]               (hyperbolic_model.py:802-812)
//   h0'       = GRUCell([emb_rel | x_mean], h0)         (hyperbolic_model.py:813-818)
// torch.nn.GRUCell semantics, gate order (r, z, n):
//   r = s(Wir x + bir + Whr h + bhr), z = s(Wiz x + biz + Whz h + bhz)
//   n = tanh(Win x + bin + r (Whn h + bhn)),  h' = (1 - z) n + z h
//
// Decomposition: a workgroup owns 16 relation rows x ONE 16-column tile of the output;
// its 4 waves split the K = 3d reduction (2d input columns then d hidden columns) into
// contiguous k-step ranges and each accumulates r, z, n_in, n_h tiles
// (v_mfma_f32_16x16x4_f32); the 4 partials are summed through LDS and the gate epilogue
// runs on the sum.  Grid = ceil(R2/16) x ceil(d/16): ~380 workgroups at R2 = 460, d = 200,
// each with a ~40-step MFMA chain per wave, instead of one long chain per output tile.
// The A rows [emb_rel | x_mean | h0] are staged once per workgroup; x_mean is either
// gathered in-kernel from the r_to_e spans (short spans, the per-snapshot case) or read
// from a precomputed buffer (regcn_segment_mean_f32, long spans).
//
// Weights are packed per 16-column tile (regcn_pack_linear_f32):
//   Wp[g][s][jt][lane] = W[g*d + 16 jt + lane%16][4 s + lane/16]
// (W row-major out x in, as nn.Linear / nn.GRUCell store it).
#include "common.h"
#include "gather.h"
#include "regcn_internal.h"
#include "rowtile.h"

namespace regcn {

constexpr int GW = 4;  // waves per workgroup (the finish maps C register q to wave q)
constexpr int GTHR = 64 * GW;

__global__ __launch_bounds__(GTHR) void k_rel_gru(RelGruArgs p) {
  extern __shared__ float lds[];
  const int d = p.d, K = 3 * d, lda = tile_lda(K);
  float* A = lds;                      // TM x lda: [emb_rel | x_mean | h0]
  f4* red = reinterpret_cast<f4*>(lds + TM * lda);  // [GW][4 acc][64 lanes]
  const int lane = threadIdx.x & 63, w = wave_id();
  const int r0 = blockIdx.x * TM, jt = blockIdx.y;
  const int n_valid = min(TM, p.R2 - r0);
  const int col = lane * 4;

  // ---- stage the 16 A rows (wave w: rows w, w + 4, ...)
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

  // ---- K split over the waves: steps [0, S_in) read W_ih, [S_in, S_in + S_h) W_hh
  const int S_in = (2 * d) >> 2, S_h = d >> 2, S = S_in + S_h;
  const int NT = (d + 15) >> 4;
  const int sb = (S * w) / GW, se = (S * (w + 1)) / GW;
  f4 ar = {0.f, 0.f, 0.f, 0.f}, az = ar, ai = ar, ah = ar;
  const float* arow = A + (lane & 15) * lda + (lane >> 4);
  const int gs_in = S_in * NT * 64, gs_h = S_h * NT * 64;  // per-gate stride of the packs
  // B (3 gates) and A operands ride in rings GR k-steps ahead of their MFMAs; every load
  // is unconditional (clamped step) so the waits are counted, not drained.
  constexpr int GR = 8;
  // steps [beg, end) of one weight (W: packed base, off: its first global step, gs: gate
  // stride); the n gate accumulates into accn (n_in for W_ih, n_h for W_hh)
  auto segment = [&](int beg, int end, const float* W, int off, int gs, f4& accn) {
    if (beg >= end) return;
    const float* bb = W + (int64_t)jt * 64 + lane;
    float ra[GR], rr_[GR], rz[GR], rn[GR];
#pragma unroll
    for (int i = 0; i < GR; ++i) {
      const int st = min(beg + i, end - 1);
      const float* b = bb + (int64_t)(st - off) * NT * 64;
      rr_[i] = b[0];
      rz[i] = b[gs];
      rn[i] = b[2 * gs];
      ra[i] = arow[4 * st];
    }
    for (int s0 = beg; s0 < end; s0 += GR) {
#pragma unroll
      for (int i = 0; i < GR; ++i) {
        if (s0 + i < end) {  // wave-uniform
          ar = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[i], rr_[i], ar, 0, 0, 0);
          az = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[i], rz[i], az, 0, 0, 0);
          accn = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[i], rn[i], accn, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        const int st = min(s0 + i + GR, end - 1);
        const float* b = bb + (int64_t)(st - off) * NT * 64;
        rr_[i] = b[0];
        rz[i] = b[gs];
        rn[i] = b[2 * gs];
        ra[i] = arow[4 * st];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  segment(sb, min(se, S_in), p.w_ih, 0, gs_in, ai);
  segment(max(sb, S_in), se, p.w_hh, S_in, gs_h, ah);
  red[(w * 4 + 0) * 64 + lane] = ar;
  red[(w * 4 + 1) * 64 + lane] = az;
  red[(w * 4 + 2) * 64 + lane] = ai;
  red[(w * 4 + 3) * 64 + lane] = ah;
  __syncthreads();

  // ---- wave w finishes C register q = w: row 4 (lane >> 4) + w, column 16 jt + lane % 16
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
    const float nn = tanhf(v[2] + p.b_ih[2 * d + n] + r * (v[3] + p.b_hh[2 * d + n]));
    const float h = A[i * lda + 2 * d + n];
    p.h_out[(int64_t)(r0 + i) * d + n] = (1.f - z) * nn + z * h;
  }
}

// Wp[g][s][jt][lane] = W[g*n_out + 16 jt + lane%16][4 s + lane/16]  (zero padded)
__global__ void k_pack_linear(const float* __restrict__ W, int n_gates, int n_out, int n_in, float* __restrict__ Wp) {
  const int S = (n_in + 3) >> 2, NT = (n_out + 15) >> 4;
  const int per_gate = S * NT * 64;
  const int total = n_gates * per_gate;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int g = idx / per_gate, rem = idx - g * per_gate;
    const int lane = rem & 63, t = rem >> 6;
    const int jt = t % NT, s = t / NT;
    const int o = 16 * jt + (lane & 15), k = 4 * s + (lane >> 4);
    Wp[idx] = (o < n_out && k < n_in) ? W[((int64_t)g * n_out + o) * n_in + k] : 0.f;
  }
}

size_t packed_linear_floats(int n_gates, int n_out, int n_in) {
  return (size_t)n_gates * ((n_in + 3) / 4) * ((n_out + 15) / 16) * 64;
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
  dim3 grid((unsigned)((a.R2 + TM - 1) / TM), (unsigned)((a.d + 15) / 16));
  const size_t lds = (size_t)TM * tile_lda(3 * a.d) * 4 + (size_t)GW * 4 * 64 * 16;
  hipLaunchKernelGGL(k_rel_gru, grid, dim3(GTHR), lds, st, a);
  return check_launch("k_rel_gru");
}

}  // namespace regcn
