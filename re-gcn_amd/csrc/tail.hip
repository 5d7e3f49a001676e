// Fused elementwise tail of a training-path layer and of the time gate,
// forward and backward, replacing ~10 forward and ~15 backward torch elementwise launches
// on V x d tensors per use (the replayed training step is bound by such launches):
//
//   a = clamp(agg, -10, 10)                     [CLAMP_IN]   hyperbolic_layers.py:296 / :672
//   a = a + (pos[v] ? lx : ex)                  [lx != 0]    self / evolve loop :273-280
//                                               (lx, ex rows loop_ld apart: the two halves
//                                                of one x [W_loop | W_evolve] product)
//   g = sigmoid(z + bias); a = g a + (1 - g) p  [z != 0]     skip gate :315-318, time gate
//                                                            hyperbolic_model.py:852-860
//   a = clamp(a, -10, 10)                       [CLAMP_OUT]  :319
//   a = a > 0 ? a : slope a                     [LEAKY]      rrelu in eval form :320
//
// The forward keeps torch's fp32 op order with no contraction (__fmul_rn / __fadd_rn); it
// differs from the op-by-op composition only through sigmoid's expf (1 / (1 + expf(-x)) as
// torch's kernel, ocml expf: last-ulp differences).  The backward recomputes the forward from its inputs and
// applies torch's derivative conventions (clamp passes the gradient on the closed interval,
// leaky_relu uses x > 0, sigmoid' = (1 - y) y); the bias gradient (a column sum of dz) is
// left to the caller.  Memory-bound: float4 per lane, one pass.
#include "regcn_internal.h"
#include "common.h"

namespace regcn {
namespace {

constexpr int TAIL_THR = 256;

__device__ __forceinline__ float clamp10(float x) { return clampf(x, -10.f, 10.f); }
__device__ __forceinline__ bool in10(float x) { return x >= -10.f && x <= 10.f; }

template <bool BWD>
__global__ __launch_bounds__(TAIL_THR) void k_tail(TailArgs t) {
  const int64_t n4 = t.V * t.d / 4;
  for (int64_t i4 = (int64_t)blockIdx.x * TAIL_THR + threadIdx.x; i4 < n4; i4 += (int64_t)gridDim.x * TAIL_THR) {
    const int64_t e0 = i4 * 4;
    const int64_t v = e0 / t.d;
    const int j0 = (int)(e0 - v * t.d);
    const f4 agg = *reinterpret_cast<const f4*>(t.agg + e0);
    f4 lx = {0.f, 0.f, 0.f, 0.f}, z = lx, p = lx, b = lx, gy = lx;
    bool pos = false;
    if (t.lx) {
      pos = t.pos[v] != 0;
      lx = *reinterpret_cast<const f4*>((pos ? t.lx : t.ex) + v * t.loop_ld + j0);
    }
    if (t.z) {
      z = *reinterpret_cast<const f4*>(t.z + e0);
      p = *reinterpret_cast<const f4*>(t.p + e0);
      if (t.bias) b = *reinterpret_cast<const f4*>(t.bias + j0);
    }
    if (BWD) gy = *reinterpret_cast<const f4*>(t.gy + e0);
    f4 out, dagg, dl, dz, dp;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float a = (t.flags & REGCN_TAIL_CLAMP_IN) ? clamp10(agg[e]) : agg[e];
      if (t.lx) a = __fadd_rn(a, lx[e]);
      const float s1 = a;  // gate input
      float gt = 0.f, om = 0.f;
      if (t.z) {
        gt = 1.f / (1.f + expf(-__fadd_rn(z[e], b[e])));
        om = __fsub_rn(1.f, gt);
        a = __fadd_rn(__fmul_rn(gt, a), __fmul_rn(om, p[e]));
      }
      const float s2 = a;  // clamp_out input
      if (t.flags & REGCN_TAIL_CLAMP_OUT) a = clamp10(a);
      const float s3 = a;  // leaky input
      if (t.flags & REGCN_TAIL_LEAKY) a = a > 0.f ? a : __fmul_rn(a, t.slope);
      out[e] = a;
      if (BWD) {
        float g = gy[e];
        if (t.flags & REGCN_TAIL_LEAKY) g = s3 > 0.f ? g : __fmul_rn(g, t.slope);
        if ((t.flags & REGCN_TAIL_CLAMP_OUT) && !in10(s2)) g = 0.f;
        if (t.z) {
          const float dgt = __fadd_rn(__fmul_rn(g, s1), -__fmul_rn(g, p[e]));
          dz[e] = __fmul_rn(__fmul_rn(dgt, om), gt);
          dp[e] = __fmul_rn(g, om);
          g = __fmul_rn(g, gt);
        }
        dl[e] = g;
        dagg[e] = ((t.flags & REGCN_TAIL_CLAMP_IN) && !in10(agg[e])) ? 0.f : g;
      }
    }
    if (!BWD) {
      *reinterpret_cast<f4*>(t.out + e0) = out;
    } else {
      if (t.dagg) *reinterpret_cast<f4*>(t.dagg + e0) = dagg;
      if (t.lx) {
        const f4 zero = {0.f, 0.f, 0.f, 0.f};
        if (t.dlx) *reinterpret_cast<f4*>(t.dlx + v * t.loop_ld + j0) = pos ? dl : zero;
        if (t.dex) *reinterpret_cast<f4*>(t.dex + v * t.loop_ld + j0) = pos ? zero : dl;
      }
      if (t.z) {
        if (t.dz) *reinterpret_cast<f4*>(t.dz + e0) = dz;
        if (t.dp) *reinterpret_cast<f4*>(t.dp + e0) = dp;
      }
    }
  }
}

// Lorentz centroid -> Poincare ball of a Lorentz layer's message sums (S0, Sv), one wave
// per row (lane l: columns 4l..4l+3, d <= 256), forward and backward:
//   ip = -S0^2 + |Sv|^2, sc = sqrt(max(-c ip, eps)), c0 = S0 / sc,
//   y = (Sv / sc) / max(1 + sqrt(c) c0, eps)          (hyperbolic_layers.py:613-625, :669)
// The backward follows torch's conventions for the clamps (gradient on x >= eps).
template <bool BWD>
__global__ __launch_bounds__(256) void k_centroid(const float* __restrict__ S0, const float* __restrict__ Sv,
                                                  int64_t V, int d, float c, float sqc,
                                                  const float* __restrict__ gy, float* __restrict__ y,
                                                  float* __restrict__ dS0, float* __restrict__ dSv) {
  const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (v >= V) return;
  const int col = 4 * (threadIdx.x & 63);
  const float s0 = S0[v];
  const f4 sv = load4(Sv + v * d, col, d);
  const float ip = -s0 * s0 + wave_sum(dot4(sv, sv));
  const float inner = -ip * c;
  const float sc = sqrtf(fmaxf(inner, REGCN_EPS));
  const float c0 = s0 / sc;
  const float dn = 1.f + c0 * sqc;
  const float den = fmaxf(dn, REGCN_EPS);
  const f4 u = sv / sc;
  const f4 yy = u / den;
  if (!BWD) {
    store4(y + v * d, col, d, yy);
    return;
  }
  const f4 g = load4(gy + v * d, col, d);
  const float dden = -wave_sum(dot4(g, yy)) / den;
  const float dc0 = dn >= REGCN_EPS ? dden * sqc : 0.f;
  const f4 du = g / den;
  const float dsc = -dc0 * s0 / (sc * sc) - wave_sum(dot4(du, sv)) / (sc * sc);
  const float dinner = inner >= REGCN_EPS ? dsc * 0.5f / sc : 0.f;
  const float dip = -c * dinner;
  if ((threadIdx.x & 63) == 0) dS0[v] = dc0 / sc + dip * (-2.f * s0);
  store4(dSv + v * d, col, d, du / sc + (2.f * dip) * sv);
}

// Givens rotation (REF: reflection) of interleaved pairs (hyperbolic_decoder.py:1032-1051,
// :1392-1401): for pair i, (x1, x2) = (x[2i], x[2i+1]), t = ang[i]:
//   rotation   out = (cos x1 - sin x2, sin x1 + cos x2)
//   reflection out = (cos x1 + sin x2, sin x1 - cos x2)      (torch's op order, no contraction)
// backward: rotation   dx = (cos g1 + sin g2, cos g2 - sin g1),
//                      dt = g2 (cos x1 - sin x2) - g1 (sin x1 + cos x2);
//           reflection dx = (cos g1 + sin g2, sin g1 - cos g2),
//                      dt = g1 (cos x2 - sin x1) + g2 (cos x1 + sin x2).
template <bool BWD, bool REF>
__global__ __launch_bounds__(256) void k_givens(const float* __restrict__ x, const float* __restrict__ ang,
                                                int64_t n_pairs, const float* __restrict__ gy,
                                                float* __restrict__ out, float* __restrict__ dx,
                                                float* __restrict__ dang) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_pairs; i += (int64_t)gridDim.x * 256) {
    const f2 xv = *reinterpret_cast<const f2*>(x + 2 * i);
    const float t = ang[i];
    const float co = cosf(t), si = sinf(t);
    if (!BWD) {
      f2 o;
      if (REF) {
        o.x = __fadd_rn(__fmul_rn(co, xv.x), __fmul_rn(si, xv.y));
        o.y = __fsub_rn(__fmul_rn(si, xv.x), __fmul_rn(co, xv.y));
      } else {
        o.x = __fsub_rn(__fmul_rn(co, xv.x), __fmul_rn(si, xv.y));
        o.y = __fadd_rn(__fmul_rn(si, xv.x), __fmul_rn(co, xv.y));
      }
      *reinterpret_cast<f2*>(out + 2 * i) = o;
    } else {
      const f2 g = *reinterpret_cast<const f2*>(gy + 2 * i);
      f2 d;
      d.x = co * g.x + si * g.y;
      if (REF) {
        d.y = si * g.x - co * g.y;
        dang[i] = g.x * (co * xv.y - si * xv.x) + g.y * (co * xv.x + si * xv.y);
      } else {
        d.y = co * g.y - si * g.x;
        dang[i] = g.y * (co * xv.x - si * xv.y) - g.x * (si * xv.x + co * xv.y);
      }
      *reinterpret_cast<f2*>(dx + 2 * i) = d;
    }
  }
}

}  // namespace

int tail(const TailArgs& t, int backward, hipStream_t st) {
  if (t.V < 0 || t.d <= 0 || (t.d & 3)) return set_error(REGCN_EINVAL, "tail needs d %% 4 == 0 (d=%d)", t.d);
  if (!t.agg || (!backward && !t.out) || (backward && !t.gy)) return set_error(REGCN_EINVAL, "null pointer");
  if (t.lx && (!t.ex || !t.pos)) return set_error(REGCN_EINVAL, "tail: the self loop needs lx, ex and pos");
  if (t.lx && (t.loop_ld < t.d || (t.loop_ld & 3))) return set_error(REGCN_EINVAL, "tail needs loop_ld >= d, loop_ld %% 4 == 0");
  if (t.z && !t.p) return set_error(REGCN_EINVAL, "tail: the gate needs z and p");
  const uintptr_t al = (uintptr_t)t.agg | (uintptr_t)t.lx | (uintptr_t)t.ex | (uintptr_t)t.z | (uintptr_t)t.p |
                       (uintptr_t)t.bias | (uintptr_t)t.gy | (uintptr_t)t.out | (uintptr_t)t.dagg | (uintptr_t)t.dlx |
                       (uintptr_t)t.dex | (uintptr_t)t.dz | (uintptr_t)t.dp;
  if (al & 15) return set_error(REGCN_EINVAL, "tail needs 16-byte aligned rows");
  const int64_t n4 = t.V * t.d / 4;
  if (n4 == 0) return 0;
  const unsigned grid = (unsigned)std::min<int64_t>((n4 + TAIL_THR - 1) / TAIL_THR, 8192);
  if (backward) hipLaunchKernelGGL(k_tail<true>, dim3(grid), dim3(TAIL_THR), 0, st, t);
  else hipLaunchKernelGGL(k_tail<false>, dim3(grid), dim3(TAIL_THR), 0, st, t);
  return check_launch("k_tail");
}

int centroid(const float* S0, const float* Sv, int64_t V, int d, float c, float sqc, const float* gy, float* y,
             float* dS0, float* dSv, hipStream_t st) {
  if (V < 0 || d <= 0 || d > 256 || (d & 3)) return set_error(REGCN_EINVAL, "centroid needs d %% 4 == 0, d <= 256");
  if (!S0 || !Sv || (gy ? (!dS0 || !dSv) : !y)) return set_error(REGCN_EINVAL, "null pointer");
  if (V == 0) return 0;
  const dim3 grid((unsigned)((V + 3) / 4));
  if (gy) hipLaunchKernelGGL(k_centroid<true>, grid, dim3(256), 0, st, S0, Sv, V, d, c, sqc, gy, y, dS0, dSv);
  else hipLaunchKernelGGL(k_centroid<false>, grid, dim3(256), 0, st, S0, Sv, V, d, c, sqc, gy, y, dS0, dSv);
  return check_launch("k_centroid");
}

int givens(const float* x, const float* ang, int64_t n_pairs, int reflect, const float* gy, float* out, float* dx, float* dang,
           hipStream_t st) {
  if (n_pairs < 0 || !x || !ang || (gy ? (!dx || !dang) : !out)) return set_error(REGCN_EINVAL, "null pointer");
  if (((uintptr_t)x | (uintptr_t)gy | (uintptr_t)out | (uintptr_t)dx) & 7)
    return set_error(REGCN_EINVAL, "givens needs 8-byte aligned pairs");
  if (n_pairs == 0) return 0;
  const unsigned grid = (unsigned)std::min<int64_t>((n_pairs + 255) / 256, 8192);
  if (gy && reflect) hipLaunchKernelGGL((k_givens<true, true>), dim3(grid), dim3(256), 0, st, x, ang, n_pairs, gy, out, dx, dang);
  else if (gy) hipLaunchKernelGGL((k_givens<true, false>), dim3(grid), dim3(256), 0, st, x, ang, n_pairs, gy, out, dx, dang);
  else if (reflect) hipLaunchKernelGGL((k_givens<false, true>), dim3(grid), dim3(256), 0, st, x, ang, n_pairs, gy, out, dx, dang);
  else hipLaunchKernelGGL((k_givens<false, false>), dim3(grid), dim3(256), 0, st, x, ang, n_pairs, gy, out, dx, dang);
  return check_launch("k_givens");
}

}  // namespace regcn
