// Backward kernels of the training path.
//
// Gradients follow torch autograd through the reference's op sequence
// (hyperbolic_src/hyperbolic_ops.py, hyperbolic_layers.py), including its clamp
// subgradients: a clamped quantity passes gradient only inside [lo, hi] (inclusive, as
// torch.clamp's backward), a norm clamped to eps passes none below it.
//
//  * Row maps.  log0, exp0, project, apply_radius and get_radius are radial: y = s(|x|) x,
//    so dx = s g + k (x.g) x with k = s'(|x|) / |x|; a chain of radial maps on one row stays
//    of that form.  mobius_add's gradient is a combination of (g, x, y) whose coefficients
//    need five row dot products.  One wave per row, lane l owns columns [4l, 4l + 4).
//  * Union aggregation (agg[v] = norm[v] sum_e w_e (x[src] + rel[type]),
//    w_e = exp(-gamma |r_src - r_dst|)): three passes over the snapshot's edge lists, each
//    a deterministic segment reduction (no atomics) -- destination rows (per-edge weight,
//    radius terms of the destination), source rows (dx, radius terms of the source: the
//    src-sorted transpose), relation types (drel: the type-sorted transpose).
//  * Lorentz messages (S[v] = sum_e to_lorentz(exp0(blockdiag(W_type) x_src + rel_type))):
//    the raw sums forward, then per edge dm = dL/dm recomputed from (x_src, W, rel, dS[dst])
//    in the source pass (dx = W^T dm) and the type pass (drel = sum dm, dW = sum x dm^T).
#include "common.h"
#include "gather.h"
#include "regcn_internal.h"

namespace regcn {
namespace {

// y = s x, dx = s g + kk (x.g) x
struct Rad {
  float s, kk;
};

// project_to_ball on a row of norm n (hyperbolic_ops.py:37-74).
__device__ __forceinline__ Rad rad_project(float n, const Curv& k) {
  const float nc = fmaxf(n, REGCN_EPS);
  const float s = fminf(nc, k.mx) / nc;
  const float ds = nc > k.mx ? -k.mx / (nc * nc) : 0.f;
  return Rad{s, n >= REGCN_EPS ? ds / n : 0.f};
}

// log_map_zero (hyperbolic_ops.py:97-116): atanh(min(sc n, 1 - eps)) / (sc n).
__device__ __forceinline__ Rad rad_log0(float n, const Curv& k) {
  const float nc = fmaxf(n, REGCN_EPS);
  const float z = k.sqrt_c * nc;
  const float zc = fminf(z, k.atanh_mx);
  const float at = atanhf(zc);
  const float s = at / z;
  const float dzc = z <= k.atanh_mx ? k.sqrt_c / (1.f - zc * zc) : 0.f;  // d atanh(zc) / d nc
  const float ds = (dzc * z - at * k.sqrt_c) / (z * z);
  return Rad{s, n >= REGCN_EPS ? ds / n : 0.f};
}

// exp_map_zero before its projection: tanh(sc n) / (sc n); *dsdn = its derivative.
__device__ __forceinline__ float exp0_t(float n, const Curv& k, float* dsdn) {
  const float nc = fmaxf(n, REGCN_EPS);
  const float z = k.sqrt_c * nc;
  const float th = tanhf(z);
  *dsdn = n >= REGCN_EPS ? (k.sqrt_c * (1.f - th * th) * z - th * k.sqrt_c) / (z * z) : 0.f;
  return th / z;
}

// exp0 (tanh stage then projection) as one radial map of x, |x| = n.
__device__ __forceinline__ Rad rad_exp0(float n, const Curv& k) {
  float dt;
  const float t = exp0_t(n, k, &dt);
  const Rad P = rad_project(t * n, k);
  // y = s_P(t n) t x: d/dn [s_P(t n) t] = s_P' (t' n + t) t + s_P t'
  const float dsp = P.kk * (t * n);  // s_P' (0 below eps)
  const float ds = dsp * (dt * n + t) * t + P.s * dt;
  return Rad{P.s * t, n >= REGCN_EPS ? ds / n : 0.f};
}

enum BwdOp : int { B_LOG0 = 0, B_EXP0 = 1, B_PROJECT = 2, B_APPLY_RADIUS = 3, B_RADIUS = 4, B_MOBIUS = 5 };

// dx (and dy: mobius_add's second operand; apply_radius: d radius) of one row op.
template <int OP>
__global__ __launch_bounds__(256) void k_rowmap_bwd(const float* __restrict__ x, const float* __restrict__ y,
                                                    const float* __restrict__ g, int64_t rows, int d, Curv k,
                                                    float* __restrict__ dx, float* __restrict__ dy) {
  const int lane = threadIdx.x & 63, col = lane * 4;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < rows; i += nw) {
    const f4 xv = load4(x + i * d, col, d);
    if constexpr (OP == B_RADIUS) {  // r = max(|x|, eps): dx = g_r x / |x|
      const float n = sqrtf(wave_sum(dot4(xv, xv)));
      const float gr = g[i];
      store4(dx + i * d, col, d, n >= REGCN_EPS ? xv * (gr / n) : f4{0.f, 0.f, 0.f, 0.f});
      continue;
    }
    const f4 gv = load4(g + i * d, col, d);
    if constexpr (OP == B_MOBIUS) {
      const f4 yv = load4(y + i * d, col, d);
      const float c = k.c;
      const float x2 = wave_sum(dot4(xv, xv)), y2 = wave_sum(dot4(yv, yv)), xy = wave_sum(dot4(xv, yv));
      const float xg = wave_sum(dot4(xv, gv)), yg = wave_sum(dot4(yv, gv));
      const float A = 1.f + 2.f * c * xy + c * y2, Bc = 1.f - c * x2;
      const float D = 1.f + 2.f * c * xy + c * c * x2 * y2 + REGCN_EPS;
      const float nu = sqrtf(fmaxf(A * A * x2 + 2.f * A * Bc * xy + Bc * Bc * y2, 0.f)) / D;
      const Rad P = rad_project(nu, k);
      const float ug = (A * xg + Bc * yg) / D;
      // gu = a1 g + a2 x + a3 y
      const float a1 = P.s, a2 = P.kk * ug * A / D, a3 = P.kk * ug * Bc / D;
      const float gux = a1 * xg + a2 * x2 + a3 * xy, guy = a1 * yg + a2 * xy + a3 * y2;
      const float guu = (A * gux + Bc * guy) / D;
      const float gA = gux / D, gB = guy / D, gD = -guu / D;
      const float gxy = 2.f * c * gA + 2.f * c * gD;
      const float gy2 = c * gA + c * c * x2 * gD;
      const float gx2 = -c * gB + c * c * y2 * gD;
      const float fa = A / D, fb = Bc / D;
      // gx = fa gu + gxy y + 2 gx2 x ; gy = fb gu + gxy x + 2 gy2 y
      store4(dx + i * d, col, d, gv * (fa * a1) + xv * (fa * a2 + 2.f * gx2) + yv * (fa * a3 + gxy));
      store4(dy + i * d, col, d, gv * (fb * a1) + xv * (fb * a2 + gxy) + yv * (fb * a3 + 2.f * gy2));
      continue;
    }
    const float n = sqrtf(wave_sum(dot4(xv, xv)));
    const float a = wave_sum(dot4(xv, gv));
    Rad R;
    if constexpr (OP == B_LOG0) R = rad_log0(n, k);
    else if constexpr (OP == B_EXP0) R = rad_exp0(n, k);
    else if constexpr (OP == B_PROJECT) R = rad_project(n, k);
    else {  // apply_radius: (x / max(|x|, eps)) clamp(r, eps, rmax)
      const float r = y[i];
      const float rc = fminf(fmaxf(r, REGCN_EPS), k.rmax);
      const float nc = fmaxf(n, REGCN_EPS);
      R = Rad{rc / nc, n >= REGCN_EPS ? (-rc / (nc * nc)) / n : 0.f};
      if (lane == 0) dy[i] = (r >= REGCN_EPS && r <= k.rmax) ? a / nc : 0.f;
    }
    store4(dx + i * d, col, d, gv * R.s + xv * (R.kk * a));
  }
}

// ------------------------------------------------------------------------- union backward
// Rows whose edges are walked serially (a Zipf hub has hundreds) run one workgroup per row,
// its LW waves on contiguous slices of the edges, partials combined in wave order.
constexpr int LW = 8;

// Pass 1, destination rows: per in-edge (CSR position p) the weight w_p and
// q_p = (G[v] norm[v] . (x[u] + rel[t])) dw_p/dr_u; the destination's radius gradient
// -sum q_p goes to drd[v].
__global__ __launch_bounds__(64 * LW) void k_union_bwd_dst(const float* __restrict__ x, const float* __restrict__ radius,
                                                           const float* __restrict__ rel, const float* __restrict__ norm,
                                                           const int* __restrict__ rowptr, const int* __restrict__ col_src,
                                                           const int* __restrict__ col_type, const float* __restrict__ G,
                                                           int V, int d, float gamma, float* __restrict__ we,
                                                           float* __restrict__ qe, float* __restrict__ drd) {
  __shared__ float part[LW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, col = lane * 4;
  for (int v = blockIdx.x; v < V; v += gridDim.x) {
    const int b = rowptr[v], e = rowptr[v + 1];
    const int q = (e - b + LW - 1) / LW;
    float acc = 0.f;
    if (e > b) {
      const f4 gv = load4(G + (int64_t)v * d, col, d) * norm[v];
      const float rv = radius[v];
      for (int p = b + wv * q; p < min(e, b + (wv + 1) * q); ++p) {
        const int u = col_src[p], t = col_type[p];
        const f4 m = load4(x + (int64_t)u * d, col, d) + load4(rel + (int64_t)t * d, col, d);
        const float s = wave_sum(dot4(gv, m));
        const float diff = radius[u] - rv;
        const float w = expf(-gamma * fabsf(diff));
        const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
        const float qq = s * (-gamma * w * sg);
        if (lane == 0) {
          we[p] = w;
          qe[p] = qq;
        }
        acc -= qq;
      }
    }
    if (lane == 0) part[wv] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = part[0];
#pragma unroll
      for (int w = 1; w < LW; ++w) t += part[w];
      drd[v] = t;
    }
    __syncthreads();
  }
}

// Pass 2, source rows (src-sorted positions sp[sptr[u] .. sptr[u+1])):
// dx[u] = sum_p w_p norm[dst] G[dst];  dradius[u] = drd[u] + sum_p q_p.
__global__ __launch_bounds__(64 * LW) void k_union_bwd_src(const float* __restrict__ norm, const int* __restrict__ sptr,
                                                           const int* __restrict__ sp, const int* __restrict__ csr_dst,
                                                           const float* __restrict__ G, const float* __restrict__ we,
                                                           const float* __restrict__ qe, const float* __restrict__ drd,
                                                           int V, int d, float* __restrict__ dx,
                                                           float* __restrict__ dradius) {
  __shared__ f4 part[LW][64];
  __shared__ float partq[LW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, col = lane * 4;
  for (int u = blockIdx.x; u < V; u += gridDim.x) {
    const int b = sptr[u], e = sptr[u + 1];
    const int q = (e - b + LW - 1) / LW;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    float qs = 0.f;
    for (int i = b + wv * q; i < min(e, b + (wv + 1) * q); ++i) {
      const int p = sp[i], v = csr_dst[p];
      acc += load4(G + (int64_t)v * d, col, d) * (we[p] * norm[v]);
      qs += qe[p];
    }
    part[wv][lane] = acc;
    if (lane == 0) partq[wv] = qs;
    __syncthreads();
    if (wv == 0) {
      f4 sx = part[0][lane];
      float sq = partq[0];
#pragma unroll
      for (int w = 1; w < LW; ++w) {
        sx += part[w][lane];
        sq += partq[w];
      }
      store4(dx + (int64_t)u * d, col, d, sx);
      if (lane == 0) dradius[u] = drd[u] + sq;
    }
    __syncthreads();
  }
}

// Pass 3, relation types (type-sorted positions): drel[t] = sum_p w_p norm[dst] G[dst].
// One workgroup per type, its 4 waves on contiguous quarters, combined in wave order.
__global__ __launch_bounds__(256) void k_union_bwd_type(const float* __restrict__ norm, const int* __restrict__ tptr,
                                                        const int* __restrict__ tp, const int* __restrict__ csr_dst,
                                                        const float* __restrict__ G, const float* __restrict__ we,
                                                        int R2, int d, float* __restrict__ drel) {
  __shared__ f4 part[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, col = lane * 4;
  for (int t = blockIdx.x; t < R2; t += gridDim.x) {
    const int b = tptr[t], e = tptr[t + 1];
    const int q = (e - b + 3) / 4;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = b + wv * q; i < min(e, b + (wv + 1) * q); ++i) {
      const int p = tp[i], v = csr_dst[p];
      acc += load4(G + (int64_t)v * d, col, d) * (we[p] * norm[v]);
    }
    part[wv][lane] = acc;
    __syncthreads();
    if (wv == 0) store4(drel + (int64_t)t * d, col, d, ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane]);
    __syncthreads();
  }
}

// ------------------------------------------------------------------------ Lorentz messages
// Lorentz point of exp0(m): L0 = (1 + c p2) / (sc den), Li = (2 phi / den) m, p2 = |exp0(m)|^2,
// den = max(1 - c p2, eps) (hyperbolic_ops.py:476-499); phi = exp0 factor incl. projection.
struct LPoint {
  float L0, beta_phi;  // Li = beta_phi m
};

__device__ __forceinline__ LPoint lorentz_point(float n2, const Curv& k) {
  float p2;
  const float phi = exp0_factor(n2, k, &p2);
  const float den = fmaxf(1.f - k.c * p2, REGCN_EPS);
  return LPoint{(1.f + k.c * p2) / (k.sqrt_c * den), 2.f * phi / den};
}

// dL/dm for upstream (g0, gv) at message m (|m| = n): dm = bp gv + coef m.
__device__ __forceinline__ void lorentz_point_bwd(float n, float g0, float gm, const Curv& k, float* bp,
                                                  float* coef) {
  const Rad E = rad_exp0(n, k);      // phi = E.s, phi'/n = E.kk
  const float phi = E.s;
  const float p2 = phi * phi * n * n;
  const float den_raw = 1.f - k.c * p2;
  const bool open = den_raw >= REGCN_EPS;
  const float den = fmaxf(den_raw, REGCN_EPS);
  const float dalpha = open ? 2.f * k.c / (k.sqrt_c * den * den) : k.c / (k.sqrt_c * REGCN_EPS);
  const float beta = 2.f / den;
  const float dbeta = open ? 2.f * k.c / (den * den) : 0.f;
  const float P1 = 2.f * phi * (E.kk * n * n + phi);  // dp2/dm = P1 m
  *bp = beta * phi;
  *coef = g0 * dalpha * P1 + gm * (dbeta * P1 * phi + beta * E.kk);
}

template <int S>
__device__ __forceinline__ f4 wfrag_apply_t(const WFrag<S>& w, f4 dm) {  // W^T dm per block
  if constexpr (S == 1) return dm * w.w[0];
  else if constexpr (S == 2)
    return f4{w.w[0].x * dm.x + w.w[0].y * dm.y, w.w[0].z * dm.x + w.w[0].w * dm.y,
              w.w[1].x * dm.z + w.w[1].y * dm.w, w.w[1].z * dm.z + w.w[1].w * dm.w};
  else return f4{dot4(w.w[0], dm), dot4(w.w[1 % WFrag<S>::NV], dm), dot4(w.w[2 % WFrag<S>::NV], dm),
                 dot4(w.w[3 % WFrag<S>::NV], dm)};
}

template <int S>
__device__ __forceinline__ void wfrag_outer_acc(WFrag<S>& acc, f4 xs, f4 dm) {  // dW += x dm^T per block
  if constexpr (S == 1) acc.w[0] += xs * dm;
  else if constexpr (S == 2) {
    acc.w[0] += f4{xs.x * dm.x, xs.x * dm.y, xs.y * dm.x, xs.y * dm.y};
    acc.w[1] += f4{xs.z * dm.z, xs.z * dm.w, xs.w * dm.z, xs.w * dm.w};
  } else {
    acc.w[0] += dm * xs.x;
    acc.w[1 % WFrag<S>::NV] += dm * xs.y;
    acc.w[2 % WFrag<S>::NV] += dm * xs.z;
    acc.w[3 % WFrag<S>::NV] += dm * xs.w;
  }
}

// Raw Lorentz sums (training forward): S0[v] = sum_e L0_e, Sv[v] = sum_e Li_e.  One
// workgroup per destination row, its LW waves on contiguous slices of the row's edges,
// combined in wave order: a hub row's serial chain (one wave reduction per edge) is 1/LW as
// long as with one wave per row.
template <int S>
__global__ __launch_bounds__(64 * LW) void k_lorentz_raw(const float* __restrict__ x, const float* __restrict__ rel,
                                                     const float* __restrict__ W, const int* __restrict__ rowptr,
                                                     const int* __restrict__ col_src, const int* __restrict__ col_type,
                                                     int V, int d, int wstride, Curv k, float* __restrict__ S0,
                                                     float* __restrict__ Sv) {
  __shared__ f4 part[LW][64];
  __shared__ float part0[LW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, col = lane * 4;
  const bool active = col < d;
  const int colc = min(col, d - 4);
  for (int v = blockIdx.x; v < V; v += gridDim.x) {
    const int b = rowptr[v], e = rowptr[v + 1];
    const int q = (e - b + LW - 1) / LW;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    float acc0 = 0.f;
    for (int p = b + wv * q; p < min(e, b + (wv + 1) * q); ++p) {
      const int u = col_src[p], t = col_type[p];
      WFrag<S> wf;
      wf.load(W + (int64_t)t * wstride, colc);
      f4 m = wf.apply(*reinterpret_cast<const f4*>(x + (int64_t)u * d + colc)) +
             *reinterpret_cast<const f4*>(rel + (int64_t)t * d + colc);
      if (!active) m = f4{0.f, 0.f, 0.f, 0.f};
      const LPoint L = lorentz_point(wave_sum(dot4(m, m)), k);
      acc0 += L.L0;
      acc += m * L.beta_phi;
    }
    part[wv][lane] = acc;
    if (lane == 0) part0[wv] = acc0;
    __syncthreads();
    if (wv == 0) {
      f4 sv = part[0][lane];
      float s0 = part0[0];
#pragma unroll
      for (int w = 1; w < LW; ++w) {
        sv += part[w][lane];
        s0 += part0[w];
      }
      store4(Sv + (int64_t)v * d, col, d, sv);
      if (lane == 0) S0[v] = s0;
    }
    __syncthreads();
  }
}

// dm of CSR edge p (message recomputed from its source row and relation).
template <int S>
__device__ __forceinline__ f4 lorentz_edge_dm(const float* __restrict__ x, const float* __restrict__ rel,
                                              const WFrag<S>& wf, f4 xs, int t, int v, const float* __restrict__ g0,
                                              const float* __restrict__ gS, int d, int col, int colc, bool active,
                                              const Curv& k) {
  f4 m = wf.apply(xs) + *reinterpret_cast<const f4*>(rel + (int64_t)t * d + colc);
  if (!active) m = f4{0.f, 0.f, 0.f, 0.f};
  const f4 gv = load4(gS + (int64_t)v * d, col, d);
  const float n = sqrtf(wave_sum(dot4(m, m)));
  const float gm = wave_sum(dot4(gv, m));
  float bp, coef;
  lorentz_point_bwd(n, g0[v], gm, k, &bp, &coef);
  return active ? gv * bp + m * coef : f4{0.f, 0.f, 0.f, 0.f};
}

// Source pass: dx[u] = sum over u's out-edges of blockdiag(W_t)^T dm_e; one workgroup per
// source row, LW waves on contiguous slices of its out-edges, combined in wave order.
template <int S>
__global__ __launch_bounds__(64 * LW) void k_lorentz_bwd_src(const float* __restrict__ x, const float* __restrict__ rel,
                                                         const float* __restrict__ W, const int* __restrict__ sptr,
                                                         const int* __restrict__ sp, const int* __restrict__ csr_dst,
                                                         const int* __restrict__ col_type, const float* __restrict__ g0,
                                                         const float* __restrict__ gS, int V, int d, int wstride,
                                                         Curv k, float* __restrict__ dx) {
  __shared__ f4 part[LW][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, col = lane * 4;
  const bool active = col < d;
  const int colc = min(col, d - 4);
  for (int u = blockIdx.x; u < V; u += gridDim.x) {
    const f4 xs = *reinterpret_cast<const f4*>(x + (int64_t)u * d + colc);
    const int b = sptr[u], e = sptr[u + 1];
    const int q = (e - b + LW - 1) / LW;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = b + wv * q; i < min(e, b + (wv + 1) * q); ++i) {
      const int p = sp[i], v = csr_dst[p], t = col_type[p];
      WFrag<S> wf;
      wf.load(W + (int64_t)t * wstride, colc);
      const f4 dm = lorentz_edge_dm<S>(x, rel, wf, xs, t, v, g0, gS, d, col, colc, active, k);
      acc += wfrag_apply_t<S>(wf, dm);
    }
    part[wv][lane] = acc;
    __syncthreads();
    if (wv == 0) {
      f4 sx = part[0][lane];
#pragma unroll
      for (int w = 1; w < LW; ++w) sx += part[w][lane];
      store4(dx + (int64_t)u * d, col, d, sx);
    }
    __syncthreads();
  }
}

// Type pass: drel[t] = sum dm_e, dW[t] = sum_e per-block x_src dm_e^T (one workgroup per type,
// 4 waves on contiguous quarters of its edges, combined in wave order).
template <int S>
__global__ __launch_bounds__(256) void k_lorentz_bwd_type(const float* __restrict__ x, const float* __restrict__ rel,
                                                          const float* __restrict__ W, const int* __restrict__ tptr,
                                                          const int* __restrict__ tp, const int* __restrict__ csr_dst,
                                                          const int* __restrict__ col_src, const float* __restrict__ g0,
                                                          const float* __restrict__ gS, int R2, int d, int wstride,
                                                          Curv k, float* __restrict__ drel, float* __restrict__ dW) {
  constexpr int NV = WFrag<S>::NV;
  __shared__ f4 part[4][64][NV + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, col = lane * 4;
  const bool active = col < d;
  const int colc = min(col, d - 4);
  for (int t = blockIdx.x; t < R2; t += gridDim.x) {
    const int b = tptr[t], e = tptr[t + 1];
    const int q = (e - b + 3) / 4;
    WFrag<S> wf, gw;
    wf.load(W + (int64_t)t * wstride, colc);
#pragma unroll
    for (int j = 0; j < NV; ++j) gw.w[j] = f4{0.f, 0.f, 0.f, 0.f};
    f4 gr = {0.f, 0.f, 0.f, 0.f};
    for (int i = b + wv * q; i < min(e, b + (wv + 1) * q); ++i) {
      const int p = tp[i], v = csr_dst[p], u = col_src[p];
      const f4 xs = *reinterpret_cast<const f4*>(x + (int64_t)u * d + colc);
      const f4 dm = lorentz_edge_dm<S>(x, rel, wf, xs, t, v, g0, gS, d, col, colc, active, k);
      gr += dm;
      wfrag_outer_acc<S>(gw, active ? xs : f4{0.f, 0.f, 0.f, 0.f}, dm);
    }
    part[wv][lane][0] = gr;
#pragma unroll
    for (int j = 0; j < NV; ++j) part[wv][lane][j + 1] = gw.w[j];
    __syncthreads();
    if (wv == 0) {
      store4(drel + (int64_t)t * d, col, d, ((part[0][lane][0] + part[1][lane][0]) + part[2][lane][0]) + part[3][lane][0]);
      if (active) {
#pragma unroll
        for (int j = 0; j < NV; ++j)
          *reinterpret_cast<f4*>(dW + (int64_t)t * wstride + S * col + 4 * j) =
              ((part[0][lane][j + 1] + part[1][lane][j + 1]) + part[2][lane][j + 1]) + part[3][lane][j + 1];
      }
    }
    __syncthreads();
  }
}

inline unsigned waves_grid(int64_t n) {
  const int64_t b = (n + 3) / 4;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(b, 16384));
}

int check_d(int d) {
  if (d <= 0 || d > 256 || (d & 3)) return set_error(REGCN_ENOTSUP, "backward kernels need d %% 4 == 0 and d <= 256 (d=%d)", d);
  return 0;
}

}  // namespace

int rowmap_bwd(int op, const float* x, const float* y, const float* g, int64_t rows, int d, float c, float* dx,
               float* dy, hipStream_t st) {
  int rc = check_d(d);
  if (rc) return rc;
  if (!x || !g || !dx) return set_error(REGCN_EINVAL, "null pointer");
  if ((op == B_APPLY_RADIUS || op == B_MOBIUS) && (!y || !dy)) return set_error(REGCN_EINVAL, "null pointer");
  if (rows == 0) return 0;
  const Curv k = make_curv(c);
  const dim3 gr(waves_grid(rows)), b(256);
  switch (op) {
    case B_LOG0: hipLaunchKernelGGL(k_rowmap_bwd<B_LOG0>, gr, b, 0, st, x, y, g, rows, d, k, dx, dy); break;
    case B_EXP0: hipLaunchKernelGGL(k_rowmap_bwd<B_EXP0>, gr, b, 0, st, x, y, g, rows, d, k, dx, dy); break;
    case B_PROJECT: hipLaunchKernelGGL(k_rowmap_bwd<B_PROJECT>, gr, b, 0, st, x, y, g, rows, d, k, dx, dy); break;
    case B_APPLY_RADIUS:
      hipLaunchKernelGGL(k_rowmap_bwd<B_APPLY_RADIUS>, gr, b, 0, st, x, y, g, rows, d, k, dx, dy);
      break;
    case B_RADIUS: hipLaunchKernelGGL(k_rowmap_bwd<B_RADIUS>, gr, b, 0, st, x, y, g, rows, d, k, dx, dy); break;
    case B_MOBIUS: hipLaunchKernelGGL(k_rowmap_bwd<B_MOBIUS>, gr, b, 0, st, x, y, g, rows, d, k, dx, dy); break;
    default: return set_error(REGCN_EINVAL, "unknown row-map backward op %d", op);
  }
  return check_launch("k_rowmap_bwd");
}

int union_bwd(const regcn_edge_bwd_desc* a, float gamma, hipStream_t st) {
  int rc = check_d(a->d);
  if (rc) return rc;
  if (!a->x || !a->radius || !a->rel || !a->norm || !a->G || !a->dx || !a->drel || !a->dradius || !a->edge_scratch)
    return set_error(REGCN_EINVAL, "null pointer");
  const int V = a->V, d = a->d, R2 = a->R2;
  float* we = a->edge_scratch;
  float* qe = we + a->E;
  float* drd = qe + a->E;
  const dim3 b(256);
  const dim3 gr((unsigned)std::max(1, std::min(V, 65535))), bl(64 * LW);  // one workgroup per row
  hipLaunchKernelGGL(k_union_bwd_dst, gr, bl, 0, st, a->x, a->radius, a->rel, a->norm, a->rowptr,
                     a->col_src, a->col_type, a->G, V, d, gamma, we, qe, drd);
  hipLaunchKernelGGL(k_union_bwd_src, gr, bl, 0, st, a->norm, a->sptr, a->sp, a->csr_dst, a->G, we, qe,
                     drd, V, d, a->dx, a->dradius);
  hipLaunchKernelGGL(k_union_bwd_type, dim3(std::max(1, std::min(R2, 65535))), b, 0, st, a->norm, a->tptr, a->tp,
                     a->csr_dst, a->G, we, R2, d, a->drel);
  return check_launch("union_bwd");
}

int lorentz_raw(const float* x, const float* rel, const float* W, const int* rowptr, const int* col_src,
                const int* col_type, int V, int d, int nb, float c, float* S0, float* Sv, hipStream_t st) {
  int rc = check_d(d);
  if (rc) return rc;
  if (nb <= 0 || d % nb) return set_error(REGCN_EINVAL, "d=%d not divisible by num_bases=%d", d, nb);
  const int s = d / nb, ws = nb * s * s;
  if (!x || !rel || !W || !rowptr || !S0 || !Sv) return set_error(REGCN_EINVAL, "null pointer");
  const Curv k = make_curv(c);
  const dim3 g((unsigned)std::max(1, std::min(V, 65535))), b(64 * LW);  // one workgroup per row
  if (s == 1) hipLaunchKernelGGL(k_lorentz_raw<1>, g, b, 0, st, x, rel, W, rowptr, col_src, col_type, V, d, ws, k, S0, Sv);
  else if (s == 2) hipLaunchKernelGGL(k_lorentz_raw<2>, g, b, 0, st, x, rel, W, rowptr, col_src, col_type, V, d, ws, k, S0, Sv);
  else if (s == 4) hipLaunchKernelGGL(k_lorentz_raw<4>, g, b, 0, st, x, rel, W, rowptr, col_src, col_type, V, d, ws, k, S0, Sv);
  else return set_error(REGCN_ENOTSUP, "training Lorentz layer needs block size d/num_bases in {1, 2, 4} (got %d)", s);
  return check_launch("k_lorentz_raw");
}

int lorentz_bwd(const regcn_edge_bwd_desc* a, int nb, float c, hipStream_t st) {
  int rc = check_d(a->d);
  if (rc) return rc;
  const int V = a->V, d = a->d, R2 = a->R2;
  if (nb <= 0 || d % nb) return set_error(REGCN_EINVAL, "d=%d not divisible by num_bases=%d", d, nb);
  const int s = d / nb, ws = nb * s * s;
  if (!a->x || !a->rel || !a->W || !a->G || !a->G0 || !a->dx || !a->drel || !a->dW)
    return set_error(REGCN_EINVAL, "null pointer");
  const Curv k = make_curv(c);
  const dim3 g((unsigned)std::max(1, std::min(V, 65535))), gt(std::max(1, std::min(R2, 65535))), b(256);
#define LB(SS)                                                                                                   \
  {                                                                                                              \
  hipLaunchKernelGGL(k_lorentz_bwd_src<SS>, g, dim3(64 * LW), 0, st, a->x, a->rel, a->W, a->sptr, a->sp, a->csr_dst,       \
                     a->col_type, a->G0, a->G, V, d, ws, k, a->dx);                                              \
  hipLaunchKernelGGL(k_lorentz_bwd_type<SS>, gt, b, 0, st, a->x, a->rel, a->W, a->tptr, a->tp, a->csr_dst,     \
                     a->col_src, a->G0, a->G, R2, d, ws, k, a->drel, a->dW);                               \
  }
  if (s == 1) LB(1)
  else if (s == 2) LB(2)
  else if (s == 4) LB(4)
  else return set_error(REGCN_ENOTSUP, "training Lorentz layer needs block size d/num_bases in {1, 2, 4} (got %d)", s);
#undef LB
  return check_launch("lorentz_bwd");
}

}  // namespace regcn
