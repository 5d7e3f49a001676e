// Row-wise Poincaré / Lorentz maps.
//
// HBM-bound: each op reads and writes whole rows once.  One 64-lane wave per
// row; lane l holds elements l, l+64, ... (EPL = ceil(d/64) per lane), so every
// wave-instruction touches 256 contiguous bytes for any d.  Row norms are
// wave reductions.  Reference: hyperbolic_src/hyperbolic_ops.py.
#include "common.h"
#include "regcn_internal.h"

namespace regcn {

enum RowOp : int {
  OP_LOG0 = 0,
  OP_EXP0 = 1,
  OP_PROJECT = 2,
  OP_APPLY_RADIUS = 3,
  OP_RADIUS = 4,
  OP_MOBIUS_ADD = 5,
  OP_TO_LORENTZ = 6,
  OP_TO_POINCARE = 7,
  OP_PROLOGUE = 8,      // x = log0(h), r = max(|h|, eps) in one pass
  OP_SUMSQ = 9,         // |x|^2 (scorer row norms)
  OP_LN_ROUNDTRIP = 10, // exp0(normalize(log0(x)))  (hyperbolic_model.py:926-929)
  OP_INIT = 11,         // h = apply_radius(exp0(x), r_s); also log0(h), |h|  (:779-782)
  OP_INIT_LN = 12,      // same with exp0(normalize(x))
};

template <int EPL>
struct Frag {
  float v[EPL];
  __device__ __forceinline__ void load(const float* row, int d, int lane, int off = 0) {
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      int col = lane + j * WAVE;
      v[j] = col < d ? row[col + off] : 0.f;
    }
  }
  __device__ __forceinline__ void store(float* row, int d, int lane, int off = 0) const {
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      int col = lane + j * WAVE;
      if (col < d) row[col + off] = v[j];
    }
  }
  __device__ __forceinline__ float sumsq() const {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) s += v[j] * v[j];
    return wave_sum(s);
  }
  __device__ __forceinline__ float dot(const Frag& o) const {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) s += v[j] * o.v[j];
    return wave_sum(s);
  }
  __device__ __forceinline__ void scale(float f) {
#pragma unroll
    for (int j = 0; j < EPL; ++j) v[j] *= f;
  }
};

template <int EPL, int OP>
__global__ __launch_bounds__(256) void k_rowmap(const float* __restrict__ a, const float* __restrict__ b,
                                                const float* __restrict__ vec, int64_t rows, int d,
                                                Curv k, float* __restrict__ out, float* __restrict__ out2,
                                                float* __restrict__ out3, const int32_t* __restrict__ src,
                                                const int32_t* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < rows; i += nwaves) {
    // OP_INIT / OP_INIT_LN over a row list (regcn_init_entity_rows_f32): input row src[i],
    // output row dst[i] (i without dst); the other ops run rows in place (src = dst = NULL)
    const int64_t r = src ? (int64_t)src[i] : i;
    const int64_t t = dst ? (int64_t)dst[i] : (src ? i : r);
    Frag<EPL> x;
    if (OP == OP_TO_POINCARE) {
      x.load(a + r * (d + 1), d, lane, 1);
      float y0 = a[r * (d + 1)];
      x.scale(1.0f / fmaxf(1.0f + y0 * k.sqrt_c, REGCN_EPS));        // hyperbolic_ops.py:516-518
      x.store(out + r * d, d, lane);
      continue;
    }
    x.load(a + r * d, d, lane);
    float n2 = x.sumsq();
    if (OP == OP_LOG0) {
      x.scale(log0_factor(n2, k));
      x.store(out + r * d, d, lane);
    } else if (OP == OP_PROLOGUE) {
      float rad = row_radius(n2);
      x.scale(log0_factor(n2, k));
      x.store(out + r * d, d, lane);
      if (lane == 0) out2[r] = rad;
    } else if (OP == OP_EXP0) {
      x.scale(exp0_factor(n2, k));
      x.store(out + r * d, d, lane);
    } else if (OP == OP_PROJECT) {
      x.scale(project_factor(n2, k));
      x.store(out + r * d, d, lane);
    } else if (OP == OP_APPLY_RADIUS) {
      float n = row_radius(n2);
      float rr = fminf(fmaxf(vec[r], REGCN_EPS), k.rmax);
#pragma unroll
      for (int j = 0; j < EPL; ++j) x.v[j] = x.v[j] * fdiv(rr, n);
      x.store(out + r * d, d, lane);
    } else if (OP == OP_RADIUS) {
      if (lane == 0) out[r] = row_radius(n2);
    } else if (OP == OP_SUMSQ) {
      if (lane == 0) out[r] = n2;
    } else if (OP == OP_LN_ROUNDTRIP) {
      x.scale(log0_factor(n2, k));
      x.scale(frcp(fmaxf(fsqrt(x.sumsq()), 1e-12f)));
      x.scale(exp0_factor(x.sumsq(), k));
      x.store(out + r * d, d, lane);
    } else if (OP == OP_INIT || OP == OP_INIT_LN) {
      if (OP == OP_INIT_LN) {
        x.scale(frcp(fmaxf(fsqrt(n2), 1e-12f)));
        n2 = x.sumsq();
      }
      x.scale(exp0_factor(n2, k));
      {
        const float n = row_radius(x.sumsq());
        const float rr = fminf(fmaxf(vec[r], REGCN_EPS), k.rmax);
#pragma unroll
        for (int j = 0; j < EPL; ++j) x.v[j] = x.v[j] * fdiv(rr, n);
      }
      if (out) x.store(out + t * d, d, lane);
      const float h2 = x.sumsq();
      if (lane == 0 && out3) out3[t] = row_radius(h2);
      if (out2) {
        x.scale(log0_factor(h2, k));
        x.store(out2 + t * d, d, lane);
      }
    } else if (OP == OP_MOBIUS_ADD) {                                   // hyperbolic_ops.py:118-143
      Frag<EPL> y;
      y.load(b + r * d, d, lane);
      float y2 = y.sumsq(), xy = x.dot(y);
      float A = 1.f + 2.f * k.c * xy + k.c * y2;
      float B = 1.f - k.c * n2;
      float den = 1.f + 2.f * k.c * xy + k.c * k.c * n2 * y2 + REGCN_EPS;
#pragma unroll
      for (int j = 0; j < EPL; ++j) x.v[j] = (A * x.v[j] + B * y.v[j]) / den;
      x.scale(project_factor(x.sumsq(), k));
      x.store(out + r * d, d, lane);
    } else if (OP == OP_TO_LORENTZ) {                                   // hyperbolic_ops.py:476-499
      float den = fmaxf(1.f - k.c * n2, REGCN_EPS);
      if (lane == 0) out[r * (d + 1)] = (1.f + k.c * n2) / (k.sqrt_c * den);
#pragma unroll
      for (int j = 0; j < EPL; ++j) x.v[j] = 2.f * x.v[j] / den;
      x.store(out + r * (d + 1), d, lane, 1);
    }
  }
}

// The initial entity state (OP_INIT / OP_INIT_LN) with the next row's loads in flight: HBM-bound
// (2.4 KB per row) with one row per wave the loads of a wave's next row wait on the current
// row's reduction chain; here row i + nwaves is fetched (EPL + 1 registers) before row i is
// mapped, so a wave keeps two rows of loads outstanding.  The same arithmetic as k_rowmap's
// OP_INIT branch, so the same bits.
template <int EPL, int OP>
__global__ __launch_bounds__(256) void k_init_rows(const float* __restrict__ a, const float* __restrict__ vec,
                                                   int64_t rows, int d, Curv k, float* __restrict__ out,
                                                   float* __restrict__ out2, float* __restrict__ out3,
                                                   const int32_t* __restrict__ src, const int32_t* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (i >= rows) return;
  Frag<EPL> nx;
  float nv;
  {
    const int64_t r = src ? (int64_t)src[i] : i;
    nx.load(a + r * d, d, lane);
    nv = vec[r];
  }
  for (; i < rows; i += nwaves) {
    Frag<EPL> x = nx;
    const float rv = nv;
    const int64_t nxt = i + nwaves;
    if (nxt < rows) {
      const int64_t r = src ? (int64_t)src[nxt] : nxt;
      nx.load(a + r * d, d, lane);
      nv = vec[r];
    }
    const int64_t t = dst ? (int64_t)dst[i] : i;
    float n2 = x.sumsq();
    if (OP == OP_INIT_LN) {
      x.scale(frcp(fmaxf(fsqrt(n2), 1e-12f)));
      n2 = x.sumsq();
    }
    x.scale(exp0_factor(n2, k));
    {
      const float n = row_radius(x.sumsq());
      const float rr = fminf(fmaxf(rv, REGCN_EPS), k.rmax);
#pragma unroll
      for (int j = 0; j < EPL; ++j) x.v[j] = x.v[j] * fdiv(rr, n);
    }
    if (out) x.store(out + t * d, d, lane);
    const float h2 = x.sumsq();
    if (lane == 0 && out3) out3[t] = row_radius(h2);
    if (out2) {
      x.scale(log0_factor(h2, k));
      x.store(out2 + t * d, d, lane);
    }
  }
}

// The same map with 16-B accesses: lane l holds elements 4l .. 4l + 3 of the row (d % 4 == 0,
// d <= 256, 16-B aligned rows), so a row moves in one dwordx4 load and one dwordx4 store per
// output instead of ceil(d / 64) dword ones; the next row's load is in flight as above.  The
// row sums run in a different order than k_rowmap's (4 consecutive elements per lane), so the
// last bits may differ from it.
__device__ __forceinline__ float sq4(const float4& v) { return v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w; }
__device__ __forceinline__ void scale4(float4& v, float f) { v.x *= f; v.y *= f; v.z *= f; v.w *= f; }

template <int OP>
__global__ __launch_bounds__(256) void k_init_rows4(const float* __restrict__ a, const float* __restrict__ vec,
                                                    int64_t rows, int d, Curv k, float* __restrict__ out,
                                                    float* __restrict__ out2, float* __restrict__ out3,
                                                    const int32_t* __restrict__ src, const int32_t* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const bool on = lane < (d >> 2);
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (i >= rows) return;
  float4 nx = make_float4(0.f, 0.f, 0.f, 0.f);
  float nv;
  {
    const int64_t r = src ? (int64_t)src[i] : i;
    if (on) nx = reinterpret_cast<const float4*>(a + r * d)[lane];
    nv = vec[r];
  }
  for (; i < rows; i += nwaves) {
    float4 x = nx;
    const float rv = nv;
    const int64_t nxt = i + nwaves;
    if (nxt < rows) {
      const int64_t r = src ? (int64_t)src[nxt] : nxt;
      if (on) nx = reinterpret_cast<const float4*>(a + r * d)[lane];
      nv = vec[r];
    }
    const int64_t t = dst ? (int64_t)dst[i] : i;
    float n2 = wave_sum(sq4(x));
    if (OP == OP_INIT_LN) {
      scale4(x, frcp(fmaxf(fsqrt(n2), 1e-12f)));
      n2 = wave_sum(sq4(x));
    }
    scale4(x, exp0_factor(n2, k));
    {
      const float n = row_radius(wave_sum(sq4(x)));
      const float rr = fminf(fmaxf(rv, REGCN_EPS), k.rmax);
      x = x * fdiv(rr, n);
    }
    if (out && on) reinterpret_cast<float4*>(out + t * d)[lane] = x;
    const float h2 = wave_sum(sq4(x));
    if (lane == 0 && out3) out3[t] = row_radius(h2);
    if (out2) {
      scale4(x, log0_factor(h2, k));
      if (on) reinterpret_cast<float4*>(out2 + t * d)[lane] = x;
    }
  }
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int OP>
static int launch_init(const float* a, const float* vec, int64_t rows, int d, const Curv& k, float* out,
                       float* out2, float* out3, hipStream_t st, const int32_t* src, const int32_t* dst) {
  if (rows == 0) return 0;
  int64_t blocks = (rows + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  dim3 g((unsigned)blocks), blk(256);
  if (d % 4 == 0 && d <= 256 && aligned16(a) && (!out || aligned16(out)) && (!out2 || aligned16(out2))) {
    hipLaunchKernelGGL((k_init_rows4<OP>), g, blk, 0, st, a, vec, rows, d, k, out, out2, out3, src, dst);
    return check_launch("k_init_rows4");
  }
  int epl = (d + 63) / 64;
  if (epl <= 1) hipLaunchKernelGGL((k_init_rows<1, OP>), g, blk, 0, st, a, vec, rows, d, k, out, out2, out3, src, dst);
  else if (epl <= 2) hipLaunchKernelGGL((k_init_rows<2, OP>), g, blk, 0, st, a, vec, rows, d, k, out, out2, out3, src, dst);
  else if (epl <= 4) hipLaunchKernelGGL((k_init_rows<4, OP>), g, blk, 0, st, a, vec, rows, d, k, out, out2, out3, src, dst);
  else if (epl <= 8) hipLaunchKernelGGL((k_init_rows<8, OP>), g, blk, 0, st, a, vec, rows, d, k, out, out2, out3, src, dst);
  else if (epl <= 16) hipLaunchKernelGGL((k_init_rows<16, OP>), g, blk, 0, st, a, vec, rows, d, k, out, out2, out3, src, dst);
  else return set_error(REGCN_EINVAL, "row width d=%d exceeds 1024", d);
  return check_launch("k_init_rows");
}

// REGCN_INIT_PLAIN=1: the initial state through k_rowmap (no prefetch), for A/B measurements
static bool init_plain() {
  static const bool v = [] { const char* e = getenv("REGCN_INIT_PLAIN"); return e && e[0] == '1'; }();
  return v;
}

template <int OP>
static int launch_rowmap(const float* a, const float* b, const float* vec, int64_t rows, int d,
                         const Curv& k, float* out, float* out2, float* out3, hipStream_t st,
                         const int32_t* src = nullptr, const int32_t* dst = nullptr) {
  if (rows == 0) return 0;
  int64_t blocks = (rows + 3) / 4;
  if (blocks > 8192) blocks = 8192;                      // grid-stride beyond 8 blocks/CU
  dim3 g((unsigned)blocks), blk(256);
  int epl = (d + 63) / 64;
  if (epl <= 1) hipLaunchKernelGGL((k_rowmap<1, OP>), g, blk, 0, st, a, b, vec, rows, d, k, out, out2, out3, src, dst);
  else if (epl <= 2) hipLaunchKernelGGL((k_rowmap<2, OP>), g, blk, 0, st, a, b, vec, rows, d, k, out, out2, out3, src, dst);
  else if (epl <= 4) hipLaunchKernelGGL((k_rowmap<4, OP>), g, blk, 0, st, a, b, vec, rows, d, k, out, out2, out3, src, dst);
  else if (epl <= 8) hipLaunchKernelGGL((k_rowmap<8, OP>), g, blk, 0, st, a, b, vec, rows, d, k, out, out2, out3, src, dst);
  else if (epl <= 16) hipLaunchKernelGGL((k_rowmap<16, OP>), g, blk, 0, st, a, b, vec, rows, d, k, out, out2, out3, src, dst);
  else return set_error(REGCN_EINVAL, "row width d=%d exceeds 1024", d);
  return check_launch("k_rowmap");
}

int rowmap(int op, const float* a, const float* b, const float* vec, int64_t rows, int d, float c,
           float* out, float* out2, float* out3, hipStream_t st) {
  if (d <= 0) return set_error(REGCN_EINVAL, "d must be positive");
  // the initial state may skip h (out) when x is written (its consumers read x and |h| only)
  const bool init_op = op == OP_INIT || op == OP_INIT_LN;
  if (!a || (!out && !(init_op && out2))) return set_error(REGCN_EINVAL, "null pointer");
  Curv k = make_curv(c);
  switch (op) {
    case OP_LOG0: return launch_rowmap<OP_LOG0>(a, b, vec, rows, d, k, out, out2, out3, st);
    case OP_EXP0: return launch_rowmap<OP_EXP0>(a, b, vec, rows, d, k, out, out2, out3, st);
    case OP_PROJECT: return launch_rowmap<OP_PROJECT>(a, b, vec, rows, d, k, out, out2, out3, st);
    case OP_APPLY_RADIUS:
      if (!vec) return set_error(REGCN_EINVAL, "apply_radius needs a radius vector");
      return launch_rowmap<OP_APPLY_RADIUS>(a, b, vec, rows, d, k, out, out2, out3, st);
    case OP_RADIUS: return launch_rowmap<OP_RADIUS>(a, b, vec, rows, d, k, out, out2, out3, st);
    case OP_MOBIUS_ADD:
      if (!b) return set_error(REGCN_EINVAL, "mobius_add needs y");
      return launch_rowmap<OP_MOBIUS_ADD>(a, b, vec, rows, d, k, out, out2, out3, st);
    case OP_TO_LORENTZ: return launch_rowmap<OP_TO_LORENTZ>(a, b, vec, rows, d, k, out, out2, out3, st);
    case OP_TO_POINCARE: return launch_rowmap<OP_TO_POINCARE>(a, b, vec, rows, d, k, out, out2, out3, st);
    case OP_PROLOGUE:
      if (!out2) return set_error(REGCN_EINVAL, "prologue needs a radius output");
      return launch_rowmap<OP_PROLOGUE>(a, b, vec, rows, d, k, out, out2, out3, st);
    case OP_SUMSQ: return launch_rowmap<OP_SUMSQ>(a, b, vec, rows, d, k, out, out2, out3, st);
    case OP_LN_ROUNDTRIP: return launch_rowmap<OP_LN_ROUNDTRIP>(a, b, vec, rows, d, k, out, out2, out3, st);
    case OP_INIT:
    case OP_INIT_LN:
      if (!vec) return set_error(REGCN_EINVAL, "init needs the static radius");
      if (!init_plain()) {
        if (op == OP_INIT) return launch_init<OP_INIT>(a, vec, rows, d, k, out, out2, out3, st, nullptr, nullptr);
        return launch_init<OP_INIT_LN>(a, vec, rows, d, k, out, out2, out3, st, nullptr, nullptr);
      }
      if (op == OP_INIT) return launch_rowmap<OP_INIT>(a, b, vec, rows, d, k, out, out2, out3, st);
      return launch_rowmap<OP_INIT_LN>(a, b, vec, rows, d, k, out, out2, out3, st);
  }
  return set_error(REGCN_EINVAL, "unknown row op %d", op);
}

int init_rows(const float* dyn, const float* r_static, const int32_t* src, const int32_t* dst, int64_t n, int d,
              float c, int layer_norm, float* h, float* x, float* r, hipStream_t st) {
  if (d <= 0) return set_error(REGCN_EINVAL, "d must be positive");
  if (n < 0) return set_error(REGCN_EINVAL, "negative row count");
  if (n == 0) return 0;
  if (!dyn || !r_static || !src || !x || !r) return set_error(REGCN_EINVAL, "null pointer");
  Curv k = make_curv(c);
  if (init_plain()) {
    if (layer_norm) return launch_rowmap<OP_INIT_LN>(dyn, nullptr, r_static, n, d, k, h, x, r, st, src, dst);
    return launch_rowmap<OP_INIT>(dyn, nullptr, r_static, n, d, k, h, x, r, st, src, dst);
  }
  if (layer_norm) return launch_init<OP_INIT_LN>(dyn, r_static, n, d, k, h, x, r, st, src, dst);
  return launch_init<OP_INIT>(dyn, r_static, n, d, k, h, x, r, st, src, dst);
}


// ------------------------------------------------------- owner-partition row exchange
// The rows of x (d floats) and |h| (1 float) the next layer of another rank reads, packed as
// one record of stride d + 4 floats (16-B aligned records: the x part moves as 16-B vectors;
// float d holds |h|, d+1..d+3 are padding) for one all_to_all (parallel.ExchangePlan); the
// unpack scatters the received records back.  HBM-bound, 2 x 816 B of traffic per row: a wave
// moves XR_ROWS records, all loads issued before the stores (lane l: the 16-B group l of each,
// d <= 252; lane d/4 the radius).
constexpr int XR_ROWS = 4;
__global__ __launch_bounds__(256) void k_pack_rows(const float* __restrict__ x, const float* __restrict__ r,
                                                   const int64_t* __restrict__ idx, int64_t n, int d,
                                                   float* __restrict__ out) {
  const int64_t i0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * XR_ROWS;
  const int lane = threadIdx.x & 63, q = d >> 2;
  f4 v[XR_ROWS];
#pragma unroll
  for (int u = 0; u < XR_ROWS; ++u) {
    const int64_t i = min(i0 + u, n - 1);
    const int64_t src = idx[i];
    if (lane < q) v[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x + src * d) + lane);
    else v[u] = f4{lane == q ? r[src] : 0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int u = 0; u < XR_ROWS; ++u)
    if (i0 + u < n && lane <= q) reinterpret_cast<f4*>(out + (i0 + u) * (d + 4))[lane] = v[u];
}

__global__ __launch_bounds__(256) void k_unpack_rows(const float* __restrict__ in, const int64_t* __restrict__ idx,
                                                     int64_t n, int d, float* __restrict__ x, float* __restrict__ r) {
  const int64_t i0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * XR_ROWS;
  const int lane = threadIdx.x & 63, q = d >> 2;
  f4 v[XR_ROWS];
  int64_t dst[XR_ROWS];
#pragma unroll
  for (int u = 0; u < XR_ROWS; ++u) {
    const int64_t i = min(i0 + u, n - 1);
    dst[u] = idx[i];
    v[u] = lane <= q ? __builtin_nontemporal_load(reinterpret_cast<const f4*>(in + i * (d + 4)) + lane)
                     : f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int u = 0; u < XR_ROWS; ++u) {
    if (i0 + u >= n) continue;
    if (lane < q) reinterpret_cast<f4*>(x + dst[u] * d)[lane] = v[u];
    else if (lane == q) r[dst[u]] = v[u].x;
  }
}

// The send side of the halo exchange: rows idx[i] of x and |h| gathered into a contiguous x
// block (stride d) and |h| vector, which two all_to_alls deliver straight into the receivers'
// halo rows (no scatter on the receiving side; parallel.ExchangePlan).
constexpr int GR_ROWS = 8;  // rows in flight per wave in the halo gather
__global__ __launch_bounds__(256) void k_gather_rows(const float* __restrict__ x, const float* __restrict__ r,
                                                     const int64_t* __restrict__ idx, int64_t n, int d,
                                                     float* __restrict__ x_out, float* __restrict__ r_out) {
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t i0 = ((int64_t)blockIdx.x * 4 + wv) * GR_ROWS;
  const int lane = threadIdx.x & 63, q = d >> 2;
  // the wave's GR_ROWS source ids in one load (lane u), then broadcast: one round trip
  const int64_t my = idx[min(i0 + min(lane, GR_ROWS - 1), n - 1)];
  f4 v[GR_ROWS];
#pragma unroll
  for (int u = 0; u < GR_ROWS; ++u) {
    const int64_t src = __builtin_amdgcn_readlane((int)my, u) | ((int64_t)__builtin_amdgcn_readlane((int)(my >> 32), u) << 32);
    // plain loads: the rows were just written by the chunk's tail and are served by the caches
    if (lane < q) v[u] = reinterpret_cast<const f4*>(x + src * d)[lane];
    else v[u] = f4{lane == q ? r[src] : 0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int u = 0; u < GR_ROWS; ++u) {
    if (i0 + u >= n) break;
    if (lane < q) reinterpret_cast<f4*>(x_out + (i0 + u) * d)[lane] = v[u];
    else if (lane == q) r_out[i0 + u] = v[u].x;
  }
}

int gather_rows(const float* x, const float* r, const int64_t* idx, int64_t n, int d, float* x_out, float* r_out,
                hipStream_t st) {
  if (n < 0) return set_error(REGCN_EINVAL, "negative row count");
  if (n == 0) return 0;
  if (!x || !r || !idx || !x_out || !r_out) return set_error(REGCN_EINVAL, "null pointer");
  if (d <= 0 || (d & 3) || d > 4 * (WAVE - 1)) return set_error(REGCN_EINVAL, "row gather needs d %% 4 == 0, d <= 252");
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(x_out)) & 15)
    return set_error(REGCN_EINVAL, "row gather needs 16-B aligned x and output");
  const int64_t blocks = (n + 4 * GR_ROWS - 1) / (4 * GR_ROWS);
  if (blocks > 0x7fffffffL) return set_error(REGCN_EINVAL, "row gather grid too large");
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)blocks), dim3(256), 0, st, x, r, idx, n, d, x_out, r_out);
  return check_launch("k_gather_rows");
}

int exchange_rows(int pack, float* x, float* r, const int64_t* idx, int64_t n, int d, float* buf, hipStream_t st) {
  if (n < 0) return set_error(REGCN_EINVAL, "negative row count");
  if (n == 0) return 0;
  if (!x || !r || !idx || !buf) return set_error(REGCN_EINVAL, "null pointer");
  if (d <= 0 || (d & 3) || d > 4 * (WAVE - 1)) return set_error(REGCN_EINVAL, "row exchange needs d %% 4 == 0, d <= 252");
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(buf)) & 15)
    return set_error(REGCN_EINVAL, "row exchange needs 16-B aligned x and buffer");
  const int64_t blocks = (n + 4 * XR_ROWS - 1) / (4 * XR_ROWS);
  if (blocks > 0x7fffffffL) return set_error(REGCN_EINVAL, "row exchange grid too large");
  if (pack) hipLaunchKernelGGL(k_pack_rows, dim3((unsigned)blocks), dim3(256), 0, st, x, r, idx, n, d, buf);
  else hipLaunchKernelGGL(k_unpack_rows, dim3((unsigned)blocks), dim3(256), 0, st, buf, idx, n, d, x, r);
  return check_launch(pack ? "k_pack_rows" : "k_unpack_rows");
}

}  // namespace regcn
