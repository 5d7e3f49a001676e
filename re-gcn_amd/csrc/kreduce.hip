// Long-K products of the training backward:
//     C (M x N) = sum_k A(k, m) B(k, n)  (+ C0),   M, N <= a few hundred, K up to |V|.
// They are the weight gradients x^T dy of the encoder's (V x d) @ (d x d) products
// (hyperbolic_layers.py self loop / evolve loop / neighbour weight / skip gate,
// hyperbolic_model.py time gate: K = V, M = N = d), the cross-entropy backward's
// dq = coef E (K = |V| candidates, M = queries) and de = coef^T Q (K = queries, M = |V|),
// and the decoders' nn.Linear products on a mini-batch of queries (M = 64-128, N = K = d:
// a library GEMM runs these on ONE 256 x 224 macro tile, 33-46 us each).
// A library GEMM tiles the small output into a few dozen macro tiles and walks the whole K
// in each (measured 54 us for 7128 x 200 x 200 on 49 workgroups); here K is split over
// workgroups (and over the waves of a workgroup) so a launch fills the 256 CUs; a long K's
// split partials are summed by a second pass in a fixed order (deterministic; no atomics).
//
// A workgroup (4 waves) owns a 32 x 32 output tile (2 x 2 v_mfma_f32_16x16x4_f32 tiles) and
// one K chunk, whose 32-k groups its waves take round-robin; the four partial tiles are
// summed through LDS in wave order, so a short K (the K = d products) needs no second
// launch.  Operands are read straight from global memory (L1/L2 absorb the reuse): in a
// group of 32 k, lane (lo = l & 15, q = l >> 4) supplies at MFMA step e (0..7) the A value
// A(32u + 8q + e, m0 + lo) and the B value B(32u + 8q + e, n0 + lo); any permutation of k is
// a valid order for a sum as long as A and B agree, and this one lets an M-major A (an
// N-major B) be read as two float4 per lane.  The next group's operands are loaded (clamped, masked to zero
// past the chunk end) before the current group's MFMAs, so loads overlap the math with no
// branch in the loop.
#include <algorithm>

#include "regcn_internal.h"
#include "common.h"

namespace regcn {
namespace {

constexpr int KR_THR = 256;
constexpr int KR_TARGET_WG = 512;  // ~2 workgroups per CU
constexpr int KR_WAVES = 4;
constexpr int KR_TILE = 32;        // output tile per workgroup

constexpr int KG = 8;  // k per lane per group: a group covers 4 * KG = 32 k

// One operand's fragments for a group: o[i][e] = X(kk + e, idx[i]) (0 past kend).
// KM: X stored K-major (x[k * ld + r]); otherwise R-major (x[r * K + k]), read as float4
// when VEC (K % 4 == 0, 16-B aligned).  Past the chunk end the address is clamped (a valid
// read) and the value masked to zero, so the loop has no branch.
template <bool KM, bool VEC>
__device__ __forceinline__ void kr_operand(float (&o)[2][KG], const float* __restrict__ x, int64_t kk, int64_t kend,
                                           const int* idx, int64_t ld, int64_t K) {
  if (KM || !VEC) {
#pragma unroll
    for (int e = 0; e < KG; ++e) {
      const int64_t k = kk + e;
      const bool ok = k < kend;
      const int64_t kc = ok ? k : kend - 1;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float v = KM ? x[kc * ld + idx[i]] : x[(int64_t)idx[i] * K + kc];
        o[i][e] = ok ? v : 0.f;
      }
    }
  } else {
#pragma unroll
    for (int h = 0; h < KG / 4; ++h) {
      const int64_t kb = kk + 4 * h;  // a multiple of 4
      const int64_t kbc = kb < kend ? kb : ((kend - 1) & ~(int64_t)3);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f4 v = *reinterpret_cast<const f4*>(x + (int64_t)idx[i] * K + kbc);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[i][4 * h + e] = (kb + e < kend) ? v[e] : 0.f;
      }
    }
  }
}

struct KrOps {
  float a[2][KG];
  float b[2][KG];
};

// AK/BK: A (B) K-major: a[k * M + m] (b[k * N + n]); else M-major a[m * K + k] (N-major
// b[n * K + k]), float4 reads when AV (BV).
template <bool AK, bool AV, bool BK, bool BV>
__global__ __launch_bounds__(KR_THR) void k_kreduce(const float* __restrict__ a, const float* __restrict__ b,
                                                    int64_t K, int M, int N, int64_t chunk,
                                                    const float* __restrict__ c0, int64_t c0_ld, float* __restrict__ out) {
  __shared__ float red[KR_WAVES - 1][16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tiles_n = (N + KR_TILE - 1) / KR_TILE;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - tm * tiles_n;
  const int64_t kbeg = (int64_t)blockIdx.y * chunk;
  const int64_t kend = min(K, kbeg + chunk);
  const int mb = tm * KR_TILE, nb = tn * KR_TILE;
  const int lo = lane & 15, q = lane >> 4;
  int mrow[2], ncol[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    mrow[i] = min(mb + 16 * i + lo, M - 1);
    ncol[i] = min(nb + 16 * i + lo, N - 1);
  }
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // wave w takes the chunk's groups w, w + 4, ... (32 k each)
  constexpr int GK = 4 * KG, STRIDE = KR_WAVES * GK;
  KrOps cur, nxt;
  kr_operand<AK, AV>(cur.a, a, kbeg + w * GK + KG * q, kend, mrow, M, K);
  kr_operand<BK, BV>(cur.b, b, kbeg + w * GK + KG * q, kend, ncol, N, K);
  for (int64_t k0 = kbeg + w * GK; k0 < kend; k0 += STRIDE) {
    kr_operand<AK, AV>(nxt.a, a, k0 + STRIDE + KG * q, kend, mrow, M, K);
    kr_operand<BK, BV>(nxt.b, b, k0 + STRIDE + KG * q, kend, ncol, N, K);
#pragma unroll
    for (int e = 0; e < KG; ++e)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.a[i][e], cur.b[j][e], acc[i][j], 0, 0, 0);
    cur = nxt;
  }

  // the four waves' partial tiles summed in wave order (deterministic) through LDS
  if (w > 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[w - 1][(2 * i + j) * 4 + r][lane] = acc[i][j][r];
  }
  __syncthreads();
  if (w > 0) return;
#pragma unroll
  for (int u = 0; u < KR_WAVES - 1; ++u)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] += red[u][(2 * i + j) * 4 + r][lane];

  // C/D layout: lane l holds rows 4 (l >> 4) + r, column l & 15 of each 16 x 16 tile.
  float* dst = gridDim.y > 1 ? out + (int64_t)blockIdx.y * M * N : out;
  const bool add = gridDim.y == 1 && c0 != nullptr;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = nb + 16 * j + lo;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mb + 16 * i + 4 * q + r;
        if (m < M && n < N) {
          const float v = acc[i][j][r];
          dst[(int64_t)m * N + n] = add ? v + c0[m * c0_ld + n] : v;
        }
      }
    }
}

// out[m][n] = C0[m * c0_ld + n] + sum_s part[s][m][n], splits in order (deterministic);
// one element per thread, 8 split loads in flight.
__global__ __launch_bounds__(256) void k_kreduce_sum(const float* __restrict__ part, int nsplit, int64_t mn, int N,
                                                     const float* __restrict__ c0, int64_t c0_ld,
                                                     float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= mn) return;
  float s = c0 ? c0[(i / N) * c0_ld + i % N] : 0.f;
  int p = 0;
  for (; p + 8 <= nsplit; p += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(p + u) * mn + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; p < nsplit; ++p) s += part[(int64_t)p * mn + i];
  out[i] = s;
}

void kr_plan(int64_t K, int M, int N, int64_t* nsplit, int64_t* chunk) {
  const int64_t tiles = (int64_t)((M + KR_TILE - 1) / KR_TILE) * ((N + KR_TILE - 1) / KR_TILE);
  const int64_t groups = (K + 4 * KG - 1) / (4 * KG);
  int64_t ns = (KR_TARGET_WG + tiles - 1) / tiles;
  // at least 2 groups per wave (8 per workgroup) in a split: shorter K runs unsplit, its
  // four waves' partials reduced in LDS, with no second launch
  ns = std::min(ns, std::max<int64_t>(1, groups / (2 * KR_WAVES)));
  ns = std::max<int64_t>(1, ns);
  const int64_t gpc = std::max<int64_t>(1, (groups + ns - 1) / ns);
  *chunk = gpc * 4 * KG;
  *nsplit = std::max<int64_t>(1, (K + *chunk - 1) / *chunk);
}

}  // namespace

size_t kreduce_workspace_floats(int64_t K, int M, int N) {
  if (K <= 0 || M <= 0 || N <= 0) return 0;
  int64_t ns, chunk;
  kr_plan(K, M, N, &ns, &chunk);
  return ns > 1 ? (size_t)ns * M * N : 0;
}

template <bool AK, bool AV>
static void kr_launch_b(int b_mode, dim3 grid, hipStream_t st, const float* A, const float* B, int64_t K, int M, int N,
                        int64_t chunk, const float* C0, int64_t c0_ld, float* dst) {
  if (b_mode == 0)
    hipLaunchKernelGGL((k_kreduce<AK, AV, true, false>), grid, dim3(KR_THR), 0, st, A, B, K, M, N, chunk, C0, c0_ld, dst);
  else if (b_mode == 1)
    hipLaunchKernelGGL((k_kreduce<AK, AV, false, true>), grid, dim3(KR_THR), 0, st, A, B, K, M, N, chunk, C0, c0_ld, dst);
  else
    hipLaunchKernelGGL((k_kreduce<AK, AV, false, false>), grid, dim3(KR_THR), 0, st, A, B, K, M, N, chunk, C0, c0_ld, dst);
}

// layout mode of an operand: 0 K-major, 1 R-major with float4 reads, 2 R-major scalar
static int kr_mode(int kmajor, const float* p, int64_t K) {
  return kmajor ? 0 : ((K % 4 == 0 && ((uintptr_t)p & 15) == 0) ? 1 : 2);
}

int kreduce_gemm(const float* A, int a_kmajor, const float* B, int b_kmajor, int64_t K, int M, int N, const float* C0,
                 int64_t c0_ld, float* out, float* ws, hipStream_t st) {
  if (M <= 0 || N <= 0 || K < 0) return set_error(REGCN_EINVAL, "kreduce_gemm needs M, N > 0, K >= 0 (M=%d N=%d)", M, N);
  if ((int64_t)M * N > 0x7fffffffL) return set_error(REGCN_EINVAL, "kreduce_gemm needs M * N < 2^31");
  if (!out || (K > 0 && (!A || !B))) return set_error(REGCN_EINVAL, "null pointer");
  if (C0 && c0_ld < 0) return set_error(REGCN_EINVAL, "kreduce_gemm needs c0_ld >= 0");
  const int64_t mn = (int64_t)M * N;
  const dim3 sum_grid((unsigned)((mn + 255) / 256));
  if (K == 0) {  // empty sum: out = C0 (or zeros)
    hipLaunchKernelGGL(k_kreduce_sum, sum_grid, dim3(256), 0, st, (const float*)nullptr, 0, mn, N, C0, c0_ld, out);
    return check_launch("k_kreduce_sum");
  }
  int64_t ns, chunk;
  kr_plan(K, M, N, &ns, &chunk);
  if (ns > 1 && !ws) return set_error(REGCN_EINVAL, "kreduce_gemm needs a workspace of %zu floats",
                                      kreduce_workspace_floats(K, M, N));
  if (ns > 65535) return set_error(REGCN_EINVAL, "kreduce_gemm: too many K splits");
  const dim3 grid((unsigned)(((M + KR_TILE - 1) / KR_TILE) * ((N + KR_TILE - 1) / KR_TILE)), (unsigned)ns);
  float* dst = ns > 1 ? ws : out;
  const int am = kr_mode(a_kmajor, A, K), bm = kr_mode(b_kmajor, B, K);
  if (am == 0) kr_launch_b<true, false>(bm, grid, st, A, B, K, M, N, chunk, C0, c0_ld, dst);
  else if (am == 1) kr_launch_b<false, true>(bm, grid, st, A, B, K, M, N, chunk, C0, c0_ld, dst);
  else kr_launch_b<false, false>(bm, grid, st, A, B, K, M, N, chunk, C0, c0_ld, dst);
  int rc = check_launch("k_kreduce");
  if (rc || ns == 1) return rc;
  hipLaunchKernelGGL(k_kreduce_sum, sum_grid, dim3(256), 0, st, (const float*)ws, (int)ns, mn, N, C0, c0_ld, out);
  return check_launch("k_kreduce_sum");
}

}  // namespace regcn
