// The decoder front of one predict in one launch:
//   - RotH entity queries     (HyperbolicRotH._query, hyperbolic_decoder.py:1065-1085)
//   - RotHRel relation queries (HyperbolicRotHRel._query, hyperbolic_decoder.py:1223-1234)
//   - the relation scorer's candidates exp0(R) (:1243)
//   - the predict's all_triples = [test; inverse test] (hyperbolic_model.py:915-919)
// so the entity and relation decoders need no second stream and no torch glue.
//
// Tiles of 4 query rows on v_mfma_f32_4x4x1_16b_f32.  A query is a chain of small
// dependent GEMMs (d x d): on a 16-row tile (rowtile.h, query.hip) each takes ~3.5 us of one
// CU's fp32 MFMA issue (16x16x4: 32 cycles per SIMD per 2 kflop) and a predict has only
// B / 16 ~ 30 such tiles, so the chip idles while each tile runs its chain.  The 4x4x1 form
// issues 512 flop in 16 cycles: a 4-row GEMM is 200 x 16 cycles ~ 1.3 us per wave, and 4x
// as many workgroups share the chip.
//
// Layout: a workgroup = 4 waves = 4 rows x 256 columns.  Lane l of wave w holds column
// c = 64 w + l of all 4 rows (v[r], r = 0..3).  4x4x1_16b (tools/probe/mfma4_probe.hip):
// block b = l / 4 multiplies A rows 0..3 (A operand of lane 4b + r = A[r][k]) by columns
// 4b..4b+3 (B operand of lane l = B[k][l]); D register r of lane l = row r, column l.  So
// lane l supplies A[l & 3][k] and W[c][k], and receives row r of column c in register r.
// Weights are packed k4 (regcn_pack_k4_f32): Wq[g][c][e] = W[c][4g + e], 256 columns, so a
// wave's B operands for 4 k-steps are one coalesced 1 KB float4 load.
//
// Row reductions: the 4 per-row partials of a lane fold to one (row l & 3) by two quad
// transposition steps (DPP), then a 16-lane DPP ring sum, two xor shuffles and one LDS
// exchange across the waves; per-row scalar factors are evaluated once per lane for its
// own row and quad-broadcast (DPP) to the 4 rows each lane holds.
#include "common.h"
#include "regcn_internal.h"

namespace regcn {
namespace {

constexpr int QR = 4;         // query rows per workgroup
constexpr int QW = 4;         // waves per workgroup
constexpr int QT = 64 * QW;   // threads
constexpr int QCOLS = 64 * QW;  // columns covered (packed width)
constexpr int RB = 12;        // B k-groups in flight per chain (global)

__host__ __device__ inline int q4_lda(int d) { return d + 4; }  // 4 rows at distinct bank quads

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_no() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int R>
__device__ __forceinline__ float quad_bcast(float v) {  // lane (l & ~3) + R
  return dpp<R | (R << 2) | (R << 4) | (R << 6)>(v);
}
__device__ __forceinline__ void spread4(float own, float out[4]) {
  out[0] = quad_bcast<0>(own);
  out[1] = quad_bcast<1>(own);
  out[2] = quad_bcast<2>(own);
  out[3] = quad_bcast<3>(own);
}
// Sum over the wave of per-row partials s[0..3]; returns the total of row (l & 3).
__device__ __forceinline__ float wave_rows(const float s[4]) {
  const int l = lane_id();
  const bool h2 = l & 2, h1 = l & 1;
  const float send0 = h2 ? s[0] : s[2], send1 = h2 ? s[1] : s[3];
  const float keep0 = h2 ? s[2] : s[0], keep1 = h2 ? s[3] : s[1];
  const float u0 = keep0 + dpp<0x4E>(send0);  // quad_perm [2,3,0,1]: lane l ^ 2
  const float u1 = keep1 + dpp<0x4E>(send1);
  const float send = h1 ? u0 : u1, keep = h1 ? u1 : u0;
  float v = keep + dpp<0xB1>(send);  // quad_perm [1,0,3,2]: lane l ^ 1; row (l & 3), quad sum
  v += dpp<0x124>(v);                // row_ror:4 (same l & 3)
  v += dpp<0x128>(v);                // row_ror:8
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

// Cross-wave per-row sums through LDS (two buffers: one barrier per reduction).
struct Red4 {
  float* red;  // LDS: 2 buffers x 2 quantities x QW x QR
  int buf;
  __device__ __forceinline__ float own(const float s[4]) {
    const int l = lane_id(), w = wave_no();
    const float vs = wave_rows(s);
    float* b = red + buf * 2 * QW * QR;
    if (l < QR) b[w * QR + l] = vs;
    __syncthreads();
    const int r = l & 3;
    const float os = (b[r] + b[QR + r]) + (b[2 * QR + r] + b[3 * QR + r]);
    buf ^= 1;
    return os;
  }
  // totals of row (l & 3) of two quantities
  __device__ __forceinline__ void own2(const float s[4], const float t[4], float& os, float& ot) {
    const int l = lane_id(), w = wave_no();
    const float vs = wave_rows(s), vt = wave_rows(t);
    float* b = red + buf * 2 * QW * QR;
    if (l < QR) {
      b[w * QR + l] = vs;
      b[QW * QR + w * QR + l] = vt;
    }
    __syncthreads();
    const int r = l & 3;
    os = (b[r] + b[QR + r]) + (b[2 * QR + r] + b[3 * QR + r]);
    const float* bt = b + QW * QR;
    ot = (bt[r] + bt[QR + r]) + (bt[2 * QR + r] + bt[3 * QR + r]);
    buf ^= 1;
  }
};

__device__ __forceinline__ void sq4(const float v[4], float s[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) s[r] = v[r] * v[r];
}
__device__ __forceinline__ void scale4(float v[4], float own_f) {
  float f[4];
  spread4(own_f, f);
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] *= f[r];
}
// row maps with the row's |x|^2 known (n2: own row), as rowtile.h's *_known
__device__ __forceinline__ void project4(float v[4], float& n2, const Curv& k) {
  const float f = project_factor(n2, k);
  scale4(v, f);
  n2 *= f * f;
}
__device__ __forceinline__ void log04(float v[4], float& n2, const Curv& k) {
  const float f = log0_factor(n2, k);
  scale4(v, f);
  n2 *= f * f;
}
__device__ __forceinline__ void exp04(float v[4], float& n2, const Curv& k) {  // exp0 + project
  float o;
  const float f = exp0_factor(n2, k, &o);
  scale4(v, f);
  n2 = o;
}

// mobius_add(x, y) + project (hyperbolic_ops.py:118-143), |x|^2 and |y|^2 known.
__device__ __forceinline__ void mobius4(Red4& rr, float x[4], float& x2, const float y[4], float y2, const Curv& k) {
  float p[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) p[r] = x[r] * y[r];
  const float xy = rr.own(p);
  const float A = 1.f + 2.f * k.c * xy + k.c * y2;
  const float B = 1.f - k.c * x2;
  const float den = 1.f + 2.f * k.c * xy + k.c * k.c * x2 * y2 + REGCN_EPS;
  float fa[4], fb[4], fd[4];
  spread4(A, fa);
  spread4(B, fb);
  spread4(den, fd);
#pragma unroll
  for (int r = 0; r < 4; ++r) x[r] = (fa[r] * x[r] + fb[r] * y[r]) / fd[r];
  x2 = fmaxf(A * A * x2 + 2.f * A * B * xy + B * B * y2, 0.f) / (den * den);
  project4(x, x2, k);
}

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0); }

// acc[n] += A_n[4 x d_in] (LDS, stride lda) @ W_n^T (packed k4) for N chains in one k-loop.
// With one chain the k-steps alternate between two accumulators (no back-to-back dependent
// MFMA); they are added at the end.
template <int N>
__device__ __forceinline__ void gemm4(f4 (&acc)[N], const float* const (&A)[N], const float* const (&W)[N], int lda,
                                      int d_in) {
  const int l = lane_id();
  const int c = 64 * wave_no() + l;
  const int G = d_in >> 2;
  const f4* wp[N];
  const float* ap[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    wp[n] = reinterpret_cast<const f4*>(W[n]) + c;
    ap[n] = A[n] + (l & 3) * lda;
  }
  f4 acc2[N];
#pragma unroll
  for (int n = 0; n < N; ++n) acc2[n] = f4{0.f, 0.f, 0.f, 0.f};
  f4 br[N][RB];
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int n = 0; n < N; ++n) br[n][i] = wp[n][(int64_t)min(i, G - 1) * QCOLS];
  // A operands one k-group ahead (LDS latency under the previous group's MFMAs)
  f4 ar[N][2];
#pragma unroll
  for (int n = 0; n < N; ++n) ar[n][0] = *reinterpret_cast<const f4*>(ap[n]);
  auto step = [&](int g, int i) {  // i: ring slot (RB even: slot parity = group parity)
#pragma unroll
    for (int n = 0; n < N; ++n) ar[n][(i + 1) & 1] = *reinterpret_cast<const f4*>(ap[n] + 4 * min(g + 1, G - 1));
    const int pa = i & 1;
    if (N == 1) {
      acc[0] = mfma4(ar[0][pa].x, br[0][i].x, acc[0]);
      acc2[0] = mfma4(ar[0][pa].z, br[0][i].z, acc2[0]);
      acc[0] = mfma4(ar[0][pa].y, br[0][i].y, acc[0]);
      acc2[0] = mfma4(ar[0][pa].w, br[0][i].w, acc2[0]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int n = 0; n < N; ++n) acc[n] = mfma4(ar[n][pa][e], br[n][i][e], acc[n]);
    }
  };
  int g = 0;
  for (; g + RB <= G; g += RB) {
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      step(g + i, i);
      __builtin_amdgcn_sched_barrier(0);
      const int nx = min(g + i + RB, G - 1);
#pragma unroll
      for (int n = 0; n < N; ++n) br[n][i] = wp[n][(int64_t)nx * QCOLS];  // unconditional: countable
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int i = 0; i < RB; ++i)
    if (g + i < G) step(g + i, i);
  if (N == 1) acc[0] += acc2[0];
}

__device__ __forceinline__ float colv(const float* p, int c, int n) { return c < n ? p[c] : 0.f; }

// 4 rows of a row-major matrix at column c (0 past d)
__device__ __forceinline__ void load_rows4(float v[4], const float* M, const int* ids, int c, int d) {
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = c < d ? M[(int64_t)ids[r] * d + c] : 0.f;
}
__device__ __forceinline__ void to_lds4(float* T, int lda, const float v[4], int c, int d) {
  if (c < d) {
#pragma unroll
    for (int r = 0; r < 4; ++r) T[r * lda + c] = v[r];
  }
}

// givens_rotation (hyperbolic_decoder.py:1032-1051): pairs (2k, 2k+1) are columns c, c ^ 1,
// i.e. lanes l, l ^ 1; angle k = c >> 1.
template <typename AngleFn>
__device__ __forceinline__ void givens4(float v[4], int c, int d, AngleFn angle) {
  const bool odd = c & 1, ok = c < d;
  const int k2 = min(c, d - 1) >> 1;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float x = v[r];
    const float partner = dpp<0xB1>(x);
    float si, co;
    sincosf(angle(r, k2), &si, &co);
    const float y = odd ? (si * partner + co * x) : (co * x - si * partner);
    v[r] = ok ? y : 0.f;
  }
}

__global__ __launch_bounds__(QT) void k_queries4(regcn_roth_queries_desc p, Curv k) {
  extern __shared__ float lds[];
  const int d = p.d, lda = q4_lda(d);
  float* S0 = lds;               // 4 x lda: the MLP input rows
  float* T1 = S0 + QR * lda;     // relation rows (entity tiles), fc1 output
  float* T2 = T1 + QR * lda;     // fc1 output (entity tiles) / angles
  Red4 rr{T2 + QR * lda, 0};
  int* ids = reinterpret_cast<int*>(T2 + QR * lda + 4 * QW * QR);  // s[4], r[4], o[4]
  const int l = lane_id(), c = 64 * wave_no() + l;
  const int n_qt = (p.B + QR - 1) / QR;
  const int n_ent = p.q_ent ? n_qt : 0, n_rel = p.q_rel ? n_qt : 0;
  int blk = blockIdx.x;
  const int kind = blk < n_ent ? 0 : blk < n_ent + n_rel ? 1 : 2;
  blk -= kind == 0 ? 0 : kind == 1 ? n_ent : n_ent + n_rel;

  if (kind == 2) {  // relation candidates: exp0(R) rows
    const int r0 = blk * QR;
    const int n = min(QR, p.n_cand - r0);
    int rid[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) rid[r] = r0 + min(r, n - 1);
    float v[4], s[4];
    load_rows4(v, p.rel, rid, c, d);
    sq4(v, s);
    float n2 = rr.own(s);
    exp04(v, n2, k);
    if (c < d) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r < n) p.cand[(int64_t)(r0 + r) * d + c] = v[r];
    }
    return;
  }
  const int b0 = blk * QR;
  const int nq = min(QR, p.B - b0);
  if (threadIdx.x < QR) {
    const int b = b0 + min((int)threadIdx.x, nq - 1);
    const bool inv = b >= p.n_test;
    const int64_t* t = p.trip + 3 * (int64_t)(inv ? b - p.n_test : b);
    const int64_t s = inv ? t[2] : t[0], rl = t[1] + (inv ? p.num_rels : 0), o = inv ? t[0] : t[2];
    ids[threadIdx.x] = (int)s;
    ids[QR + threadIdx.x] = (int)rl;
    ids[2 * QR + threadIdx.x] = (int)o;
    if (kind == 0 && p.all_triples && (int)threadIdx.x < nq) {
      int64_t* at = p.all_triples + 3 * (int64_t)b;
      at[0] = s;
      at[1] = rl;
      at[2] = o;
    }
  }
  __syncthreads();
  int sid[4], rid[4], oid[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    sid[r] = ids[r];
    rid[r] = ids[QR + r];
    oid[r] = ids[2 * QR + r];
  }
  float v[4], s[4];
  load_rows4(v, p.ent, sid, c, d);
  const bool ent = kind == 0;
  float o[4], n2 = 0.f, n2o = 0.f;
  if (ent) {  // s_tan = log0(project(E[s])); relation rows for rot_proj / trans_proj
    float rl[4];
    load_rows4(rl, p.rel, rid, c, d);
    to_lds4(T1, lda, rl, c, d);
    sq4(v, s);
    n2 = rr.own(s);
    project4(v, n2, k);
  } else {  // s_tan = log0(E[s]); |E[o]|^2 for the final mobius_add
    load_rows4(o, p.ent, oid, c, d);
    float t[4];
    sq4(v, s);
    sq4(o, t);
    rr.own2(s, t, n2, n2o);
  }
  log04(v, n2, k);
  to_lds4(S0, lda, v, c, d);
  __syncthreads();

  // reshape MLP: s_tan + fc2(relu(fc1(s_tan))); RotH: rot_proj and trans_proj of the
  // relation rows in the same k-loop as fc1
  float tr[4] = {0.f, 0.f, 0.f, 0.f};
  f4 h1;
  if (ent) {
    f4 acc[3] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const float* const As[3] = {S0, T1, T1};
    const float* const Ws[3] = {p.w1, p.w_trans, p.w_rot};
    gemm4<3>(acc, As, Ws, lda, d);
    h1 = acc[0];
    const float bt = colv(p.b_trans, c, d), brt = colv(p.b_rot, c, d / 2);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      tr[r] = c < d ? acc[1][r] + bt : 0.f;
      if (c < d / 2) T2[r * lda + c] = acc[2][r] + brt;  // angles
    }
  } else {
    f4 acc[1] = {{0.f, 0.f, 0.f, 0.f}};
    const float* const As[1] = {S0};
    const float* const Ws[1] = {p.rw1};
    gemm4<1>(acc, As, Ws, lda, d);
    h1 = acc[0];
  }
  const float b1 = colv(ent ? p.b1 : p.rb1, c, d);
  float* H = T1;    // relu(fc1) rows; entity tiles: over the relation rows
  __syncthreads();  // every wave is done reading the fc1 operands
  {
    float hv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) hv[r] = fmaxf(h1[r] + b1, 0.f);
    to_lds4(H, lda, hv, c, d);
  }
  __syncthreads();
  {
    f4 acc[1] = {{0.f, 0.f, 0.f, 0.f}};
    const float* const As[1] = {H};
    const float* const Ws[1] = {ent ? p.w2 : p.rw2};
    gemm4<1>(acc, As, Ws, lda, d);
    const float b2 = colv(ent ? p.b2 : p.rb2, c, d);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = c < d ? v[r] + (acc[0][r] + b2) : 0.f;
  }
  if (ent) {
    givens4(v, c, d, [&](int r, int k2) { return T2[r * lda + k2]; });
    float a[4], b[4];  // |rot|^2 and |trans|^2 in one barrier (a rotation keeps the norm)
    sq4(v, a);
    sq4(tr, b);
    float n2t;
    rr.own2(a, b, n2, n2t);
    exp04(v, n2, k);
    project4(v, n2, k);
    exp04(tr, n2t, k);
    project4(tr, n2t, k);
    mobius4(rr, v, n2, tr, n2t, k);
  } else {
    givens4(v, c, d, [&](int, int k2) { return p.global_rot[k2]; });
    sq4(v, s);
    n2 = rr.own(s);
    exp04(v, n2, k);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = -v[r];
    mobius4(rr, v, n2, o, n2o, k);
  }
  float* out = ent ? p.q_ent : p.q_rel;
  if (c < d) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r < nq) out[(int64_t)(b0 + r) * d + c] = v[r];
  }
}

// Wq[g][c][e] = W[c][4g + e] (c < n_out), 0 for n_out <= c < QCOLS.
__global__ void k_pack_k4(const float* __restrict__ W, int n_out, int n_in, float* __restrict__ out) {
  const int64_t n = (int64_t)(n_in / 4) * QCOLS;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(i / QCOLS), c = (int)(i % QCOLS);
    f4 v = {0.f, 0.f, 0.f, 0.f};
    if (c < n_out) v = *reinterpret_cast<const f4*>(W + (int64_t)c * n_in + 4 * g);
    reinterpret_cast<f4*>(out)[i] = v;
  }
}

}  // namespace

size_t packed_k4_floats(int n_out, int n_in) { return (size_t)(n_in / 4) * QCOLS * 4; }

int pack_k4(const float* W, int n_out, int n_in, float* out, hipStream_t st) {
  if (!W || !out) return set_error(REGCN_EINVAL, "null pointer");
  if (n_out <= 0 || n_out > QCOLS || n_in <= 0 || (n_in & 3))
    return set_error(REGCN_EINVAL, "k4 packing needs 0 < n_out <= %d and n_in %% 4 == 0", QCOLS);
  const int64_t n = (int64_t)(n_in / 4) * QCOLS;
  hipLaunchKernelGGL(k_pack_k4, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0, st, W, n_out,
                     n_in, out);
  return check_launch("k_pack_k4");
}

int roth_queries(const regcn_roth_queries_desc& a, hipStream_t st) {
  const int d = a.d;
  if (d <= 0 || d > QCOLS || (d & 3)) return set_error(REGCN_EINVAL, "queries need d %% 4 == 0, d <= %d", QCOLS);
  if (a.B < 0 || a.n_test < 0 || a.B > 2 * a.n_test) return set_error(REGCN_EINVAL, "B must be <= 2 * n_test");
  if (a.n_cand < 0 || (a.n_cand && (!a.rel || !a.cand))) return set_error(REGCN_EINVAL, "candidates need rel and cand");
  if ((a.q_ent || a.q_rel || a.all_triples) && a.B && (!a.ent || !a.trip)) return set_error(REGCN_EINVAL, "null pointer");
  if (a.q_ent && (!a.rel || !a.w1 || !a.b1 || !a.w2 || !a.b2 || !a.w_rot || !a.b_rot || !a.w_trans || !a.b_trans))
    return set_error(REGCN_EINVAL, "RotH queries need rel, fc1/fc2, rot_proj, trans_proj");
  if (a.q_rel && (!a.rw1 || !a.rb1 || !a.rw2 || !a.rb2 || !a.global_rot))
    return set_error(REGCN_EINVAL, "RotHRel queries need fc1/fc2 and global_rot");
  if (a.all_triples && !a.q_ent) return set_error(REGCN_EINVAL, "all_triples is written by the entity query tiles");
  const int n_qt = (a.B + QR - 1) / QR;
  const int grid = (a.q_ent ? n_qt : 0) + (a.q_rel ? n_qt : 0) + (a.n_cand + QR - 1) / QR;
  if (!grid) return 0;
  const size_t lds = (size_t)(3 * QR * q4_lda(d) + 4 * QW * QR + 3 * QR) * 4;
  hipLaunchKernelGGL(k_queries4, dim3(grid), dim3(QT), lds, st, a, make_curv(a.c));
  return check_launch("k_queries4");
}

}  // namespace regcn
