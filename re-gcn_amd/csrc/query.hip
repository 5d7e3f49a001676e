// Decoder query construction in one launch: everything
// between the final entity embedding and the all-entity scorer for the RotH decoders.
//
// RotH entity query (HyperbolicRotH._query, hyperbolic_decoder.py:1065-1085):
//   s = log0(project(E[s_i]));  s += fc2(relu(fc1(s)))         (reshape MLP, :1060-1063)
//   a = rot_proj(R[r_i]);  rot = exp0(givens(s, a));  t = exp0(trans_proj(R[r_i]))
//   q = mobius_add(project(rot), project(t))
// RotH relation query (HyperbolicRotHRel._query, hyperbolic_decoder.py:1223-1234):
//   s = log0(E[s_i]);  s += fc2(relu(fc1(s)));  rot = exp0(givens(s, global_rot))
//   q = mobius_add(-rot, E[o_i]);   and the candidates exp0(R) (:1243) in extra tiles.
// The (s, r, o) of query b come from the test triples: b < n_test reads trip[b],
// otherwise the inverse (o, r + num_rels, s) of trip[b - n_test] (hyperbolic_model.py:917),
// so the inverse triples never need to be materialised before the decoders.
//
// Each workgroup (4 waves) owns 16 queries and all d columns (rowtile.h): the four small
// GEMMs (fc1, fc2, rot_proj, trans_proj; nn.Linear weights packed transposed) run on fp32
// MFMA from LDS tiles, the row maps reduce across the waves through LDS.
#include "common.h"
#include "regcn_internal.h"
#include "rowtile.h"

namespace regcn {

__device__ __forceinline__ void add_bias(Frag& acc, const float* b, int d_out) {
  float bb[TPW];
  col_load(bb, b, d_out);
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc.t[j][r] += bb[j];
}

// Linear layer y = x W^T + b with packed W^T: acc from an LDS tile, plus the bias.
__device__ __forceinline__ void linear(Frag& acc, const float* T, int lda, const float* Wp, const float* b, int d,
                                       int d_out) {
  acc.zero();
  mfma_tile(acc, T, lda, Wp, d);
  add_bias(acc, b, d_out);
}

__device__ __forceinline__ void frag_to_tile(const Frag& a, float* T, int lda, int d) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float* row = T + frag_row(r) * lda;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int col = frag_col(j);
      if (col < d) row[col] = a.t[j][r];
    }
  }
}

// givens_rotation (hyperbolic_decoder.py:1032-1051): pairs (2k, 2k+1) rotated by angle k.
// A pair sits in adjacent lanes (columns 16j + l%16), so the partner is lane l ^ 1.
// Columns >= d (padding lanes) stay 0: their angle slot is never read.
template <typename AngleFn>
__device__ __forceinline__ void givens(Frag& x, int d, AngleFn angle) {
  const bool odd = threadIdx.x & 1;
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int col = frag_col(j);
    const bool ok = col < d;
    const int k2 = min(col, d - 1) >> 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = x.t[j][r];
      const float partner = __shfl_xor(v, 1);
      float si, co;
      sincosf(angle(r, k2), &si, &co);  // one shared range reduction
      const float y = odd ? (si * partner + co * v) : (co * v - si * partner);
      x.t[j][r] = ok ? y : 0.f;
    }
  }
}

// HyperbolicOps.mobius_add (hyperbolic_ops.py:118-143) + its final project, with the row
// norms x2 / y2 known: one reduction (<x, y>); the result's norm follows from them.
__device__ __forceinline__ void mobius_known(RowRed& rr, Frag& x, const float x2[4], const Frag& y, const float y2[4],
                                             const Curv& k) {
  float xy[4], n2[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < TPW; ++j) s += x.t[j][r] * y.t[j][r];
    xy[r] = s;
  }
  rr.allreduce(xy);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float A = 1.f + 2.f * k.c * xy[r] + k.c * y2[r];
    const float B = 1.f - k.c * x2[r];
    const float den = 1.f + 2.f * k.c * xy[r] + k.c * k.c * x2[r] * y2[r] + REGCN_EPS;
#pragma unroll
    for (int j = 0; j < TPW; ++j) x.t[j][r] = (A * x.t[j][r] + B * y.t[j][r]) / den;
    n2[r] = fmaxf(A * A * x2[r] + 2.f * A * B * xy[r] + B * B * y2[r], 0.f) / (den * den);
  }
  project_known(x, n2, k);
}

template <int MODE>  // 0: RotH entity query, 1: RotH relation query (+ exp0 candidates)
__global__ __launch_bounds__(NTHR) void k_query(QueryArgs p) {
  extern __shared__ float lds[];
  const int d = p.d, lda = tile_lda(d);
  float* T0 = lds;
  float* T1 = T0 + TM * lda;
  float* T2 = T1 + TM * lda;
  RowRed rr{T2 + TM * lda, 0};
  int* ids = reinterpret_cast<int*>(T2 + TM * lda + RED_FLOATS);  // s[16], r[16], o[16]
  const int n_qt = (p.B + TM - 1) / TM;

  if (MODE == 1 && (int)blockIdx.x >= n_qt) {  // candidate tiles: exp0(R)
    const int r0 = (blockIdx.x - n_qt) * TM;
    const int n = min(TM, p.n_cand - r0);
    if (threadIdx.x < TM) ids[threadIdx.x] = r0 + min((int)threadIdx.x, n - 1);
    __syncthreads();
    Frag c;
    frag_load(c, p.rel, ids, n, d);
    frag_exp0(rr, c, p.k);
    frag_store(c, p.cand_out, ids, n, d);
    return;
  }
  const int b0 = blockIdx.x * TM;
  const int nq = min(TM, p.B - b0);
  if (threadIdx.x < TM) {
    const int b = b0 + min((int)threadIdx.x, nq - 1);
    const bool inv = b >= p.n_test;
    const int64_t* t = p.trip + 3 * (int64_t)(inv ? b - p.n_test : b);
    ids[threadIdx.x] = (int)(inv ? t[2] : t[0]);
    ids[TM + threadIdx.x] = (int)t[1] + (inv ? p.num_rels : 0);
    ids[2 * TM + threadIdx.x] = (int)(inv ? t[0] : t[2]);
  }
  __syncthreads();
  const int* sid = ids;
  const int* rid = ids + TM;
  const int* oid = ids + 2 * TM;

  Frag s, o;
  float n2s[4], n2o[4];
  frag_load(s, p.ent, sid, nq, d);
  if (MODE == 1) {  // |E[s]|^2 and |E[o]|^2 in one barrier
    frag_load(o, p.ent, oid, nq, d);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        a += s.t[j][r] * s.t[j][r];
        b += o.t[j][r] * o.t[j][r];
      }
      n2s[r] = a;
      n2o[r] = b;
    }
    rr.allreduce2(n2s, n2o);
  } else {
    rr.sumsq(s, n2s);
    project_known(s, n2s, p.k);
  }
  log0_known(s, n2s, p.k);
  frag_to_tile(s, T0, lda, d);
  if (MODE == 0) stage_rows<false>(T1, lda, p.rel, rid, d, nq);
  __syncthreads();

  Frag h1, tr;
  if (MODE == 0) {  // fc1, trans_proj and rot_proj are independent: one k-loop, 3 x 4 chains
    Frag acc[3];
    const float* Ts[3] = {T0, T1, T1};
    const float* Ws[3] = {p.w1, p.wtr, p.wrot};
#pragma unroll
    for (int n = 0; n < 3; ++n) acc[n].zero();
    mfma_tiles<3, RING>(acc, Ts, Ws, lda, d);
    h1 = acc[0];
    tr = acc[1];
    add_bias(h1, p.b1, d);
    add_bias(tr, p.btr, d);
    add_bias(acc[2], p.brot, d / 2);
    frag_to_tile(acc[2], T2, lda, d / 2);
  } else {
    linear(h1, T0, lda, p.w1, p.b1, d, d);
  }
#pragma unroll
  for (int j = 0; j < TPW; ++j) h1.t[j] = f4{fmaxf(h1.t[j].x, 0.f), fmaxf(h1.t[j].y, 0.f), fmaxf(h1.t[j].z, 0.f),
                                           fmaxf(h1.t[j].w, 0.f)};
  __syncthreads();  // every wave is done reading T0
  frag_to_tile(h1, T0, lda, d);
  __syncthreads();
  Frag s2;
  linear(s2, T0, lda, p.w2, p.b2, d, d);
#pragma unroll
  for (int j = 0; j < TPW; ++j) s.t[j] += s2.t[j];

  if (MODE == 0) {
    givens(s, d, [&](int r, int k2) { return T2[frag_row(r) * lda + k2]; });
    float n2t[4];  // |rot|^2 and |trans|^2 in one barrier (a rotation keeps the norm)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        a += s.t[j][r] * s.t[j][r];
        b += tr.t[j][r] * tr.t[j][r];
      }
      n2s[r] = a;
      n2t[r] = b;
    }
    rr.allreduce2(n2s, n2t);
    exp0_known(s, n2s, p.k);
    project_known(s, n2s, p.k);
    exp0_known(tr, n2t, p.k);
    project_known(tr, n2t, p.k);
    mobius_known(rr, s, n2s, tr, n2t, p.k);
  } else {
    givens(s, d, [&](int, int k2) { return p.global_rot[k2]; });
    rr.sumsq(s, n2s);
    exp0_known(s, n2s, p.k);
#pragma unroll
    for (int j = 0; j < TPW; ++j) s.t[j] = -s.t[j];
    mobius_known(rr, s, n2s, o, n2o, p.k);
  }
  // store rows b0 .. b0 + nq - 1 (query order, not entity ids)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = frag_row(r);
    if (i >= nq) continue;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int col = frag_col(j);
      if (col < d) p.q_out[(int64_t)(b0 + i) * d + col] = s.t[j][r];
    }
  }
}

int query(const QueryArgs& a, int mode, hipStream_t st) {
  if (a.d <= 0 || a.d > MAX_D || (a.d & 3)) return set_error(REGCN_EINVAL, "query needs d %% 4 == 0, d <= 256");
  if (!a.ent || !a.trip || !a.w1 || !a.b1 || !a.w2 || !a.b2 || !a.q_out) return set_error(REGCN_EINVAL, "null pointer");
  if (a.n_test < 0 || a.B < 0 || a.B > 2 * a.n_test) return set_error(REGCN_EINVAL, "B must be <= 2 * n_test");
  if (mode == 0 && (!a.rel || !a.wrot || !a.brot || !a.wtr || !a.btr)) return set_error(REGCN_EINVAL, "RotH needs rel/rot/trans");
  if (mode == 1 && (!a.global_rot || (a.n_cand > 0 && (!a.rel || !a.cand_out))))
    return set_error(REGCN_EINVAL, "RotHRel needs global_rot and candidate buffers");
  if (mode != 0 && mode != 1) return set_error(REGCN_EINVAL, "unknown query mode %d", mode);
  const int n_qt = (a.B + TM - 1) / TM;
  const int n_ct = mode == 1 ? (a.n_cand + TM - 1) / TM : 0;
  if (n_qt + n_ct == 0) return 0;
  const size_t lds = (size_t)(3 * TM * tile_lda(a.d) + RED_FLOATS + 3 * TM) * 4;
  if (mode == 0)
    hipLaunchKernelGGL(k_query<0>, dim3(n_qt), dim3(NTHR), lds, st, a);
  else
    hipLaunchKernelGGL(k_query<1>, dim3(n_qt + n_ct), dim3(NTHR), lds, st, a);
  return check_launch("k_query");
}

}  // namespace regcn
