// Snapshot construction on the device (§8(a) row a1).
//
// Replaces the per-snapshot host build of rgcn/utils.py:78-134 (build_sub_graph + r2e) and
// the work lists of regcn_amd/graph.py.  Everything is integer work bound by HBM traffic and
// launch latency: no MFMA.  Building blocks:
//
//  * exclusive scan over [n][NC] int32 records (NC independent prefix sums per pass):
//    block partial sums -> one-workgroup scan of the block sums -> block-local scan + add;
//  * stable LSD radix sort of 32-bit keys (+ optional 32-bit values), 8-bit digits:
//    per-block digit histograms, scanned digit-major (so a digit's blocks are contiguous),
//    then a scatter that ranks each block's 4096 items in LDS in index order (wave ballot
//    match on the 8 digit bits + per-wave digit counts) and writes each digit's run of the
//    block contiguously.  Stability is what keeps the reference's edge order within a
//    destination row (DGL's in-edge order = edge-id order);
//  * one generic chunker that cuts spans {row, begin, length} into chunk / fix-up records in
//    exactly the host's order (graph.py _chunk_rows / _chunk_spans / group_fixups).
//
// Integer atomics are used only for counts (histograms, in-degrees): results are
// bitwise identical run to run and to the host build.
#include <algorithm>

#include "common.h"
#include "gather.h"
#include "regcn_internal.h"

namespace regcn {
namespace {

constexpr int BT = 256;                 // threads per block everywhere in this file
constexpr int SC_IPT = 8;               // scan: items per thread
constexpr int SC_TILE = BT * SC_IPT;    // 2048 records per block
constexpr int RX_IPT = 16;              // radix scatter: items per thread
constexpr int RX_TILE = BT * RX_IPT;    // 4096 items per block
constexpr int NCOL = 5;                 // chunker record: nchunk, slotted, groups, nonbig, big
constexpr int FIX_GROUP = 64;           // graph.py FIX_GROUP

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o);
    if (l >= o) v += t;
  }
  return v;
}

// Exclusive scan of one int per thread over the 256-thread block; *total = block sum.
__device__ __forceinline__ int block_excl_scan(int v, int* lds, int* total) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int inc = wave_incl_scan(v);
  if (l == 63) lds[w] = inc;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int s = lds[i];
    off += i < w ? s : 0;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return off + inc - v;
}

// Sum over the block, wave-reduced first (one LDS slot per wave).
__device__ __forceinline__ int block_sum(int v, int* lds) {
  int t;
  block_excl_scan(v, lds, &t);
  return t;
}

__device__ __forceinline__ int div_up(int a, int b) { return (a + b - 1) / b; }

// ------------------------------------------------------------------------------- scan
template <int NC>
__global__ __launch_bounds__(BT) void k_scan_up(const int* __restrict__ in, int n, int* __restrict__ bsum) {
  __shared__ int lds[4];
  const int base = blockIdx.x * SC_TILE + threadIdx.x * SC_IPT;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < SC_IPT; ++i)
      if (base + i < n) s += in[(int64_t)(base + i) * NC + c];
    const int tot = block_sum(s, lds);
    if (threadIdx.x == 0) bsum[blockIdx.x * NC + c] = tot;
  }
}

// One workgroup: exclusive scan of the nb block sums (in place) and the grand totals.
template <int NC>
__global__ __launch_bounds__(BT) void k_scan_mid(int* __restrict__ bsum, int nb, int* __restrict__ total) {
  __shared__ int lds[4];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    int carry = 0;
    for (int b0 = 0; b0 < nb; b0 += BT) {
      const int i = b0 + threadIdx.x;
      const int v = i < nb ? bsum[i * NC + c] : 0;
      int tot;
      const int ex = block_excl_scan(v, lds, &tot);
      if (i < nb) bsum[i * NC + c] = carry + ex;
      carry += tot;
    }
    if (threadIdx.x == 0 && total) total[c] = carry;
  }
}

// Block-local scan plus the block's offset; in == out is allowed (each thread reads its
// records before writing them).
template <int NC>
__global__ __launch_bounds__(BT) void k_scan_down(const int* in, int n, const int* __restrict__ bsum, int* out) {
  __shared__ int lds[4];
  const int base = blockIdx.x * SC_TILE + threadIdx.x * SC_IPT;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    int v[SC_IPT];
    int s = 0;
#pragma unroll
    for (int i = 0; i < SC_IPT; ++i) {
      v[i] = base + i < n ? in[(int64_t)(base + i) * NC + c] : 0;
      s += v[i];
    }
    int tot;
    int run = bsum[blockIdx.x * NC + c] + block_excl_scan(s, lds, &tot);
#pragma unroll
    for (int i = 0; i < SC_IPT; ++i) {
      if (base + i < n) out[(int64_t)(base + i) * NC + c] = run;
      run += v[i];
    }
  }
}

__global__ void k_zero_ints(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0;
}

// ------------------------------------------------------------------------- radix sort
__global__ __launch_bounds__(BT) void k_radix_hist(const uint32_t* __restrict__ keys, int n, int shift, int nb,
                                                   int* __restrict__ hist) {
  __shared__ int h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int base = blockIdx.x * RX_TILE;
  uint32_t k[RX_IPT];
#pragma unroll
  for (int r = 0; r < RX_IPT; ++r) {
    const int idx = base + r * BT + threadIdx.x;
    k[r] = idx < n ? keys[idx] : 0u;
  }
#pragma unroll
  for (int r = 0; r < RX_IPT; ++r)
    if (base + r * BT + (int)threadIdx.x < n) atomicAdd(&h[(k[r] >> shift) & 255u], 1);
  __syncthreads();
  hist[threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

// offs: digit-major exclusive scan of the histograms, 256 * nb + 1 entries (the last one is
// the total), so a block's count of digit g is offs[g*nb + b + 1] - offs[g*nb + b].
template <bool VALS>
__global__ __launch_bounds__(BT) void k_radix_scatter(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                      int n, int shift, int nb, const int* __restrict__ offs,
                                                      uint32_t* __restrict__ kout, uint32_t* __restrict__ vout) {
  __shared__ uint32_t lk[RX_TILE];
  __shared__ uint32_t lv[VALS ? RX_TILE : 1];
  __shared__ int gofs[256], lstart[256], run[256], wc[4][256], red[4];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, b = blockIdx.x;
  const int base = b * RX_TILE;
  uint32_t key[RX_IPT], val[RX_IPT];
#pragma unroll
  for (int r = 0; r < RX_IPT; ++r) {  // all loads first: 16 (32) independent loads in flight
    const int idx = base + r * BT + tid;
    key[r] = idx < n ? kin[idx] : 0u;
    val[r] = (VALS && idx < n) ? vin[idx] : 0u;
  }
  const int o = offs[tid * nb + b];
  const int cnt = offs[tid * nb + b + 1] - o;
  gofs[tid] = o;
  int tot;
  const int ls = block_excl_scan(cnt, red, &tot);
  lstart[tid] = ls;
  run[tid] = ls;
#pragma unroll
  for (int i = 0; i < 4; ++i) wc[i][tid] = 0;
  __syncthreads();
  const uint64_t below = l == 0 ? 0ull : (~0ull >> (64 - l));
  for (int r = 0; r < RX_IPT; ++r) {  // rounds in index order: stable
    const bool valid = base + r * BT + tid < n;
    const uint32_t dig = (key[r] >> shift) & 255u;
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const bool on = (dig >> bit) & 1u;
      const uint64_t bb = __ballot(on);
      m &= on ? bb : ~bb;
    }
    const int rank = __popcll(m & below);
    if (valid && rank == 0) wc[w][dig] = __popcll(m);
    __syncthreads();
    if (valid) {
      int pos = run[dig] + rank;
      for (int i = 0; i < w; ++i) pos += wc[i][dig];
      lk[pos] = key[r];
      if (VALS) lv[pos] = val[r];
    }
    __syncthreads();
    run[tid] += (wc[0][tid] + wc[1][tid]) + (wc[2][tid] + wc[3][tid]);
    wc[0][tid] = wc[1][tid] = wc[2][tid] = wc[3][tid] = 0;
    __syncthreads();
  }
  const int nvalid = min(RX_TILE, n - base);
  for (int j = tid; j < nvalid; j += BT) {  // each digit's run of the block is contiguous
    const uint32_t k = lk[j];
    const int dig = (k >> shift) & 255u;
    const int g = gofs[dig] + (j - lstart[dig]);
    kout[g] = k;
    if (VALS) vout[g] = lv[j];
  }
}

// ------------------------------------------------------------------------- call 1 kernels
struct Tri {
  int s, r, o;
};

__device__ __forceinline__ Tri load_tri(const int64_t* __restrict__ tr, int t) {
  return Tri{(int)tr[3 * (int64_t)t], (int)tr[3 * (int64_t)t + 1], (int)tr[3 * (int64_t)t + 2]};
}

// Edges in the reference order (utils.py:116-118): e < T: s -> o, type r; e >= T: o -> s,
// type r + R.  Keys for the destination sort, edge types, r2e pairs.  (In-degrees come from
// the sorted keys, k_bounds: Zipf hubs made per-edge atomics on in_deg the slowest part.)
__global__ __launch_bounds__(BT) void k_expand(const int64_t* __restrict__ tr, int T, int V, int R,
                                               uint32_t* __restrict__ key, uint32_t* __restrict__ val,
                                               int64_t* __restrict__ etype,
                                               uint32_t* __restrict__ pkey, int* __restrict__ stats) {
  const int E = 2 * T;
  for (int e = blockIdx.x * BT + threadIdx.x; e < E; e += gridDim.x * BT) {
    const bool fwd = e < T;
    const int t = fwd ? e : e - T;
    Tri x = load_tri(tr, t);
    const int64_t s64 = tr[3 * (int64_t)t], r64 = tr[3 * (int64_t)t + 1], o64 = tr[3 * (int64_t)t + 2];
    if (s64 < 0 || s64 >= V || o64 < 0 || o64 >= V || r64 < 0 || r64 >= R) {
      if (fwd) atomicAdd(&stats[REGCN_SNAP_INVALID], 1);
      x = Tri{0, 0, 0};  // keep the build in bounds; the caller rejects it
    }
    const int dst = fwd ? x.o : x.s;
    key[e] = (uint32_t)dst;
    val[e] = (uint32_t)e;
    if (etype) etype[e] = fwd ? x.r : x.r + R;
    pkey[e] = (uint32_t)x.r * (uint32_t)V + (uint32_t)(fwd ? x.s : x.o);  // (rel, entity) of r2e
  }
}

__global__ __launch_bounds__(BT) void k_csr_cols(const int64_t* __restrict__ tr, int T, int R, int V,
                                                 const uint32_t* __restrict__ eid, int* __restrict__ col_src,
                                                 int* __restrict__ col_type) {
  const int E = 2 * T;
  for (int i = blockIdx.x * BT + threadIdx.x; i < E; i += gridDim.x * BT) {
    const int e = (int)eid[i];
    const bool fwd = e < T;
    Tri x = load_tri(tr, fwd ? e : e - T);
    if (x.s < 0 || x.s >= V || x.o < 0 || x.o >= V || x.r < 0 || x.r >= R) x = Tri{0, 0, 0};
    col_src[i] = fwd ? x.s : x.o;
    col_type[i] = fwd ? x.r : x.r + R;
  }
}

// Segment starts of sorted keys: ptr[k] = first i with key[i] >= k, for k in [0, nkeys];
// item i writes the starts of the keys in (key[i-1], key[i]], the last item those after it.
// n items (n_dev: device count, else n).  ptr[nkeys] = n.
__global__ __launch_bounds__(BT) void k_bounds(const uint32_t* __restrict__ key, int n, const int* __restrict__ n_dev,
                                               uint32_t div, int nkeys, int* __restrict__ ptr) {
  const int i = blockIdx.x * BT + threadIdx.x;
  const int m = n_dev ? *n_dev : n;
  if (i >= m) return;
  const int k = (int)(key[i] / div);
  const int kp = i == 0 ? -1 : (int)(key[i - 1] / div);
  for (int j = kp + 1; j <= k; ++j) ptr[j] = i;
  if (i == m - 1)
    for (int j = k + 1; j <= nkeys; ++j) ptr[j] = m;
}

// in_deg from the CSR row pointers, norm = 1 / in_deg with 0 -> 1 (utils.py:110-114), max
// in-degree, rows with in-edges.
__global__ __launch_bounds__(BT) void k_degrees(const int* __restrict__ rowptr, int V, int* __restrict__ in_deg,
                                                float* __restrict__ norm, int* __restrict__ stats) {
  __shared__ int lds[4];
  const int v = blockIdx.x * BT + threadIdx.x;
  const int deg = v < V ? rowptr[v + 1] - rowptr[v] : 0;
  if (v < V) in_deg[v] = deg;
  if (v < V) norm[v] = 1.0f / (float)(deg == 0 ? 1 : deg);
  int mx = deg;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
  const int pos = block_sum(deg > 0 ? 1 : 0, lds);
  if ((threadIdx.x & 63) == 0) atomicMax(&stats[REGCN_SNAP_MAX_DEG], mx);
  if (threadIdx.x == 0 && pos) atomicAdd(&stats[REGCN_SNAP_N_POS], pos);
}

// edata['norm'] = norm[dst] * norm[src] in the reference edge order (utils.py:124).
__global__ __launch_bounds__(BT) void k_edge_norm(const int64_t* __restrict__ tr, int T, int V,
                                                  const float* __restrict__ norm, float* __restrict__ en) {
  const int E = 2 * T;
  for (int e = blockIdx.x * BT + threadIdx.x; e < E; e += gridDim.x * BT) {
    const bool fwd = e < T;
    Tri x = load_tri(tr, fwd ? e : e - T);
    if (x.s < 0 || x.s >= V || x.o < 0 || x.o >= V) x = Tri{0, 0, 0};
    const int src = fwd ? x.s : x.o, dst = fwd ? x.o : x.s;
    en[e] = norm[dst] * norm[src];
  }
}

__global__ __launch_bounds__(BT) void k_uniq_flag(const uint32_t* __restrict__ k, int n, int* __restrict__ flag) {
  const int i = blockIdx.x * BT + threadIdx.x;
  if (i < n) flag[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

// Unique (rel, entity) pairs in key order = each relation's entity set ascending (np.unique),
// written twice: forward spans, then the inverse relations' copies (utils.py:88-96).
__global__ __launch_bounds__(BT) void k_uniq_emit(const uint32_t* __restrict__ k, int n, int V,
                                                  const int* __restrict__ pos, const int* __restrict__ n_pairs,
                                                  int* __restrict__ rel_idx, uint32_t* __restrict__ ukey) {
  const int i = blockIdx.x * BT + threadIdx.x;
  if (i >= n) return;
  if (i > 0 && k[i] == k[i - 1]) return;
  const int p = pos[i];
  const int ent = (int)(k[i] % (uint32_t)V);
  rel_idx[p] = ent;
  rel_idx[*n_pairs + p] = ent;
  ukey[p] = k[i];
}

// off[r]: first unique pair of relation r (k_bounds over the unique keys / V), off[R] = pairs.
__global__ __launch_bounds__(BT) void k_rel_lists(const int* __restrict__ off, int R, const int* __restrict__ n_pairs,
                                                  int* __restrict__ cnt, int* __restrict__ rel_start,
                                                  float* __restrict__ rel_count, int* __restrict__ stats) {
  const int r = blockIdx.x * BT + threadIdx.x;
  if (r >= 2 * R) return;
  const int b = r < R ? r : r - R;
  const int c = off[b + 1] - off[b];
  if (r < R) cnt[r] = c;
  rel_start[r] = c ? off[b] + (r < R ? 0 : *n_pairs) : 0;
  rel_count[r] = (float)c;
  if (r < R && c) atomicMax(&stats[REGCN_SNAP_REL_MAX], c);
}

// ------------------------------------------------------------------------- call 2 kernels
// Row order (graph.py fused_work): rows with in-edges by descending in-degree, ties by node id
// (a stable ascending sort of kmax - 1 - deg), then the zero-in-degree rows (key kmax).
__global__ __launch_bounds__(BT) void k_row_keys(const int* __restrict__ in_deg, int V, uint32_t kmax,
                                                 uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
  const int v = blockIdx.x * BT + threadIdx.x;
  if (v >= V) return;
  const int deg = in_deg[v];
  key[v] = deg == 0 ? kmax : kmax - 1u - (uint32_t)deg;
  val[v] = (uint32_t)v;
}

// inl[i] = inline edges of the i-th positive row (0 for heavy rows over the budget).
__global__ __launch_bounds__(BT) void k_inline(const int* __restrict__ in_deg, const int* __restrict__ rows, int V,
                                               int budget, int* __restrict__ inl, int* __restrict__ stats) {
  __shared__ int lds[4];
  const int i = blockIdx.x * BT + threadIdx.x;
  const int n_pos = stats[REGCN_SNAP_N_POS];
  int deg = 0;
  if (i < n_pos) deg = in_deg[rows[i]];
  if (i < V) inl[i] = deg > budget ? 0 : deg;
  const int heavy = block_sum(deg > budget ? 1 : 0, lds);
  if (threadIdx.x == 0 && heavy) atomicAdd(&stats[REGCN_SNAP_N_HEAVY], heavy);
}

// Number of rows a greedy tile starting at row a takes (graph.py _pack_tiles):
// max(1, min(16, #{j in 1..n-a : cs[a+j] - cs[a] <= P})).
__device__ __forceinline__ int tile_rows(const int* __restrict__ cs, int a, int n, int P) {
  const int lim = min(16, n - a);
  const int c0 = cs[a];
  int cnt = 0;
  for (int j = 1; j <= lim; ++j) cnt += (cs[a + j] - c0 <= P) ? 1 : 0;  // cs is non-decreasing
  return max(1, cnt);
}

// a* = the first row >= n_heavy whose 16-row window fits P.  Past the heavy prefix inl is
// non-increasing, so every later window fits too and the tiles from there on are regular.
__global__ __launch_bounds__(BT) void k_astar(const int* __restrict__ cs, int V, int P, int* __restrict__ stats) {
  const int a = blockIdx.x * BT + threadIdx.x;
  const int n = stats[REGCN_SNAP_N_POS], nh = stats[REGCN_SNAP_N_HEAVY];
  if (a < nh || a >= n || a >= V) return;
  const bool fits = cs[min(a + 16, n)] - cs[a] <= P;
  const bool prev = a > nh && (cs[min(a + 15, n)] - cs[a - 1] <= P);
  if (fits && !prev) atomicMin(&stats[REGCN_SNAP_A_STAR], a);
}

__global__ __launch_bounds__(BT) void k_walk_cnt(const int* __restrict__ cs, int V, int P,
                                                 const int* __restrict__ stats, int* __restrict__ cnt) {
  const int a = blockIdx.x * BT + threadIdx.x;
  const int n = stats[REGCN_SNAP_N_POS], astar = stats[REGCN_SNAP_A_STAR];
  if (a >= V || a >= astar || a >= n) return;
  cnt[a] = tile_rows(cs, a, n, P);
}

// The sequential greedy prefix [0, a*): one wave walks the tile chain, 64 rows of counts
// per register window (the next window's load issued while the current one is walked).
__global__ __launch_bounds__(64) void k_walk(const int* __restrict__ cnt, int* __restrict__ tiles,
                                             int* __restrict__ item_ptr, int* __restrict__ stats) {
  const int lane = threadIdx.x;
  const int n = stats[REGCN_SNAP_N_POS];
  const int astar = min(stats[REGCN_SNAP_A_STAR], n);
  int a = 0, t = 0, base = 0;
  int cur = lane < astar ? cnt[lane] : 1;
  int nxt = 64 + lane < astar ? cnt[64 + lane] : 1;
  while (a < astar) {
    while (a - base >= 64) {
      base += 64;
      cur = nxt;
      nxt = base + 64 + lane < astar ? cnt[base + 64 + lane] : 1;
    }
    const int c = __builtin_amdgcn_readlane(cur, a - base);
    if (lane == 0) {
      tiles[2 * t] = a;
      tiles[2 * t + 1] = c;
    }
    ++t;
    a += c;
  }
  if (lane == 0) {
    stats[REGCN_SNAP_WALK_TILES] = t;
    stats[REGCN_SNAP_A_STAR] = a;  // where the regular tiles start
    stats[REGCN_SNAP_N_TILES] = t + (a < n ? div_up(n - a, 16) : 0);
    item_ptr[0] = 0;
  }
}

__global__ __launch_bounds__(BT) void k_tiles_fill(const int* __restrict__ cs, int V, const int* __restrict__ stats,
                                                   int* __restrict__ tiles, int* __restrict__ item_ptr,
                                                   int* __restrict__ local) {
  const int t = blockIdx.x * BT + threadIdx.x;
  const int nt = stats[REGCN_SNAP_N_TILES], tw = stats[REGCN_SNAP_WALK_TILES];
  const int n = stats[REGCN_SNAP_N_POS], a_end = stats[REGCN_SNAP_A_STAR];
  if (t >= nt || t >= V) return;
  int start, count;
  if (t < tw) {
    start = tiles[2 * t];
    count = tiles[2 * t + 1];
  } else {
    start = a_end + 16 * (t - tw);
    count = min(16, n - start);
    tiles[2 * t] = start;
    tiles[2 * t + 1] = count;
  }
  for (int i = 0; i < count; ++i) local[start + i] = i;
  item_ptr[t + 1] = cs[start + count];
}

// Per-tile items (graph.py fused_work): one wave per positive row copies its inline in-edges.
__global__ __launch_bounds__(BT) void k_items(const int* __restrict__ rows, const int* __restrict__ rowptr,
                                              const int* __restrict__ col_src, const int* __restrict__ col_type,
                                              const int* __restrict__ inl, const int* __restrict__ cs,
                                              const int* __restrict__ local, int V, const int* __restrict__ stats,
                                              int* __restrict__ item_src, int* __restrict__ item_tl) {
  const int lane = threadIdx.x & 63;
  const int n = stats[REGCN_SNAP_N_POS];
  const int nw = gridDim.x * (BT / 64);
  for (int i = blockIdx.x * (BT / 64) + (threadIdx.x >> 6); i < n && i < V; i += nw) {
    const int m = inl[i];
    if (m == 0) continue;
    const int f = cs[i], rp = rowptr[rows[i]], loc = local[i];
    for (int k = lane; k < m; k += 64) {
      item_src[f + k] = col_src[rp + k];
      item_tl[f + k] = (col_type[rp + k] << 4) | loc;
    }
  }
}

// ----------------------------------------------------------------------------- chunker
// Spans: mode 0 all rows (row i, CSR span), mode 1 heavy rows (row rows[i], CSR span,
// i < stats[N_HEAVY]), mode 2 relations (r in [0, 2R): r_to_e span).
struct Spans {
  int mode, n_cap, R;
  const int* beg;    // rowptr | rowptr | rel_start
  const int* len;    // in_deg | in_deg | rel_ent_count (index r mod R)
  const int* rows;   // mode 1
  const int* n_dev;  // mode 1: stats + N_HEAVY
};

__device__ __forceinline__ bool span_at(const Spans& s, int i, int& row, int& beg, int& len) {
  if (i >= s.n_cap || (s.n_dev && i >= *s.n_dev)) return false;
  if (s.mode == 0) {
    row = i;
    beg = s.beg[i];
    len = s.len[i];
  } else if (s.mode == 1) {
    row = s.rows[i];
    beg = s.beg[row];
    len = s.len[row];
  } else {
    row = i;
    beg = s.beg[i];
    len = s.len[i < s.R ? i : i - s.R];
  }
  return true;
}

struct SpanCounts {
  int nch, slotted, ng, nonbig, big;
};

__device__ __forceinline__ SpanCounts span_counts(int len, int C) {
  SpanCounts k;
  k.nch = div_up(len, C);
  const bool multi = k.nch > 1;
  k.slotted = multi ? k.nch : 0;
  k.ng = (multi && k.nch > FIX_GROUP) ? div_up(k.nch, FIX_GROUP) : 0;
  k.nonbig = (multi && k.ng == 0) ? 1 : 0;
  k.big = k.ng > 0 ? 1 : 0;
  return k;
}

__global__ __launch_bounds__(BT) void k_chunk_count(Spans s, int C, int* __restrict__ cols) {
  const int i = blockIdx.x * BT + threadIdx.x;
  if (i >= s.n_cap) return;
  int row, beg, len = 0;
  SpanCounts k = {0, 0, 0, 0, 0};
  if (span_at(s, i, row, beg, len)) k = span_counts(len, C);
  int* c = cols + (int64_t)i * NCOL;
  c[0] = k.nch;
  c[1] = k.slotted;
  c[2] = k.ng;
  c[3] = k.nonbig;
  c[4] = k.big;
}

// graph.py _chunk_rows + group_fixups order: chunks in span order; fix-ups = [first-level
// groups of the big spans, the other multi-chunk spans, the big spans' final fix-ups];
// group slots are numbered after all chunk slots.
__global__ __launch_bounds__(BT) void k_chunk_emit(Spans s, int C, const int* __restrict__ sc,
                                                   const int* __restrict__ tot, int4* __restrict__ chunks,
                                                   int4* __restrict__ fixups, int* __restrict__ st) {
  const int i = blockIdx.x * BT + threadIdx.x;
  const int NSLOTC = tot[1], G = tot[2], NB = tot[3], NBIG = tot[4];
  if (i == 0) {
    st[0] = tot[0];
    st[1] = G + NB + NBIG;
    st[2] = NSLOTC + G;
  }
  int row, beg, len;
  if (!span_at(s, i, row, beg, len) || len == 0) return;
  const SpanCounts k = span_counts(len, C);
  const int* o = sc + (int64_t)i * NCOL;
  const int co = o[0], so = o[1], gpos = o[2], nbpos = o[3], fpos = o[4];
  const bool multi = k.nch > 1;
  for (int j = 0; j < k.nch; ++j)
    chunks[co + j] = int4{row, beg + j * C, min(beg + (j + 1) * C, beg + len), multi ? so + j : -1};
  if (!multi) return;
  if (k.big) {
    for (int g = 0; g < k.ng; ++g)
      fixups[gpos + g] = int4{0, so + FIX_GROUP * g, min(so + FIX_GROUP * (g + 1), so + k.nch), NSLOTC + gpos + g + 1};
    fixups[G + NB + fpos] = int4{row, NSLOTC + gpos, NSLOTC + gpos + k.ng, 0};
  } else {
    fixups[G + nbpos] = int4{row, so, so + k.nch, 0};
  }
}

// ---------------------------------------------------------------------------- host side
inline unsigned blocks(int64_t n, int per = BT) {
  const int64_t b = (n + per - 1) / per;
  return (unsigned)(b < 1 ? 1 : b);
}

inline int bitlen(uint64_t x) {
  int b = 0;
  while (x) {
    ++b;
    x >>= 1;
  }
  return b;
}

inline int d2d(void* dst, const void* src, size_t bytes, hipStream_t st) {
  const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st);
  return e == hipSuccess ? 0 : set_error((int)e, "hipMemcpyAsync: %s", hipGetErrorString(e));
}

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

struct Layout {
  int64_t nmax, nb_rx, hist_n, bsum_n, cols_n;
  size_t k0, v0, k1, v1, hist, bsum, tot, flag, cs, inl, cnt, local, cols, roff, total;
};

Layout layout(int64_t T, int V, int R) {
  Layout L;
  const int64_t E = 2 * T;
  L.nmax = std::max<int64_t>({E, (int64_t)V, 2 * (int64_t)R, 1});
  L.nb_rx = (L.nmax + RX_TILE - 1) / RX_TILE;
  L.hist_n = 256 * L.nb_rx + 1;
  L.cols_n = std::max<int64_t>(V, 2 * (int64_t)R) + 1;
  const int64_t scan_n = std::max<int64_t>({L.hist_n, L.nmax + 1, L.cols_n * NCOL});
  L.bsum_n = ((scan_n + SC_TILE - 1) / SC_TILE + 1) * NCOL;
  size_t off = 0;
  auto take = [&](int64_t n_ints) {
    const size_t o = off;
    off += align_up((size_t)n_ints * 4);
    return o;
  };
  L.k0 = take(L.nmax);
  L.v0 = take(L.nmax);
  L.k1 = take(L.nmax);
  L.v1 = take(L.nmax);
  L.hist = take(L.hist_n);
  L.bsum = take(L.bsum_n);
  L.tot = take(8);
  L.flag = take(L.nmax + 1);
  L.cs = take((int64_t)V + 1);
  L.inl = take(V + 1);
  L.cnt = take(V + 1);
  L.local = take(V + 1);
  L.cols = take(L.cols_n * NCOL);
  L.roff = take((int64_t)R + 1);
  L.total = off;
  return L;
}

template <int NC>
int scan_excl(const int* in, int* out, int64_t n, int* total, int* bsum, hipStream_t st) {
  if (n <= 0) {
    if (total) hipLaunchKernelGGL(k_zero_ints, dim3(1), dim3(64), 0, st, total, NC);
    return check_launch("k_zero_ints");
  }
  const int nb = (int)((n + SC_TILE - 1) / SC_TILE);
  hipLaunchKernelGGL(k_scan_up<NC>, dim3(nb), dim3(BT), 0, st, in, (int)n, bsum);
  hipLaunchKernelGGL(k_scan_mid<NC>, dim3(1), dim3(BT), 0, st, bsum, nb, total);
  hipLaunchKernelGGL(k_scan_down<NC>, dim3(nb), dim3(BT), 0, st, in, (int)n, bsum, out);
  return check_launch("scan");
}

// Stable sort of (k0, v0) by the low `bits` key bits; returns which buffer pair holds the result.
int radix_sort(char* ws, const Layout& L, int64_t n, int bits, bool vals, bool* in_second, hipStream_t st) {
  uint32_t* k[2] = {(uint32_t*)(ws + L.k0), (uint32_t*)(ws + L.k1)};
  uint32_t* v[2] = {(uint32_t*)(ws + L.v0), (uint32_t*)(ws + L.v1)};
  int* hist = (int*)(ws + L.hist);
  int* bsum = (int*)(ws + L.bsum);
  int cur = 0;
  if (n > 0) {
    const int nb = (int)((n + RX_TILE - 1) / RX_TILE);
    for (int shift = 0; shift < bits; shift += 8) {
      hipLaunchKernelGGL(k_radix_hist, dim3(nb), dim3(BT), 0, st, k[cur], (int)n, shift, nb, hist);
      int rc = scan_excl<1>(hist, hist, 256 * (int64_t)nb, hist + 256 * (int64_t)nb, bsum, st);
      if (rc) return rc;
      if (vals)
        hipLaunchKernelGGL(k_radix_scatter<true>, dim3(nb), dim3(BT), 0, st, k[cur], v[cur], (int)n, shift, nb,
                           hist, k[cur ^ 1], v[cur ^ 1]);
      else
        hipLaunchKernelGGL(k_radix_scatter<false>, dim3(nb), dim3(BT), 0, st, k[cur], v[cur], (int)n, shift, nb,
                           hist, k[cur ^ 1], v[cur ^ 1]);
      rc = check_launch("k_radix_scatter");
      if (rc) return rc;
      cur ^= 1;
    }
  }
  *in_second = cur == 1;
  return 0;
}

int check_desc(const regcn_snapshot_desc* d, bool second) {
  if (!d) return set_error(REGCN_EINVAL, "null snapshot descriptor");
  if (d->T < 0 || d->V <= 0 || d->R <= 0) return set_error(REGCN_EINVAL, "bad snapshot sizes T=%lld V=%d R=%d",
                                                          (long long)d->T, d->V, d->R);
  if (2 * d->T >= (int64_t)INT32_MAX - RX_TILE) return set_error(REGCN_ENOTSUP, "snapshot too large for int32 edge ids");
  if ((uint64_t)d->V * (uint64_t)d->R > 0xFFFFFFFFull)
    return set_error(REGCN_ENOTSUP, "V * R >= 2^32 (r2e pair keys are 32-bit)");
  if ((int64_t)2 * d->R >= (1 << 27)) return set_error(REGCN_ENOTSUP, "relation ids must be < 2^27");
  if (!d->workspace || d->ws_bytes < layout(d->T, d->V, d->R).total)
    return set_error(REGCN_EINVAL, "snapshot workspace too small");
  if (!d->stats) return set_error(REGCN_EINVAL, "null stats");
  if (!second) {
    if ((d->T > 0 && !d->triples) || !d->in_deg || !d->rowptr || !d->col_src || !d->col_type || !d->norm ||
        !d->rel_ent_count || !d->rel_idx || !d->rel_start || !d->rel_count)
      return set_error(REGCN_EINVAL, "null snapshot output");
  } else {
    if (d->budget < 1 || d->pack_items < 1 || d->chunk_edges < 1) return set_error(REGCN_EINVAL, "bad work-list parameters");
    if (!d->rows || !d->tiles || !d->item_ptr || !d->item_src || !d->item_tl || !d->chunks || !d->fixups ||
        !d->heavy_chunks || !d->heavy_fixups || !d->rel_chunks || !d->rel_fixups)
      return set_error(REGCN_EINVAL, "null work-list output");
  }
  return 0;
}

}  // namespace

int snapshot_csr(const regcn_snapshot_desc* d, hipStream_t st) {
  int rc = check_desc(d, false);
  if (rc) return rc;
  const int T = (int)d->T, V = d->V, R = d->R, E = 2 * T;
  const Layout L = layout(d->T, V, R);
  char* ws = (char*)d->workspace;
  int* bsum = (int*)(ws + L.bsum);
  hipLaunchKernelGGL(k_zero_ints, dim3(1), dim3(64), 0, st, d->stats, REGCN_SNAP_NSTATS);
  if ((rc = check_launch("zero"))) return rc;
  const unsigned gE = std::min<unsigned>(blocks(E), 65536);
  // edges: destination keys, in-degrees, edge types, r2e pairs (pairs go to the second key
  // buffer; the destination sort runs first on the first pair of buffers)
  uint32_t* pairs = (uint32_t*)(ws + L.flag);  // scratch until the pair sort
  if (E > 0) {
    hipLaunchKernelGGL(k_expand, dim3(gE), dim3(BT), 0, st, d->triples, T, V, R, (uint32_t*)(ws + L.k0),
                       (uint32_t*)(ws + L.v0), d->edge_type, pairs, d->stats);
    if ((rc = check_launch("k_expand"))) return rc;
  }
  bool second;
  if ((rc = radix_sort(ws, L, E, bitlen((uint64_t)V - 1), true, &second, st))) return rc;
  if (E > 0)
    hipLaunchKernelGGL(k_bounds, dim3(blocks(E)), dim3(BT), 0, st, (const uint32_t*)(ws + (second ? L.k1 : L.k0)), E,
                       nullptr, 1u, V, d->rowptr);
  else
    hipLaunchKernelGGL(k_zero_ints, dim3(blocks(V + 1)), dim3(BT), 0, st, d->rowptr, V + 1);
  hipLaunchKernelGGL(k_degrees, dim3(blocks(V)), dim3(BT), 0, st, d->rowptr, V, d->in_deg, d->norm, d->stats);
  if ((rc = check_launch("k_degrees"))) return rc;
  if (E > 0) {
    const uint32_t* eid = (const uint32_t*)(ws + (second ? L.v1 : L.v0));
    hipLaunchKernelGGL(k_csr_cols, dim3(gE), dim3(BT), 0, st, d->triples, T, R, V, eid, d->col_src, d->col_type);
    if (d->edge_norm) hipLaunchKernelGGL(k_edge_norm, dim3(gE), dim3(BT), 0, st, d->triples, T, V, d->norm, d->edge_norm);
    if ((rc = check_launch("k_csr_cols"))) return rc;
  }
  // r2e: sort the (rel, entity) pair keys, keep the unique ones
  int* roff = (int*)(ws + L.roff);
  if (E > 0) {
    if ((rc = d2d(ws + L.k0, pairs, (size_t)E * 4, st))) return rc;
    if ((rc = radix_sort(ws, L, E, bitlen((uint64_t)V * (uint64_t)R - 1), false, &second, st))) return rc;
    const uint32_t* pk = (const uint32_t*)(ws + (second ? L.k1 : L.k0));
    int* flag = (int*)(ws + L.flag);
    hipLaunchKernelGGL(k_uniq_flag, dim3(blocks(E)), dim3(BT), 0, st, pk, E, flag);
    if ((rc = scan_excl<1>(flag, flag, E, d->stats + REGCN_SNAP_N_PAIRS, bsum, st))) return rc;
    uint32_t* ukey = (uint32_t*)(ws + (second ? L.k0 : L.k1));  // the other key buffer
    hipLaunchKernelGGL(k_uniq_emit, dim3(blocks(E)), dim3(BT), 0, st, pk, E, V, flag, d->stats + REGCN_SNAP_N_PAIRS,
                       d->rel_idx, ukey);
    hipLaunchKernelGGL(k_bounds, dim3(blocks(E)), dim3(BT), 0, st, ukey, E, d->stats + REGCN_SNAP_N_PAIRS,
                       (uint32_t)V, R, roff);
    if ((rc = check_launch("k_uniq_emit"))) return rc;
  } else {
    hipLaunchKernelGGL(k_zero_ints, dim3(blocks(R + 1)), dim3(BT), 0, st, roff, R + 1);
  }
  hipLaunchKernelGGL(k_rel_lists, dim3(blocks(2 * R)), dim3(BT), 0, st, roff, R, d->stats + REGCN_SNAP_N_PAIRS,
                     d->rel_ent_count, d->rel_start, d->rel_count, d->stats);
  return check_launch("k_rel_lists");
}

static int chunker(const Spans& s, int C, char* ws, const Layout& L, int4* chunks, int4* fixups, int* st3,
                   hipStream_t st) {
  int* cols = (int*)(ws + L.cols);
  int* tot = (int*)(ws + L.tot);
  hipLaunchKernelGGL(k_chunk_count, dim3(blocks(s.n_cap)), dim3(BT), 0, st, s, C, cols);
  int rc = check_launch("k_chunk_count");
  if (rc) return rc;
  if ((rc = scan_excl<NCOL>(cols, cols, s.n_cap, tot, (int*)(ws + L.bsum), st))) return rc;
  hipLaunchKernelGGL(k_chunk_emit, dim3(blocks(s.n_cap)), dim3(BT), 0, st, s, C, cols, tot, chunks, fixups, st3);
  return check_launch("k_chunk_emit");
}

int snapshot_work(const regcn_snapshot_desc* d, hipStream_t st) {
  int rc = check_desc(d, true);
  if (rc) return rc;
  const int V = d->V, R = d->R;
  const int64_t E = 2 * d->T;
  const Layout L = layout(d->T, V, R);
  char* ws = (char*)d->workspace;
  int* stats = d->stats;
  int* bsum = (int*)(ws + L.bsum);
  // rows: stable sort by (kmax - 1 - deg), zero rows last
  const uint32_t kmax = (uint32_t)((1ull << bitlen((uint64_t)E + 1)) - 1);
  hipLaunchKernelGGL(k_row_keys, dim3(blocks(V)), dim3(BT), 0, st, d->in_deg, V, kmax, (uint32_t*)(ws + L.k0),
                     (uint32_t*)(ws + L.v0));
  if ((rc = check_launch("k_row_keys"))) return rc;
  bool second;
  if ((rc = radix_sort(ws, L, V, bitlen(kmax), true, &second, st))) return rc;
  if ((rc = d2d(d->rows, ws + (second ? L.v1 : L.v0), (size_t)V * 4, st))) return rc;
  // tiles over the positive rows
  int* inl = (int*)(ws + L.inl);
  int* cs = (int*)(ws + L.cs);
  int* cnt = (int*)(ws + L.cnt);
  int* local = (int*)(ws + L.local);
  hipLaunchKernelGGL(k_zero_ints, dim3(1), dim3(64), 0, st, stats + REGCN_SNAP_N_HEAVY, REGCN_SNAP_NSTATS - REGCN_SNAP_N_HEAVY);
  hipLaunchKernelGGL(k_inline, dim3(blocks(V)), dim3(BT), 0, st, d->in_deg, d->rows, V, d->budget, inl, stats);
  if ((rc = check_launch("k_inline"))) return rc;
  if ((rc = scan_excl<1>(inl, cs, V, cs + V, bsum, st))) return rc;
  if ((rc = d2d(stats + REGCN_SNAP_N_ITEMS, cs + V, 4, st))) return rc;
  if ((rc = d2d(stats + REGCN_SNAP_A_STAR, stats + REGCN_SNAP_N_POS, 4, st))) return rc;
  hipLaunchKernelGGL(k_astar, dim3(blocks(V)), dim3(BT), 0, st, cs, V, d->pack_items, stats);
  hipLaunchKernelGGL(k_walk_cnt, dim3(blocks(V)), dim3(BT), 0, st, cs, V, d->pack_items, stats, cnt);
  hipLaunchKernelGGL(k_walk, dim3(1), dim3(64), 0, st, cnt, d->tiles, d->item_ptr, stats);
  hipLaunchKernelGGL(k_tiles_fill, dim3(blocks(V)), dim3(BT), 0, st, cs, V, stats, d->tiles, d->item_ptr, local);
  if ((rc = check_launch("tiles"))) return rc;
  hipLaunchKernelGGL(k_items, dim3(std::min<unsigned>(blocks(V, 4), 65536)), dim3(BT), 0, st, d->rows, d->rowptr,
                     d->col_src, d->col_type, inl, cs, local, V, stats, d->item_src, d->item_tl);
  if ((rc = check_launch("k_items"))) return rc;
  // chunk lists: heavy rows, all rows, relation spans
  const int C = d->chunk_edges;
  Spans heavy{1, V, R, d->rowptr, d->in_deg, d->rows, stats + REGCN_SNAP_N_HEAVY};
  if ((rc = chunker(heavy, C, ws, L, (int4*)d->heavy_chunks, (int4*)d->heavy_fixups, stats + REGCN_SNAP_HEAVY_CHUNKS, st)))
    return rc;
  Spans all{0, V, R, d->rowptr, d->in_deg, nullptr, nullptr};
  if ((rc = chunker(all, C, ws, L, (int4*)d->chunks, (int4*)d->fixups, stats + REGCN_SNAP_CHUNKS, st))) return rc;
  // forward relations only: an inverse id's span holds the same entities in the same order
  // (rgcn/utils.py:88-89), so its mean is a copy of the forward one (regcn_segment_mean_f32 callers)
  Spans rel{2, R, R, d->rel_start, d->rel_ent_count, nullptr, nullptr};
  return chunker(rel, C, ws, L, (int4*)d->rel_chunks, (int4*)d->rel_fixups, stats + REGCN_SNAP_REL_CHUNKS, st);
}

size_t snapshot_ws_bytes(int64_t T, int V, int R) { return layout(T, V, R).total; }

// ------------------------------------------------------------------- transposed edge lists
namespace {
__global__ __launch_bounds__(BT) void k_iota_keys(const int* __restrict__ keys, int n, uint32_t* __restrict__ k,
                                                  uint32_t* __restrict__ v) {
  const int i = blockIdx.x * BT + threadIdx.x;
  if (i < n) {
    k[i] = (uint32_t)keys[i];
    v[i] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(BT) void k_csr_dst(const int* __restrict__ rowptr, int V, int* __restrict__ csr_dst) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (BT / 64);
  for (int v = blockIdx.x * (BT / 64) + (threadIdx.x >> 6); v < V; v += nw)
    for (int p = rowptr[v] + lane; p < rowptr[v + 1]; p += 64) csr_dst[p] = v;
}

Layout tlayout(int E, int V, int R2) { return layout(((int64_t)E + 1) / 2, V, (R2 + 1) / 2); }
}  // namespace

size_t transpose_ws_bytes(int E, int V, int R2) { return tlayout(E, V, R2).total; }

int snapshot_transpose(const regcn_transpose_desc* d, hipStream_t st) {
  if (!d) return set_error(REGCN_EINVAL, "null transpose descriptor");
  const int V = d->V, E = d->E, R2 = d->R2;
  if (V <= 0 || E < 0 || R2 <= 0) return set_error(REGCN_EINVAL, "bad transpose sizes");
  if (!d->rowptr || !d->csr_dst || !d->sptr || !d->tptr || (E > 0 && (!d->col_src || !d->col_type || !d->sp || !d->tp)))
    return set_error(REGCN_EINVAL, "null pointer");
  const Layout L = tlayout(E, V, R2);
  if (!d->workspace || d->ws_bytes < L.total) return set_error(REGCN_EINVAL, "transpose workspace too small");
  char* ws = (char*)d->workspace;
  int rc;
  hipLaunchKernelGGL(k_csr_dst, dim3(std::min<unsigned>(blocks(V, 4), 65536)), dim3(BT), 0, st, d->rowptr, V, d->csr_dst);
  if ((rc = check_launch("k_csr_dst"))) return rc;
  const int* keys[2] = {d->col_src, d->col_type};
  int* ptr[2] = {d->sptr, d->tptr};
  int* pos[2] = {d->sp, d->tp};
  const int nkeys[2] = {V, R2};
  for (int w = 0; w < 2; ++w) {
    if (E == 0) {
      hipLaunchKernelGGL(k_zero_ints, dim3(blocks(nkeys[w] + 1)), dim3(BT), 0, st, ptr[w], nkeys[w] + 1);
      if ((rc = check_launch("k_zero_ints"))) return rc;
      continue;
    }
    hipLaunchKernelGGL(k_iota_keys, dim3(blocks(E)), dim3(BT), 0, st, keys[w], E, (uint32_t*)(ws + L.k0),
                       (uint32_t*)(ws + L.v0));
    bool second;
    if ((rc = radix_sort(ws, L, E, bitlen((uint64_t)nkeys[w] - 1), true, &second, st))) return rc;
    hipLaunchKernelGGL(k_bounds, dim3(blocks(E)), dim3(BT), 0, st, (const uint32_t*)(ws + (second ? L.k1 : L.k0)), E,
                       nullptr, 1u, nkeys[w], ptr[w]);
    if ((rc = d2d(pos[w], ws + (second ? L.v1 : L.v0), (size_t)E * 4, st))) return rc;
  }
  return 0;
}

// ------------------------------------------------------------------- row / type edge order
namespace {
// keys of the second (row) pass: the destination of each type-sorted CSR position
__global__ __launch_bounds__(BT) void k_row_of(const int* __restrict__ csr_dst, const uint32_t* __restrict__ pin,
                                               int n, uint32_t* __restrict__ k, uint32_t* __restrict__ v) {
  const int i = blockIdx.x * BT + threadIdx.x;
  if (i < n) {
    const uint32_t p = pin[i];
    k[i] = (uint32_t)csr_dst[p];
    v[i] = p;
  }
}

__global__ __launch_bounds__(BT) void k_permute2(const uint32_t* __restrict__ perm, int n, const int* __restrict__ a,
                                                 const int* __restrict__ b, int* __restrict__ oa, int* __restrict__ ob) {
  const int i = blockIdx.x * BT + threadIdx.x;
  if (i < n) {
    const uint32_t p = perm[i];
    oa[i] = a[p];
    ob[i] = b[p];
  }
}
}  // namespace

size_t row_type_ws_bytes(int E, int V, int R2) {
  return tlayout(E, V, R2).total + align_up((size_t)std::max(E, 1) * 4);
}

// Stable LSD radix sort by type, then stably by destination row: CSR positions in (row,
// type, position) order.
int row_type_order(int V, int E, int R2, const int* rowptr, const int* col_src, const int* col_type, int* out_src,
                   int* out_type, void* workspace, size_t ws_bytes, hipStream_t st) {
  if (V <= 0 || E < 0 || R2 <= 0) return set_error(REGCN_EINVAL, "bad row/type order sizes");
  if (E == 0) return 0;
  if (!rowptr || !col_src || !col_type || !out_src || !out_type) return set_error(REGCN_EINVAL, "null pointer");
  if (!workspace || ws_bytes < row_type_ws_bytes(E, V, R2))
    return set_error(REGCN_EINVAL, "row/type order workspace too small");
  const Layout L = tlayout(E, V, R2);
  char* ws = (char*)workspace;
  int* csr_dst = (int*)(ws + L.total);
  int rc;
  hipLaunchKernelGGL(k_csr_dst, dim3(std::min<unsigned>(blocks(V, 4), 65536)), dim3(BT), 0, st, rowptr, V, csr_dst);
  if ((rc = check_launch("k_csr_dst"))) return rc;
  hipLaunchKernelGGL(k_iota_keys, dim3(blocks(E)), dim3(BT), 0, st, col_type, E, (uint32_t*)(ws + L.k0),
                     (uint32_t*)(ws + L.v0));
  bool second;
  if ((rc = radix_sort(ws, L, E, bitlen((uint64_t)R2 - 1), true, &second, st))) return rc;
  hipLaunchKernelGGL(k_row_of, dim3(blocks(E)), dim3(BT), 0, st, csr_dst,
                     (const uint32_t*)(ws + (second ? L.v1 : L.v0)), E, (uint32_t*)(ws + L.k0),
                     (uint32_t*)(ws + L.v0));
  if ((rc = check_launch("k_row_of"))) return rc;
  if ((rc = radix_sort(ws, L, E, bitlen((uint64_t)V - 1), true, &second, st))) return rc;
  hipLaunchKernelGGL(k_permute2, dim3(blocks(E)), dim3(BT), 0, st, (const uint32_t*)(ws + (second ? L.v1 : L.v0)), E,
                     col_src, col_type, out_src, out_type);
  return check_launch("k_permute2");
}

// ----------------------------------------------------------------- row / source edge order
namespace {
__global__ __launch_bounds__(BT) void k_permute1(const uint32_t* __restrict__ perm, int n, const int* __restrict__ a,
                                                 int* __restrict__ oa) {
  const int i = blockIdx.x * BT + threadIdx.x;
  if (i < n) oa[i] = a[perm[i]];
}
}  // namespace

size_t row_src_ws_bytes(int E, int V) { return row_type_ws_bytes(E, V, 2); }

namespace {
// per item: its row's position in rows[] (tile start + tile-local row), one wave per tile
__global__ __launch_bounds__(BT) void k_item_rowpos(const int* __restrict__ tiles, const int* __restrict__ item_ptr,
                                                    const int* __restrict__ item_tl, int n_tiles,
                                                    int* __restrict__ rowpos) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (BT / 64);
  for (int t = blockIdx.x * (BT / 64) + (threadIdx.x >> 6); t < n_tiles; t += nw)
    for (int i = item_ptr[t] + lane; i < item_ptr[t + 1]; i += 64) rowpos[i] = tiles[2 * t] + (item_tl[i] & 15);
}
}  // namespace

size_t item_src_ws_bytes(int n_items, int V) { return row_type_ws_bytes(n_items, V, 2); }

// Stable LSD radix sort of the items by a key, then stably by row position: each row's items in
// ascending key order (ties keep CSR order), rows and tiles unchanged.  by_type = 0: the key is
// the source id (a row's duplicate sources adjacent, regcn_layer_desc.item_src_runs); 1: the
// item_tl word (type << 4 | local row; within a row: the relation type), a row's same-type
// items adjacent (regcn_layer_desc.item_crel: their weights summed per (row, type)).
static int item_order(int V, int key_bits, int by_type, int n_tiles, int n_items, const int* tiles,
                      const int* item_ptr, const int* item_src, const int* item_tl, int* out_src, int* out_tl,
                      void* workspace, size_t ws_bytes, hipStream_t st) {
  if (V <= 0 || n_tiles < 0 || n_items < 0) return set_error(REGCN_EINVAL, "bad item order sizes");
  if (n_items == 0) return 0;
  if (!tiles || !item_ptr || !item_src || !item_tl || !out_src || !out_tl) return set_error(REGCN_EINVAL, "null pointer");
  if (!workspace || ws_bytes < item_src_ws_bytes(n_items, V)) return set_error(REGCN_EINVAL, "item order workspace too small");
  const Layout L = tlayout(n_items, V, 2);
  char* ws = (char*)workspace;
  int* rowpos = (int*)(ws + L.total);
  int rc;
  hipLaunchKernelGGL(k_item_rowpos, dim3(std::min<unsigned>(blocks(n_tiles, 4), 65536)), dim3(BT), 0, st, tiles,
                     item_ptr, item_tl, n_tiles, rowpos);
  if ((rc = check_launch("k_item_rowpos"))) return rc;
  hipLaunchKernelGGL(k_iota_keys, dim3(blocks(n_items)), dim3(BT), 0, st, by_type ? item_tl : item_src, n_items,
                     (uint32_t*)(ws + L.k0), (uint32_t*)(ws + L.v0));
  bool second;
  if ((rc = radix_sort(ws, L, n_items, key_bits, true, &second, st))) return rc;
  hipLaunchKernelGGL(k_row_of, dim3(blocks(n_items)), dim3(BT), 0, st, rowpos,
                     (const uint32_t*)(ws + (second ? L.v1 : L.v0)), n_items, (uint32_t*)(ws + L.k0),
                     (uint32_t*)(ws + L.v0));
  if ((rc = check_launch("k_row_of"))) return rc;
  if ((rc = radix_sort(ws, L, n_items, bitlen((uint64_t)V - 1), true, &second, st))) return rc;
  hipLaunchKernelGGL(k_permute2, dim3(blocks(n_items)), dim3(BT), 0, st, (const uint32_t*)(ws + (second ? L.v1 : L.v0)),
                     n_items, item_src, item_tl, out_src, out_tl);
  return check_launch("k_permute2");
}

int item_src_order(int V, int n_tiles, int n_items, const int* tiles, const int* item_ptr, const int* item_src,
                   const int* item_tl, int* out_src, int* out_tl, void* workspace, size_t ws_bytes, hipStream_t st) {
  if (V <= 0) return set_error(REGCN_EINVAL, "bad item order sizes");
  return item_order(V, bitlen((uint64_t)V - 1), 0, n_tiles, n_items, tiles, item_ptr, item_src, item_tl, out_src,
                    out_tl, workspace, ws_bytes, st);
}

int item_type_order(int V, int R2, int n_tiles, int n_items, const int* tiles, const int* item_ptr,
                    const int* item_src, const int* item_tl, int* out_src, int* out_tl, void* workspace,
                    size_t ws_bytes, hipStream_t st) {
  if (R2 <= 0 || R2 >= (1 << 27)) return set_error(REGCN_EINVAL, "bad relation count %d", R2);
  return item_order(V, bitlen((uint64_t)R2 * 16 - 1), 1, n_tiles, n_items, tiles, item_ptr, item_src, item_tl,
                    out_src, out_tl, workspace, ws_bytes, st);
}

// Stable LSD radix sort by source, then stably by destination row: each row's sources in
// ascending order, so a row's duplicate sources are adjacent (k_union_runs<., true>).
int row_src_order(int V, int E, const int* rowptr, const int* col_src, int* out_src, void* workspace, size_t ws_bytes,
                  hipStream_t st) {
  if (V <= 0 || E < 0) return set_error(REGCN_EINVAL, "bad row/source order sizes");
  if (E == 0) return 0;
  if (!rowptr || !col_src || !out_src) return set_error(REGCN_EINVAL, "null pointer");
  if (!workspace || ws_bytes < row_src_ws_bytes(E, V)) return set_error(REGCN_EINVAL, "row/source order workspace too small");
  const Layout L = tlayout(E, V, 2);
  char* ws = (char*)workspace;
  int* csr_dst = (int*)(ws + L.total);
  int rc;
  hipLaunchKernelGGL(k_csr_dst, dim3(std::min<unsigned>(blocks(V, 4), 65536)), dim3(BT), 0, st, rowptr, V, csr_dst);
  if ((rc = check_launch("k_csr_dst"))) return rc;
  hipLaunchKernelGGL(k_iota_keys, dim3(blocks(E)), dim3(BT), 0, st, col_src, E, (uint32_t*)(ws + L.k0),
                     (uint32_t*)(ws + L.v0));
  bool second;
  if ((rc = radix_sort(ws, L, E, bitlen((uint64_t)V - 1), true, &second, st))) return rc;
  hipLaunchKernelGGL(k_row_of, dim3(blocks(E)), dim3(BT), 0, st, csr_dst,
                     (const uint32_t*)(ws + (second ? L.v1 : L.v0)), E, (uint32_t*)(ws + L.k0),
                     (uint32_t*)(ws + L.v0));
  if ((rc = check_launch("k_row_of"))) return rc;
  if ((rc = radix_sort(ws, L, E, bitlen((uint64_t)V - 1), true, &second, st))) return rc;
  hipLaunchKernelGGL(k_permute1, dim3(blocks(E)), dim3(BT), 0, st, (const uint32_t*)(ws + (second ? L.v1 : L.v0)), E,
                     col_src, out_src);
  return check_launch("k_permute1");
}

int64_t snapshot_capacity(int what, int64_t T, int V, int R, int C) {
  const int64_t E = 2 * T, EC = E / std::max(C, 1) + 1, R2 = 2 * (int64_t)R;
  switch (what) {
    case REGCN_CAP_TILES: return std::max<int64_t>(V, 1);
    case REGCN_CAP_ITEMS: return std::max<int64_t>(E, 1);
    case REGCN_CAP_CHUNKS: return EC + std::min<int64_t>(V, E) + 1;
    case REGCN_CAP_FIXUPS: return 3 * EC + V / FIX_GROUP + 16;
    case REGCN_CAP_HEAVY_CHUNKS: return EC + std::min<int64_t>(V, E) + 1;  // heavy rows: a subset of the rows
    case REGCN_CAP_HEAVY_FIXUPS: return 3 * EC + 16;
    case REGCN_CAP_REL_CHUNKS: return 2 * EC + R2 + 1;
    case REGCN_CAP_REL_FIXUPS: return 6 * EC + R2 / FIX_GROUP + 16;
    case REGCN_CAP_REL_IDX: return std::max<int64_t>(2 * E, 1);
    default: return -1;
  }
}

}  // namespace regcn
