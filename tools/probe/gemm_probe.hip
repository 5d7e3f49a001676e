// Probe: latency of one row tile's d x d GEMM (16 rows, fp32 MFMA, B streamed from the
// packed weight) as the fused row kernels run it (rowtile.h), alone on the chip and on a
// full grid, with the weight warm in L2 or not.  Profiling tool, not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I re-gcn_amd/csrc tools/probe/gemm_probe.hip -o gpurun_out/gemm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "rowtile.h"

using namespace regcn;

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

// acc += T @ W with a B ring of R k-steps (the rowtile.h loop with the depth as a parameter)
template <int R>
__device__ __forceinline__ void tile_ring(Frag& acc, const float* T, int lda, const float* __restrict__ Wp, int d) {
  const int lane = threadIdx.x & 63;
  const int S = d >> 2;
  const bvec* bsrc = bsrc_of(Wp);
  const float* arow = T + (lane & 15) * lda + (lane >> 4);
  bvec ring[R];
  float aring[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    ring[i] = bsrc[(int64_t)min(i, S - 1) * B_STEP];
    aring[i] = arow[4 * min(i, S - 1)];
  }
  int s = 0;
  for (; s + R <= S; s += R) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      mfma_tpw(acc, aring[i], ring[i]);
      __builtin_amdgcn_sched_barrier(0);
      const int nx = min(s + i + R, S - 1);
      ring[i] = bsrc[(int64_t)nx * B_STEP];
      aring[i] = arow[4 * nx];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i)
    if (s + i < S) mfma_tpw(acc, aring[i], ring[i]);
}

// MODE 0: ring 8; 1: ring 16; 2: two chains (mfma_tiles<2, 8>); 3: A from registers only
// (B ring 8, no LDS reads: the MFMA + B-stream floor)
template <int MODE>
__global__ __launch_bounds__(NTHR) void k_probe(const float* __restrict__ X, const float* __restrict__ W,
                                                const float* __restrict__ W2, int d, int reps, float* out,
                                                long long* stamps) {
  __shared__ float T[2][TM * 226];
  const int lda = tile_lda(d);
  for (int i = threadIdx.x; i < TM * lda; i += NTHR) {
    T[0][i] = X[(blockIdx.x * TM * lda + i) % (1 << 20)];
    T[1][i] = X[(blockIdx.x * TM * lda + i + 777) % (1 << 20)];
  }
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memrealtime();
  long long c0 = __builtin_amdgcn_s_memtime();
  Frag acc, acc2;
  acc.zero();
  acc2.zero();
  for (int r = 0; r < reps; ++r) {
    if (MODE == 0) tile_ring<8>(acc, T[0], lda, W, d);
    if (MODE == 1) tile_ring<16>(acc, T[0], lda, W, d);
    if (MODE == 3) {  // the MFMA floor: operands already in registers, same instruction count
      const int lane = threadIdx.x & 63;
      float a = T[0][lane];
      bvec b = *reinterpret_cast<const bvec*>(W + 4 * lane);
      for (int s = 0; s < (d >> 2); ++s) {
        mfma_tpw(acc, a, b);
        a += 1e-7f;
      }
    }
    if (MODE == 2) {
      Frag a2[2];
      a2[0] = acc;
      a2[1] = acc2;
      const float* Ts[2] = {T[0], T[1]};
      const float* Ws[2] = {W, W2};
      mfma_tiles<2, 8>(a2, Ts, Ws, lda, d);
      acc = a2[0];
      acc2 = a2[1];
    }
  }
  long long t1 = __builtin_amdgcn_s_memrealtime();
  long long c1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < TPW; ++j) s += acc.t[j][0] + acc.t[j][1] + acc.t[j][2] + acc.t[j][3] + acc2.t[j][0];
  out[blockIdx.x * NTHR + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t1;
    if (blockIdx.x == 0) stamps[4094] = c1 - c0, stamps[4095] = t1 - t0;
  }
}

__global__ void k_flush(float* buf, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    buf[i] = buf[i] * 0.5f + 1.f;
}

template <int MODE>
void run(const char* name, int grid, bool cold, int reps, float* X, float* W, float* W2, float* out,
         long long* stamps, float* flush, size_t nflush) {
  const int d = 200;
  std::vector<double> durs;
  for (int it = 0; it < 5; ++it) {
    if (cold) hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, flush, nflush);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_probe<MODE>), dim3(grid), dim3(NTHR), 0, 0, X, W, W2, d, reps, out, stamps);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<long long> h(2 * grid);
    CK(hipMemcpy(h.data(), stamps, 16 * grid, hipMemcpyDeviceToHost));
    double mx = 0, sum = 0;
    for (int g = 0; g < grid; ++g) {
      double us = (h[2 * g + 1] - h[2 * g]) / 100.0;
      mx = std::max(mx, us);
      sum += us;
    }
    if (it >= 2) durs.push_back(sum / grid), durs.push_back(mx), durs.push_back(ms * 1e3);
  }
  double flops = 2.0 * TM * d * d * reps * (MODE == 2 ? 2 : 1);
  long long cc[2];
  CK(hipMemcpy(cc, stamps + 4094, 16, hipMemcpyDeviceToHost));
  printf("[clk %.0f MHz] ", cc[1] ? cc[0] * 100.0 / cc[1] : 0.0);
  printf("%-10s grid %4d %s reps %d: per-WG mean %.2f us max %.2f us kernel %.2f us | %.1f GF/s per WG, chip %.1f TF/s\n",
         name, grid, cold ? "cold" : "warm", reps, durs[3], durs[4], durs[5], flops / durs[3] / 1e3,
         flops * grid / durs[5] / 1e6);
}

int main() {
  const int d = 200;
  float *X, *W, *W2, *out, *flush;
  long long* stamps;
  size_t nflush = (size_t)512 << 20 >> 2;  // 512 MB: through L2 and the Infinity Cache
  CK(hipMalloc(&X, (1 << 20) * 4 + 4096));
  CK(hipMalloc(&W, d * 256 * 4));
  CK(hipMalloc(&W2, d * 256 * 4));
  CK(hipMalloc(&out, 2048 * NTHR * 4));
  CK(hipMalloc(&stamps, 4096 * 8));
  CK(hipMalloc(&flush, nflush * 4));
  std::vector<float> h(1 << 20);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(X, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(W, h.data(), d * 256 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(W2, h.data() + 5000, d * 256 * 4, hipMemcpyHostToDevice));
  CK(hipMemset(flush, 0, nflush * 4));
  for (int grid : {1, 256, 512, 768}) {
    for (bool cold : {false, true}) {
      run<0>("ring8", grid, cold, 1, X, W, W2, out, stamps, flush, nflush);
      run<1>("ring16", grid, cold, 1, X, W, W2, out, stamps, flush, nflush);
      run<2>("2chains", grid, cold, 1, X, W, W2, out, stamps, flush, nflush);
    }
    run<0>("ring8", grid, false, 8, X, W, W2, out, stamps, flush, nflush);
    run<3>("regs", grid, false, 8, X, W, W2, out, stamps, flush, nflush);
    run<1>("ring16", grid, false, 8, X, W, W2, out, stamps, flush, nflush);
  }
  return 0;
}
