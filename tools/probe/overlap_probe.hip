// Probe: do fp32 MFMA (v_mfma_f32_16x16x4_f32) and fp32 VALU work from two waves of the same
// SIMD overlap on gfx950?  One 8-wave workgroup per CU (waves w and w + 4 share a SIMD); per
// mode, what waves 0-3 (A) and 4-7 (B) run: 0 = A MFMA, B idle; 1 = A VALU, B idle; 2 = A MFMA,
// B VALU; 3 = both MFMA; 4 = both VALU; 5 = A MFMA, B transcendental (v_exp_f32).  If 2 takes
// max(0, 1) the pipes overlap, if 0 + 1 they share an issue path.  Profiling tool, not part of
// the library.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float mfma_loop(float a, float b, int n) {
  f4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
  }
  f4 s = acc[0] + acc[1] + acc[2] + acc[3];
  return s[0] + s[1] + s[2] + s[3];
}

// 8 independent fma chains, 32 VALU per iteration (the same issue count as 4 MFMAs x 8 passes)
__device__ __forceinline__ float valu_loop(float a, float b, int n) {
  float x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = a + k;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = __builtin_fmaf(x[k], b, 0.5f);
    asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k];
  return s;
}

__device__ __forceinline__ float trans_loop(float a, float b, int n) {
  float x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = a + k;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = __builtin_amdgcn_exp2f(x[k] * b);
    asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k];
  return s;
}

__global__ __launch_bounds__(512) void k_overlap(const float* in, float* out, int mode, int nm, int nv,
                                                  long long* clk) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const float a = in[l], b = in[64 + l];
  const bool A = w < 4;
  long long c0 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
  int what = 0;  // 0 idle, 1 mfma, 2 valu, 3 trans
  if (mode == 0) what = A ? 1 : 0;
  if (mode == 1) what = A ? 2 : 0;
  if (mode == 2) what = A ? 1 : 2;
  if (mode == 3) what = 1;
  if (mode == 4) what = 2;
  if (mode == 5) what = A ? 1 : 3;
  if (what == 1) r = mfma_loop(a, b, nm);
  if (what == 2) r = valu_loop(a, b, nv);
  if (what == 3) r = trans_loop(a, b, nv / 4);
  long long c1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 512 + threadIdx.x] = r;
  if (l == 0) clk[blockIdx.x * 8 + w] = c1 - c0;
}

int main() {
  float *in, *out;
  long long* clk;
  hipMalloc(&in, 128 * 4);
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&clk, 256 * 8 * 8);
  float h[128];
  for (int i = 0; i < 128; ++i) h[i] = 1e-3f * (i % 7);
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int nm = 4096, nv = 4096;
  const char* names[6] = {"A mfma, B idle", "A valu, B idle", "A mfma, B valu", "A+B mfma", "A+B valu", "A mfma, B exp"};
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 6; ++mode) {
      hipLaunchKernelGGL(k_overlap, dim3(256), dim3(512), 0, 0, in, out, mode, nm, nv, clk);
      hipEventRecord(e0);
      for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k_overlap, dim3(256), dim3(512), 0, 0, in, out, mode, nm, nv, clk);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1) printf("mode %d %-16s %8.3f ms per launch  (%d MFMA / %d x 32 VALU per wave)\n", mode, names[mode], ms / 5, 4 * nm, nv);
    }
  return 0;
}
