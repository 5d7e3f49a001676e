// Probe: operand / result lane layout and issue rate of v_mfma_f32_4x4x1_16b_f32 on gfx950.
// Profiling tool, not part of the library.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(float* out) {
  const int l = threadIdx.x;
  // pass 0: A = lane + 1, B = 1 -> D shows which A lane feeds (lane, reg)
  f4 d0 = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(l + 1), 1.f, f4{0, 0, 0, 0}, 0, 0, 0);
  // pass 1: A = 1, B = lane + 1
  f4 d1 = __builtin_amdgcn_mfma_f32_4x4x1f32(1.f, (float)(l + 1), f4{0, 0, 0, 0}, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    out[(0 * 64 + l) * 4 + r] = d0[r];
    out[(1 * 64 + l) * 4 + r] = d1[r];
  }
}

__global__ void k_rate(const float* in, float* out, int n, long long* clk) {
  float a = in[threadIdx.x], b = in[threadIdx.x + 64];
  f4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  long long c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[j], 0, 0, 0);
  }
  long long c1 = __builtin_amdgcn_s_memtime();
  f4 s = acc[0] + acc[1] + acc[2] + acc[3];
  out[threadIdx.x] = s[0] + s[1] + s[2] + s[3];
  if (threadIdx.x == 0) clk[0] = c1 - c0;
}

int main() {
  float* out;
  long long* clk;
  hipMalloc(&out, 4096 * 4);
  hipMalloc(&clk, 8);
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, out);
  float h[512];
  hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
  for (int p = 0; p < 2; ++p) {
    printf("pass %d (%s lane+1 per (lane, reg)):\n", p, p ? "B" : "A");
    for (int l = 0; l < 64; ++l) {
      printf("  l%02d:", l);
      for (int r = 0; r < 4; ++r) printf(" %3.0f", h[(p * 64 + l) * 4 + r]);
      printf(l % 4 == 3 ? "\n" : " |");
    }
  }
  const int n = 4096;
  hipLaunchKernelGGL(k_rate, dim3(1), dim3(64), 0, 0, out, out + 1024, n, clk);
  long long c;
  hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
  printf("4x4x1_16b: %.2f cycles per MFMA (4 independent accumulators, one wave)\n", (double)c / (4.0 * n));
  return 0;
}
