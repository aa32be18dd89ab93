// Register-only fp32 MFMA throughput probe (v_mfma_f32_32x32x2_f32), random operands.
// Reports TFLOP/s for 1..4 waves per SIMD: the ceiling the GEMM is measured against.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters, float seed) {
  f32x16 acc[NACC];
  for (int a = 0; a < NACC; ++a)
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
  float x = seed * (threadIdx.x + 1), y = seed * (blockIdx.x + 3);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[a], 0, 0, 0);
    x += 1e-7f;
  }
  float s = 0.f;
  for (int a = 0; a < NACC; ++a)
    for (int r = 0; r < 16; ++r) s += acc[a][r];
  if (s == 12345.f) out[0] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int wps = 1; wps <= 4; ++wps) {
    const int blocks = 256 * wps;  // 256 threads = 1 wave per SIMD per block
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(256), 0, 0, out, 100, 0.5f);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)blocks * 4 * iters * 4 * 32 * 32 * 2 * 2;
    printf("waves/SIMD=%d  %.1f TFLOP/s (%.2f ms)\n", wps, flops / (ms * 1e-3) / 1e12, ms);
  }
  return 0;
}
