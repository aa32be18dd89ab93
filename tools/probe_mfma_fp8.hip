// Probe of the scale lane map of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3).
// Workgroup (L1, L0, side): the operand on `side` holds 1.0 in all 32 bytes of lane L1 and
// 0 elsewhere, the other operand is all 1.0; lane L0's e8m0 scale on `side` is 2 (others 1).
// The output row (side A) / column (side B) that lights up is the one lane L1's data feeds,
// and its value 32 + (number of L1's elements that L0's scale governs) says which lanes'
// scales govern which data. Usage: tools/probe_mfma_fp8 [opsel_byte]
//   hipcc -O2 --offload-arch=gfx950 tools/probe_mfma_fp8.hip -o tools/probe_mfma_fp8
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void run(float* out, int side, int sbyte) {
  const int l = threadIdx.x;
  const int L1 = blockIdx.x / 64, L0 = blockIdx.x % 64;
  const int one = 0x38383838;  // four e4m3 1.0
  i32x8 data, ones;
  for (int i = 0; i < 8; ++i) { data[i] = l == L1 ? one : 0; ones[i] = one; }
  const int s1 = 127 << (8 * sbyte);
  const int s2 = (l == L0 ? 128 : 127) << (8 * sbyte);
  f4 c = {0, 0, 0, 0};
  if (side == 0)
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(data, ones, c, 0, 0, 0, s2, 0, s1);
  else
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(ones, data, c, 0, 0, 0, s1, 0, s2);
  for (int r = 0; r < 4; ++r) out[(size_t)blockIdx.x * 256 + l * 4 + r] = c[r];
}

int main(int argc, char** argv) {
  const int sbyte = argc > 1 ? atoi(argv[1]) : 0;
  float* d;
  if (hipMalloc(&d, 4096 * 256 * sizeof(float)) != hipSuccess) return 1;
  std::vector<float> h(4096 * 256);
  for (int side = 0; side < 2; ++side) {
    hipLaunchKernelGGL(run, dim3(4096), dim3(64), 0, 0, d, side, sbyte);
    if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    printf("side %c (scale byte %d): data lane L1 -> output %s ; scale lanes L0 governing it (+count)\n",
           side ? 'B' : 'A', sbyte, side ? "column" : "row");
    for (int L1 = 0; L1 < 64; ++L1) {
      int idx = -1;
      printf("L1=%2d:", L1);
      for (int L0 = 0; L0 < 64; ++L0) {
        const float* o = &h[(size_t)(L1 * 64 + L0) * 256];
        float mx = 0;
        int where = -1;
        for (int l = 0; l < 64; ++l)
          for (int r = 0; r < 4; ++r) {
            const int row = 4 * (l >> 4) + r, col = l & 15;
            if (o[l * 4 + r] > mx) { mx = o[l * 4 + r]; where = side ? col : row; }
          }
        if (L0 == 0) { idx = where; printf(" -> %d :", idx); }
        if (mx != 32.f) printf(" %d(+%g)", L0, mx - 32.f);
      }
      printf("\n");
    }
  }
  hipFree(d);
  return 0;
}
