// Conversions feeding the low-precision GEMM operands (include/savqa.h): fp32 -> bf16 casts
// (activation / weight shadows of the bf16 training mode), fp32 -> fp8-e4m3 with e8m0
// per-32-column block scales (BASELINE cfg 5's region features and the weights they meet),
// the fp8 -> bf16 expansion the backward uses, and the column sums of bf16 gradients (bias
// gradients of the low-precision GEMMs). All HBM-bound: one pass, 16-B accesses.
#include "common.h"

namespace savqa {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));

// OCP e4m3fn encoding of a finite |x| <= 448 (round to nearest even; larger values
// saturate to 448 = 0x7E, the format has no infinity). Integer arithmetic on the fp32
// bits, so it is exact and identical to torch's float8_e4m3fn conversion for in-range x.
__device__ __forceinline__ uint32_t f32_to_e4m3(float x) {
  const uint32_t u = __float_as_uint(x);
  const uint32_t sign = (u >> 24) & 0x80u;
  const uint32_t a = u & 0x7fffffffu;
  uint32_t code;
  if (a >= 0x43E80000u) {          // >= 464: rounds past the largest finite value
    code = 0x7E;
  } else if (a < 0x3C800000u) {    // < 2^-6: subnormal, units of 2^-9
    const float q = rintf(__uint_as_float(a) * 512.f);  // 0..8 (8 = smallest normal)
    code = (uint32_t)q;
  } else {
    const uint32_t e = (a >> 23) - 127 + 7;              // biased e4m3 exponent 1..15
    const uint32_t mant = a & 0x7fffffu;
    const uint32_t lsb = (mant >> 20) & 1u;
    const uint32_t r = mant + 0x7FFFFu + lsb;            // RNE at 3 mantissa bits
    uint32_t m3 = r >> 20;
    uint32_t ee = e;
    if (m3 == 8) { m3 = 0; ee += 1; }
    code = (ee << 3) | m3;
    if (code > 0x7E) code = 0x7E;
  }
  return code | sign;  // signed zero kept, as torch's float8_e4m3fn cast does
}

__device__ __forceinline__ float e4m3_to_f32(uint32_t c) {
  const uint32_t s = c & 0x80u, e = (c >> 3) & 0xF, m = c & 7u;
  float v = e ? __uint_as_float(((e + 120) << 23) | (m << 20)) : (float)m * (1.f / 512.f);
  return s ? -v : v;
}

// destination row of source row r: (r / group) * stride + r % group + offset (group <= 0:
// r) -- writes straight into the question rows of a [B][T] concat buffer
struct RowMap {
  int64_t group, stride, offset;
  __device__ __forceinline__ int64_t operator()(int64_t r) const {
    return group > 0 ? (r / group) * stride + r % group + offset : r;
  }
};

__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ in, int64_t rows,
                                                        int64_t cols, int64_t ldi,
                                                        __bf16* __restrict__ out, int64_t ldo,
                                                        int vec, RowMap map) {
  const int64_t per_row = vec ? cols / 4 : cols;
  const int64_t n = rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / per_row, c = i - r * per_row;
    const int64_t ro = map(r);
    if (vec) {
      const f4v v = *reinterpret_cast<const f4v*>(in + r * ldi + 4 * c);
      *reinterpret_cast<bf16x4*>(out + ro * ldo + 4 * c) = __builtin_convertvector(v, bf16x4);
    } else {
      out[ro * ldo + c] = (__bf16)in[r * ldi + c];
    }
  }
}

// out[r*ldo + c] = float(in[r*ldi + c]): exact widening of bf16 rows (the fp32 operands the
// key-tiled attention takes in the low-precision modes at T > 128)
__global__ __launch_bounds__(256) void widen_bf16_kernel(const __bf16* __restrict__ in, int64_t rows,
                                                         int64_t cols, int64_t ldi,
                                                         float* __restrict__ out, int64_t ldo, int vec) {
  const int64_t per_row = vec ? cols / 4 : cols;
  const int64_t n = rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / per_row, c = i - r * per_row;
    if (vec) {
      const bf16x4 v = *reinterpret_cast<const bf16x4*>(in + r * ldi + 4 * c);
      *reinterpret_cast<f4v*>(out + r * ldo + 4 * c) = __builtin_convertvector(v, f4v);
    } else {
      out[r * ldo + c] = (float)in[r * ldi + c];
    }
  }
}

// one wave per (row, 64 32-column blocks): lane = block, 32 values each
__global__ __launch_bounds__(256) void quant_fp8_kernel(const float* __restrict__ in, int64_t rows,
                                                        int64_t cols, int64_t ldi,
                                                        uint8_t* __restrict__ q, int64_t ldq,
                                                        uint8_t* __restrict__ scale, int64_t lds,
                                                        RowMap map) {
  const int64_t nb = cols / 32;
  const int64_t total = rows * nb;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / nb, b = i - r * nb;
    const float* src = in + r * ldi + b * 32;
    float v[32];
    float mx = 0.f;
#pragma unroll
    for (int k = 0; k < 32; k += 4) {
      const f4v t = *reinterpret_cast<const f4v*>(src + k);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[k + u] = t[u];
        mx = fmaxf(mx, fabsf(t[u]));
      }
    }
    // smallest power of two 2^e with mx / 2^e <= 448 (e8m0 code e + 127, clamped)
    int e = 0;
    if (mx > 0.f) {
      e = (int)ceilf(log2f(mx / 448.f));
      if (ldexpf(448.f, e - 1) >= mx) e -= 1;  // guard log2 rounding
      if (ldexpf(448.f, e) < mx) e += 1;
    }
    e = e < -127 ? -127 : (e > 127 ? 127 : e);
    const float inv = ldexpf(1.f, -e);
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      w[k] = f32_to_e4m3(v[4 * k] * inv) | (f32_to_e4m3(v[4 * k + 1] * inv) << 8) |
             (f32_to_e4m3(v[4 * k + 2] * inv) << 16) | (f32_to_e4m3(v[4 * k + 3] * inv) << 24);
    }
    const int64_t ro = map(r);
    uint4* dst = reinterpret_cast<uint4*>(q + ro * ldq + b * 32);
    dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
    dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
    scale[ro * lds + b] = (uint8_t)(e + 127);
  }
}

__global__ __launch_bounds__(256) void dequant_fp8_kernel(const uint8_t* __restrict__ q, int64_t rows,
                                                          int64_t cols, int64_t ldq,
                                                          const uint8_t* __restrict__ scale,
                                                          int64_t lds, __bf16* __restrict__ out,
                                                          int64_t ldo) {
  const int64_t per_row = cols / 4;
  const int64_t n = rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / per_row, c = (i - r * per_row) * 4;
    const uint32_t w = *reinterpret_cast<const uint32_t*>(q + r * ldq + c);
    const float s = ldexpf(1.f, (int)scale[r * lds + c / 32] - 127);
    f4v v;
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = e4m3_to_f32((w >> (8 * u)) & 0xFFu) * s;
    *reinterpret_cast<bf16x4*>(out + r * ldo + c) = __builtin_convertvector(v, bf16x4);
  }
}

// out[c] += sum_r X[r][c] (bf16 X): 256 threads = 64 columns x 4 row slices per block
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const __bf16* __restrict__ X, int64_t rows,
                                                          int64_t cols, int64_t ldx, int64_t rchunk,
                                                          float* __restrict__ out) {
  __shared__ float part[4][64];
  const int64_t c = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int sl = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * rchunk;
  const int64_t r1 = min(rows, r0 + rchunk);
  float s = 0.f;
  if (c < cols)
    for (int64_t r = r0 + sl; r < r1; r += 4) s += (float)X[r * ldx + c];
  part[sl][threadIdx.x & 63] = s;
  __syncthreads();
  if (sl == 0 && c < cols)
    atomicAdd(&out[c], (part[0][threadIdx.x] + part[1][threadIdx.x]) +
                           (part[2][threadIdx.x] + part[3][threadIdx.x]));
}

// Wide form (cols % 8 == 0, 16-B aligned rows): each lane sums 8 consecutive columns with
// 16-B loads (a wave covers 512 columns of a row), the 4 waves of a block take interleaved
// rows of its row chunk, and fold through LDS before one atomicAdd per column and block.
// (The 2-B-per-lane form above ran the bias-gradient sums at ~2.3 TB/s.)
typedef __bf16 cs_bf16x8 __attribute__((ext_vector_type(8)));
__global__ __launch_bounds__(256) void colsum_bf16_wide_kernel(const __bf16* __restrict__ X,
                                                               int64_t rows, int64_t cols,
                                                               int64_t ldx, int64_t rchunk,
                                                               float* __restrict__ out) {
  __shared__ float part[4][512];
  const int lane = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 512 + 8 * lane;
  const int64_t r0 = (int64_t)blockIdx.y * rchunk;
  const int64_t r1 = min(rows, r0 + rchunk);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int64_t r = r0 + sl;
    for (; r + 12 < r1; r += 16) {  // four rows in flight per lane
      cs_bf16x8 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = *reinterpret_cast<const cs_bf16x8*>(X + (r + 4 * u) * ldx + c);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += (float)v[u][j];
    }
    for (; r < r1; r += 4) {
      const cs_bf16x8 v = *reinterpret_cast<const cs_bf16x8*>(X + r * ldx + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += (float)v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[sl][8 * lane + j] = s[j];
  __syncthreads();
  for (int k = threadIdx.x; k < 512; k += 256) {
    const int64_t cc = (int64_t)blockIdx.x * 512 + k;
    if (cc < cols) atomicAdd(&out[cc], (part[0][k] + part[1][k]) + (part[2][k] + part[3][k]));
  }
}

// GloVe rows of a token list into a zero-padded bf16 matrix: one wave per output row, each
// lane 4 consecutive columns (16-B fp32 loads when the table rows allow, 8-B bf16 stores).
__global__ __launch_bounds__(256) void gather_rows_bf16_kernel(const float* __restrict__ table,
                                                               int64_t ldt,
                                                               const int64_t* __restrict__ ids,
                                                               int64_t n, int64_t cols,
                                                               __bf16* __restrict__ out,
                                                               int64_t ldo, bool vec) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  const float* src = table + ids[r] * ldt;
  __bf16* dst = out + r * ldo;
  for (int64_t c = 4 * lane; c < ldo; c += 256) {
    float v[4];
    if (vec && c + 4 <= cols) {
      const f4v t = *reinterpret_cast<const f4v*>(src + c);
      v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = c + j < cols ? src[c + j] : 0.f;
    }
    if (c + 4 <= ldo) {
      *reinterpret_cast<bf16x4v*>(dst + c) = bf16x4v{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    } else {
      for (int j = 0; c + j < ldo; ++j) dst[c + j] = (__bf16)v[j];
    }
  }
}

static unsigned grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

}  // namespace savqa

using namespace savqa;

extern "C" int savqa_cast_bf16(void* stream, const float* in, int64_t rows, int64_t cols, int64_t ldi,
                               void* out, int64_t ldo, int64_t group, int64_t stride,
                               int64_t offset) {
  if (rows <= 0 || cols <= 0) return 0;
  const int vec = (cols % 4 == 0) && (ldi % 4 == 0) && (ldo % 4 == 0) &&
                  (((uintptr_t)in) & 15) == 0 && (((uintptr_t)out) & 7) == 0;
  const int64_t n = rows * (vec ? cols / 4 : cols);
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), in, rows,
                     cols, ldi, static_cast<__bf16*>(out), ldo, vec, RowMap{group, stride, offset});
  return check_launch("savqa_cast_bf16");
}

extern "C" int savqa_widen_bf16(void* stream, const void* in, int64_t rows, int64_t cols,
                                int64_t ldi, float* out, int64_t ldo) {
  if (rows <= 0 || cols <= 0) return 0;
  const int vec = (cols % 4 == 0) && (ldi % 4 == 0) && (ldo % 4 == 0) &&
                  (((uintptr_t)in) & 7) == 0 && (((uintptr_t)out) & 15) == 0;
  const int64_t n = rows * (vec ? cols / 4 : cols);
  hipLaunchKernelGGL(widen_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream),
                     static_cast<const __bf16*>(in), rows, cols, ldi, out, ldo, vec);
  return check_launch("savqa_widen_bf16");
}

extern "C" int savqa_quant_fp8(void* stream, const float* in, int64_t rows, int64_t cols, int64_t ldi,
                               void* q, int64_t ldq, uint8_t* scale, int64_t lds, int64_t group,
                               int64_t stride, int64_t offset) {
  if (rows <= 0 || cols <= 0) return 0;
  if (cols % 32 || ldi % 4 || ldq % 16 || (((uintptr_t)in) & 15) || (((uintptr_t)q) & 15))
    return fail(SAVQA_EINVAL, "savqa_quant_fp8: cols % 32, 16-B aligned rows required");
  hipLaunchKernelGGL(quant_fp8_kernel, dim3(grid_for(rows * (cols / 32))), dim3(256), 0,
                     as_stream(stream), in, rows, cols, ldi, static_cast<uint8_t*>(q), ldq, scale, lds,
                     RowMap{group, stride, offset});
  return check_launch("savqa_quant_fp8");
}

extern "C" int savqa_dequant_fp8_bf16(void* stream, const void* q, int64_t rows, int64_t cols,
                                      int64_t ldq, const uint8_t* scale, int64_t lds, void* out,
                                      int64_t ldo) {
  if (rows <= 0 || cols <= 0) return 0;
  if (cols % 32 || ldq % 4 || ldo % 4 || (((uintptr_t)q) & 3) || (((uintptr_t)out) & 7))
    return fail(SAVQA_EINVAL, "savqa_dequant_fp8_bf16: cols % 32 and aligned rows required");
  hipLaunchKernelGGL(dequant_fp8_kernel, dim3(grid_for(rows * cols / 4)), dim3(256), 0,
                     as_stream(stream), static_cast<const uint8_t*>(q), rows, cols, ldq, scale, lds,
                     static_cast<__bf16*>(out), ldo);
  return check_launch("savqa_dequant_fp8_bf16");
}

extern "C" int savqa_colsum_bf16(void* stream, const void* X, int64_t rows, int64_t cols, int64_t ldx,
                                 float* out) {
  if (rows <= 0 || cols <= 0) return 0;
  if (cols % 8 == 0 && ldx % 8 == 0 && (((uintptr_t)X) & 15) == 0) {
    const int64_t cb = (cols + 511) / 512;
    int64_t chunks = (2048 + cb - 1) / cb;
    int64_t rchunk = (rows + chunks - 1) / chunks;
    if (rchunk < 64) rchunk = 64;
    chunks = (rows + rchunk - 1) / rchunk;
    hipLaunchKernelGGL(colsum_bf16_wide_kernel, dim3((unsigned)cb, (unsigned)chunks), dim3(256), 0,
                       as_stream(stream), static_cast<const __bf16*>(X), rows, cols, ldx, rchunk,
                       out);
    return check_launch("savqa_colsum_bf16");
  }
  const int64_t cb = (cols + 63) / 64;
  int64_t chunks = (2048 + cb - 1) / cb;
  int64_t rchunk = (rows + chunks - 1) / chunks;
  if (rchunk < 64) rchunk = 64;
  chunks = (rows + rchunk - 1) / rchunk;
  hipLaunchKernelGGL(colsum_bf16_kernel, dim3((unsigned)cb, (unsigned)chunks), dim3(256), 0,
                     as_stream(stream), static_cast<const __bf16*>(X), rows, cols, ldx, rchunk, out);
  return check_launch("savqa_colsum_bf16");
}

extern "C" int savqa_gather_rows_bf16(void* stream, const float* table, int64_t ldt,
                                      const int64_t* ids, int64_t n, int64_t cols, void* out,
                                      int64_t ldo) {
  if (n <= 0) return 0;
  if (cols <= 0 || ldo < cols || (ldo & 3) || (((uintptr_t)out) & 7))
    return fail(SAVQA_EINVAL, "savqa_gather_rows_bf16: need 0 < cols <= ldo, ldo % 4 == 0, 8-B aligned out");
  const bool vec = (ldt & 3) == 0 && (((uintptr_t)table) & 15) == 0;
  hipLaunchKernelGGL(gather_rows_bf16_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0,
                     as_stream(stream), table, ldt, ids, n, cols, static_cast<__bf16*>(out), ldo,
                     vec);
  return check_launch("savqa_gather_rows_bf16");
}
