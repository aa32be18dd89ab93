// Dropout of the model_v=3 path (nn.Dropout(dropout_rate) sites, reference default 0.5,
// main_itp_ddp_tar_super_node.py:466, submit.py:98). Masks come from the stateless
// counter stream in common.h (drop_bits), so every backward regenerates the forward's
// mask; nothing is stored. All kernels are HBM-bound elementwise passes (float4 per lane).
#include "common.h"

namespace savqa {

// out[i] = in[i] * keep(i) * scale -- nn.Dropout forward, and its backward (same op on dY).
__global__ __launch_bounds__(256) void dropout_kernel(const float* __restrict__ in, int64_t n,
                                                     DropParam dp, uint32_t site,
                                                     float* __restrict__ out) {
  const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= n) return;
  if (i4 + 4 <= n) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 v = *reinterpret_cast<const f4*>(in + i4);
    v.x *= drop_mul(dp, site, i4);
    v.y *= drop_mul(dp, site, i4 + 1);
    v.z *= drop_mul(dp, site, i4 + 2);
    v.w *= drop_mul(dp, site, i4 + 3);
    *reinterpret_cast<f4*>(out + i4) = v;
  } else {
    for (int64_t i = i4; i < n; ++i) out[i] = in[i] * drop_mul(dp, site, i);
  }
}

// Stack input (AttModel_x3.py:99-102 vis, :222-227 syb):
//   out[b,t,c] = Dx( z[b,t,c] + Dp(pos[t,c]) )     Dp = identity when site_pos < 0
// Element index of both masks: (b*T + t)*d + c  (the (B,T,d) tensor nn.Dropout sees).
__global__ __launch_bounds__(256) void posadd_dropout_kernel(
    const float* __restrict__ z, const float* __restrict__ pos, int64_t B, int64_t T, int64_t d,
    DropParam dp, int32_t site_pos, uint32_t site_x, float* __restrict__ out) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= B * T * d) return;
  const int64_t row = i4 / d, c = i4 - row * d, t = row % T;
  f4 zv = *reinterpret_cast<const f4*>(z + i4);
  f4 pv = *reinterpret_cast<const f4*>(pos + t * d + c);
  if (site_pos >= 0) {
    pv.x *= drop_mul(dp, site_pos, i4);
    pv.y *= drop_mul(dp, site_pos, i4 + 1);
    pv.z *= drop_mul(dp, site_pos, i4 + 2);
    pv.w *= drop_mul(dp, site_pos, i4 + 3);
  }
  f4 o = zv + pv;
  o.x *= drop_mul(dp, site_x, i4);
  o.y *= drop_mul(dp, site_x, i4 + 1);
  o.z *= drop_mul(dp, site_x, i4 + 2);
  o.w *= drop_mul(dp, site_x, i4 + 3);
  *reinterpret_cast<f4*>(out + i4) = o;
}

// Backward: dz = Dx'(g) (written over g's buffer when dz == g), and
//   dpos[t,c] += sum_b Dp'(dz[b,t,c])
// One thread per (t, 4 columns, chunk of kBChunk samples), coalesced along c; the chunk
// partial sums meet in dpos with atomics (B/kBChunk-way, fp32 order not fixed).
constexpr int kBChunk = 32;
__global__ __launch_bounds__(128) void posadd_dropout_bwd_kernel(
    const float* g, int64_t B, int64_t T, int64_t d, DropParam dp, int32_t site_pos,
    uint32_t site_x, float* dz, float* __restrict__ dpos) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const int64_t t = blockIdx.y;
  if (c >= d) return;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int64_t b1 = min(B, (int64_t)(blockIdx.z + 1) * kBChunk);
  for (int64_t b = (int64_t)blockIdx.z * kBChunk; b < b1; ++b) {
    const int64_t i4 = (b * T + t) * d + c;
    f4 v = *reinterpret_cast<const f4*>(g + i4);
    v.x *= drop_mul(dp, site_x, i4);
    v.y *= drop_mul(dp, site_x, i4 + 1);
    v.z *= drop_mul(dp, site_x, i4 + 2);
    v.w *= drop_mul(dp, site_x, i4 + 3);
    *reinterpret_cast<f4*>(dz + i4) = v;
    if (site_pos >= 0) {
      v.x *= drop_mul(dp, site_pos, i4);
      v.y *= drop_mul(dp, site_pos, i4 + 1);
      v.z *= drop_mul(dp, site_pos, i4 + 2);
      v.w *= drop_mul(dp, site_pos, i4 + 3);
    }
    acc += v;
  }
  if (dpos) {
    float* o = dpos + t * d + c;
    atomicAdd(o, acc.x);
    atomicAdd(o + 1, acc.y);
    atomicAdd(o + 2, acc.z);
    atomicAdd(o + 3, acc.w);
  }
}

}  // namespace savqa

using namespace savqa;

extern "C" int savqa_dropout(void* stream, const float* in, int64_t n, uint64_t seed, int32_t site,
                             float p, float* out) {
  if (n <= 0) return 0;
  if (p < 0.f || p > 1.f || site < 0) return fail(SAVQA_EINVAL, "savqa_dropout: bad p or site");
  if (((uintptr_t)in | (uintptr_t)out) & 15)
    return fail(SAVQA_EINVAL, "savqa_dropout: buffers must be 16-byte aligned");
  const int64_t th = (n + 3) / 4;
  hipLaunchKernelGGL(dropout_kernel, dim3((th + 255) / 256), dim3(256), 0, as_stream(stream), in, n,
                     make_drop(seed, p), (uint32_t)site, out);
  return check_launch("savqa_dropout");
}

extern "C" int savqa_posadd_dropout(void* stream, const float* z, const float* pos, int64_t B,
                                    int64_t T, int64_t d, uint64_t seed, int32_t site_pos,
                                    int32_t site_x, float p, float* out) {
  if (B <= 0 || T <= 0 || d <= 0) return 0;
  if (d % 4 || site_x < 0 || p < 0.f || p > 1.f)
    return fail(SAVQA_EINVAL, "savqa_posadd_dropout: d must be a multiple of 4, p in [0,1]");
  if (((uintptr_t)z | (uintptr_t)pos | (uintptr_t)out) & 15)
    return fail(SAVQA_EINVAL, "savqa_posadd_dropout: buffers must be 16-byte aligned");
  const int64_t th = B * T * d / 4;
  hipLaunchKernelGGL(posadd_dropout_kernel, dim3((th + 255) / 256), dim3(256), 0,
                     as_stream(stream), z, pos, B, T, d, make_drop(seed, p), site_pos,
                     (uint32_t)site_x, out);
  return check_launch("savqa_posadd_dropout");
}

extern "C" int savqa_posadd_dropout_bwd(void* stream, const float* g, int64_t B, int64_t T,
                                        int64_t d, uint64_t seed, int32_t site_pos,
                                        int32_t site_x, float p, float* dz, float* dpos) {
  if (B <= 0 || T <= 0 || d <= 0) return 0;
  if (d % 4 || site_x < 0 || p < 0.f || p > 1.f)
    return fail(SAVQA_EINVAL, "savqa_posadd_dropout_bwd: d must be a multiple of 4, p in [0,1]");
  if (((uintptr_t)g | (uintptr_t)dz | (uintptr_t)dpos) & 15)
    return fail(SAVQA_EINVAL, "savqa_posadd_dropout_bwd: buffers must be 16-byte aligned");
  hipLaunchKernelGGL(posadd_dropout_bwd_kernel, dim3((d / 4 + 127) / 128, T, (B + kBChunk - 1) / kBChunk), dim3(128), 0,
                     as_stream(stream), g, B, T, d, make_drop(seed, p), site_pos, (uint32_t)site_x,
                     dz, dpos);
  return check_launch("savqa_posadd_dropout_bwd");
}
