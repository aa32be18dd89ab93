// Residual + layer_normalization forward/backward and row flags.
//
// Reference: layer_normalization.forward, models/modules.py:62-65 (mean, UNBIASED
// std, eps=1e-8 added to std) applied to the residual sums of modules.py:304
// (attention) and :439 (feed-forward). One wave per row; rows are 512 (or 1024)
// floats, loaded as float4 (2 per lane at d=512). The forward also emits the
// exact-zero row flag sign(|sum_c y|) that the NEXT attention uses as its key and
// query mask (modules.py:257, :289), so that mask never re-reads the activations.
#include "common.h"


namespace savqa {

constexpr int LN_MAXV = 4;  // float4 per lane -> cols <= 1024
typedef __bf16 ln_bf16x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x,
                                                     const float* __restrict__ xscale,
                                                     const float* __restrict__ r, int64_t rows,
                                                     int cols, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     float* __restrict__ z_out,
                                                     float* __restrict__ y,
                                                     float* __restrict__ mean_out,
                                                     float* __restrict__ rden_out,
                                                     float* __restrict__ std_out,
                                                     float* __restrict__ flag,
                                                     __bf16* __restrict__ yb) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = cols >> 8;  // float4 per lane (cols % 256 == 0)
  const float4* xr = reinterpret_cast<const float4*>(x + row * cols);
  const float4* rr = r ? reinterpret_cast<const float4*>(r + row * cols) : nullptr;
  float4 v[LN_MAXV];
  float s = 0.f;
  const float xs = xscale ? xscale[row] : 1.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    if (i < nv) {
      float4 a = xr[lane + 64 * i];
      if (xscale) { a.x *= xs; a.y *= xs; a.z *= xs; a.w *= xs; }
      if (rr) {
        float4 b = rr[lane + 64 * i];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      v[i] = a;
      s += (a.x + a.y) + (a.z + a.w);
    }
  }
  const float mean = wave_sum(s) / (float)cols;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    if (i < nv) {
      const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, e = v[i].w - mean;
      ss += (a * a + b * b) + (c * c + e * e);
    }
  }
  const float var = wave_sum(ss) / (float)(cols - 1);
  const float sd = sqrtf(var);
  const float den = sd + eps;
  float fsum = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    if (i < nv) {
      const int c4 = lane + 64 * i;
      const float4 g = reinterpret_cast<const float4*>(gamma)[c4];
      const float4 bt = reinterpret_cast<const float4*>(beta)[c4];
      float4 o;
      o.x = g.x * (v[i].x - mean) / den + bt.x;
      o.y = g.y * (v[i].y - mean) / den + bt.y;
      o.z = g.z * (v[i].z - mean) / den + bt.z;
      o.w = g.w * (v[i].w - mean) / den + bt.w;
      reinterpret_cast<float4*>(y + row * cols)[c4] = o;
      if (yb) reinterpret_cast<ln_bf16x4*>(yb + row * cols)[c4] =
          ln_bf16x4{(__bf16)o.x, (__bf16)o.y, (__bf16)o.z, (__bf16)o.w};
      if (z_out) reinterpret_cast<float4*>(z_out + row * cols)[c4] = v[i];
      fsum += (o.x + o.y) + (o.z + o.w);
    }
  }
  if (flag) fsum = wave_sum(fsum);
  if (lane == 0) {
    mean_out[row] = mean;
    rden_out[row] = 1.f / den;
    std_out[row] = sd;
    if (flag) flag[row] = fsum != 0.f ? 1.f : 0.f;
  }
}

// Backward. 512-thread workgroups (8 waves), two per CU: each wave walks rows with a
// grid stride, keeping its dgamma/dbeta partial sums in registers; the 8 waves fold
// them through per-wave LDS rows and the workgroup stores its partial row ws[block][2 cols]
// (the caller's workspace, plain stores), which ln_bwd_reduce_kernel then adds in block
// order into dgamma/dbeta: deterministic (round 4 added the partials atomically into 16
// slots, i.e. in arrival order; 512 adders on ONE address serialised in L2). NV (float4 per
// lane = cols/256) is a template parameter, and the row loop is software-pipelined two
// deep: the loads of row r+stride are in flight while row r is reduced and written
// (one row's loads in flight per wave left every wave waiting on HBM latency).
constexpr int LN_BWD_WAVES = 8;
// grid cap: round 4 measured 1024 / 2048 blocks slower standalone (18688 x 512: 22.9 us =
// 5.0 TB/s at 512 blocks; 25.1 / 27.9 / 41.9 us) and equal in-step
constexpr int LN_BWD_BLOCKS = 512;

template <int NV, bool ADD>
struct LnBwdRow {
  float4 d[NV], z[NV], a[ADD ? NV : 1];
  float mean, rden, sd;
};

template <int NV, bool ADD>
__device__ __forceinline__ void ln_bwd_fetch(LnBwdRow<NV, ADD>& b, int64_t row, int lane, int cols,
                                             const float* __restrict__ dy,
                                             const float* __restrict__ z,
                                             const float* __restrict__ dz_add,
                                             const float* __restrict__ mean_in,
                                             const float* __restrict__ rden_in,
                                             const float* __restrict__ std_in) {
  const float4* dyr = reinterpret_cast<const float4*>(dy + row * cols);
  const float4* zr = reinterpret_cast<const float4*>(z + row * cols);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    b.d[i] = dyr[lane + 64 * i];
    b.z[i] = zr[lane + 64 * i];
    if constexpr (ADD) b.a[i] = reinterpret_cast<const float4*>(dz_add + row * cols)[lane + 64 * i];
  }
  b.mean = mean_in[row];
  b.rden = rden_in[row];
  b.sd = std_in[row];
}

template <int NV, bool ADD>
__device__ __forceinline__ void ln_bwd_row(const LnBwdRow<NV, ADD>& b, int64_t row, int lane, int cols,
                                           float invN, const float4 (&g)[NV], float4 (&dg)[NV],
                                           float4 (&db)[NV], const float* __restrict__ dz_add,
                                           float* __restrict__ dz, __bf16* __restrict__ dzb) {
  float4 gg[NV], xc[NV];
  float sg = 0.f, sgx = 0.f;
  const float mean = b.mean, rden = b.rden;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float4 d4 = b.d[i], z4 = b.z[i];
    xc[i] = make_float4(z4.x - mean, z4.y - mean, z4.z - mean, z4.w - mean);
    gg[i] = make_float4(d4.x * g[i].x, d4.y * g[i].y, d4.z * g[i].z, d4.w * g[i].w);
    sg += (gg[i].x + gg[i].y) + (gg[i].z + gg[i].w);
    sgx += (gg[i].x * xc[i].x + gg[i].y * xc[i].y) + (gg[i].z * xc[i].z + gg[i].w * xc[i].w);
    dg[i].x += d4.x * xc[i].x * rden; dg[i].y += d4.y * xc[i].y * rden;
    dg[i].z += d4.z * xc[i].z * rden; dg[i].w += d4.w * xc[i].w * rden;
    db[i].x += d4.x; db[i].y += d4.y; db[i].z += d4.z; db[i].w += d4.w;
  }
  sg = wave_sum(sg);
  sgx = wave_sum(sgx);
  const float mg = sg * invN;
  // d std / dz_k = xc_k / ((N-1) std); guard std == 0 (constant row)
  const float c = b.sd > 0.f ? sgx * rden * rden / ((float)(cols - 1) * b.sd) : 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float4 o;
    o.x = (gg[i].x - mg) * rden - c * xc[i].x;
    o.y = (gg[i].y - mg) * rden - c * xc[i].y;
    o.z = (gg[i].z - mg) * rden - c * xc[i].z;
    o.w = (gg[i].w - mg) * rden - c * xc[i].w;
    if constexpr (ADD) {
      o.x += b.a[i].x; o.y += b.a[i].y; o.z += b.a[i].z; o.w += b.a[i].w;
    }
    reinterpret_cast<float4*>(dz + row * cols)[lane + 64 * i] = o;
    if (dzb) reinterpret_cast<ln_bf16x4*>(dzb + row * cols)[lane + 64 * i] =
        ln_bf16x4{(__bf16)o.x, (__bf16)o.y, (__bf16)o.z, (__bf16)o.w};
  }
}

template <int NV, bool ADD>
__global__ __launch_bounds__(64 * LN_BWD_WAVES) void ln_bwd_kernel(const float* __restrict__ dy,
                                                     const float* __restrict__ z,
                                                     const float* __restrict__ mean_in,
                                                     const float* __restrict__ rden_in,
                                                     const float* __restrict__ std_in,
                                                     const float* __restrict__ gamma,
                                                     int64_t rows, int cols,
                                                     const float* __restrict__ dz_add,
                                                     float* __restrict__ dz,
                                                     __bf16* __restrict__ dzb,
                                                     float* __restrict__ ws) {
  __shared__ float red[LN_BWD_WAVES][2][256 * NV];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  float4 dg[NV], db[NV], g[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    dg[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    db[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    g[i] = reinterpret_cast<const float4*>(gamma)[lane + 64 * i];
  }
  const float invN = 1.f / (float)cols;
  const int64_t stride = (int64_t)gridDim.x * LN_BWD_WAVES;
  int64_t row = (int64_t)blockIdx.x * LN_BWD_WAVES + w;
  LnBwdRow<NV, ADD> b0, b1;
  if (row < rows) ln_bwd_fetch<NV, ADD>(b0, row, lane, cols, dy, z, dz_add, mean_in, rden_in, std_in);
  while (row < rows) {
    const int64_t r1 = row + stride;
    if (r1 < rows) ln_bwd_fetch<NV, ADD>(b1, r1, lane, cols, dy, z, dz_add, mean_in, rden_in, std_in);
    ln_bwd_row<NV, ADD>(b0, row, lane, cols, invN, g, dg, db, dz_add, dz, dzb);
    if (r1 >= rows) break;
    const int64_t r2 = r1 + stride;
    if (r2 < rows) ln_bwd_fetch<NV, ADD>(b0, r2, lane, cols, dy, z, dz_add, mean_in, rden_in, std_in);
    ln_bwd_row<NV, ADD>(b1, r1, lane, cols, invN, g, dg, db, dz_add, dz, dzb);
    row = r2;
  }
  // fold the 8 waves' partials: plain per-wave LDS rows, then one thread per column
  // (ds_add_f32 folding cost ~20 us per launch: LDS float atomics serialise)
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    reinterpret_cast<float4*>(&red[w][0][0])[lane + 64 * i] = dg[i];
    reinterpret_cast<float4*>(&red[w][1][0])[lane + 64 * i] = db[i];
  }
  __syncthreads();
  float* part = ws + (int64_t)blockIdx.x * 2 * cols;
  for (int c = threadIdx.x; c < 2 * cols; c += blockDim.x) {
    const int a = c >= cols, cc = c - a * cols;
    float t = 0.f;
#pragma unroll
    for (int ww = 0; ww < LN_BWD_WAVES; ++ww) t += red[ww][a][cc];
    part[c] = t;
  }
}

// dgamma[c] += sum_b ws[b][0][c]; dbeta[c] += sum_b ws[b][1][c] over the nb block partials in
// a fixed order: 16 row groups of 64 columns per 1024-thread workgroup, group r summing blocks
// r, r + 16, ... (all of its <= 32 loads issued in batches of 8), then the 16 group sums as a
// fixed pairwise tree. (4 row groups left each thread 128 loads deep at nb = 512: ~16 latency
// rounds on 16 workgroups; the relation workload lost ~1 %.)
constexpr int LN_RED_GROUPS = 16;
__global__ __launch_bounds__(1024) void ln_bwd_reduce_kernel(const float* __restrict__ ws, int cols,
                                                             int nb, float* __restrict__ dgamma,
                                                             float* __restrict__ dbeta) {
  __shared__ float red[LN_RED_GROUPS][64];
  const int rg = threadIdx.x >> 6, lc = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + lc;
  float sacc = 0.f;
  if (c < 2 * cols) {
    int b = rg;
    for (; b + 7 * LN_RED_GROUPS < nb; b += 8 * LN_RED_GROUPS) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = ws[(int64_t)(b + LN_RED_GROUPS * u) * 2 * cols + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) sacc += x[u];
    }
    for (; b < nb; b += LN_RED_GROUPS) sacc += ws[(int64_t)b * 2 * cols + c];
  }
  red[rg][lc] = sacc;
  __syncthreads();
#pragma unroll
  for (int h = LN_RED_GROUPS / 2; h > 0; h >>= 1) {
    if (rg < h) red[rg][lc] += red[rg + h][lc];
    __syncthreads();
  }
  if (rg != 0 || c >= 2 * cols) return;
  const float t = red[0][lc];
  if (c < cols) {
    if (dgamma) dgamma[c] += t;
  } else if (dbeta) {
    dbeta[c - cols] += t;
  }
}

__global__ __launch_bounds__(256) void rowflag_kernel(const float* __restrict__ X, int64_t rows,
                                                      int64_t cols, int64_t ldx,
                                                      float* __restrict__ flag) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float s = 0.f;
  for (int64_t c = lane; c < cols; c += 64) s += X[row * ldx + c];
  s = wave_sum(s);
  if (lane == 0) flag[row] = s != 0.f ? 1.f : 0.f;
}

}  // namespace savqa

using namespace savqa;

extern "C" int savqa_ln_fwd(void* stream, const float* x, const float* xscale, const float* r,
                            int64_t rows,
                            int64_t cols, const float* gamma, const float* beta, float eps,
                            float* z_out, float* y, float* mean, float* rden, float* stdv,
                            float* flag, void* yb) {
  if (rows <= 0) return 0;
  if (cols % 256 != 0 || cols > 256 * LN_MAXV)
    return fail(SAVQA_EUNSUP, "savqa_ln_fwd: cols must be a multiple of 256 and <= 1024");
  hipLaunchKernelGGL(ln_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, as_stream(stream), x, xscale,
                     r, rows, (int)cols, gamma, beta, eps, z_out, y, mean, rden, stdv, flag,
                     static_cast<__bf16*>(yb));
  return check_launch("savqa_ln_fwd");
}

extern "C" int64_t savqa_ln_bwd_workspace_bytes(int64_t cols) {
  return (int64_t)sizeof(float) * LN_BWD_BLOCKS * 2 * cols;  // one partial row per block
}

extern "C" int savqa_ln_bwd(void* stream, const float* dy, const float* z, const float* mean,
                            const float* rden, const float* stdv, const float* gamma,
                            int64_t rows, int64_t cols, const float* dz_add, float* dz,
                            float* dgamma, float* dbeta, float* ws, int64_t ws_bytes, void* dzb) {
  if (rows <= 0) return 0;
  if (cols % 256 != 0 || cols > 256 * LN_MAXV)
    return fail(SAVQA_EUNSUP, "savqa_ln_bwd: cols must be a multiple of 256 and <= 1024");
  if (!ws || ws_bytes < savqa_ln_bwd_workspace_bytes(cols) || ((uintptr_t)ws & 15))
    return fail(SAVQA_EINVAL, "savqa_ln_bwd: workspace missing, too small or not 16-B aligned");
  int64_t blocks = (rows + LN_BWD_WAVES - 1) / LN_BWD_WAVES;
  if (blocks > LN_BWD_BLOCKS) blocks = LN_BWD_BLOCKS;
  const dim3 g((unsigned)blocks), b(64 * LN_BWD_WAVES);
  hipStream_t st = as_stream(stream);
  switch (cols / 256) {
#define SAVQA_LNB(NV)                                                                        \
  case NV:                                                                                   \
    if (dz_add)                                                                              \
      hipLaunchKernelGGL((ln_bwd_kernel<NV, true>), g, b, 0, st, dy, z, mean, rden, stdv,    \
                         gamma, rows, (int)cols, dz_add, dz, static_cast<__bf16*>(dzb), ws);  \
    else                                                                                     \
      hipLaunchKernelGGL((ln_bwd_kernel<NV, false>), g, b, 0, st, dy, z, mean, rden, stdv,   \
                         gamma, rows, (int)cols, dz_add, dz, static_cast<__bf16*>(dzb), ws);  \
    break;
    SAVQA_LNB(1) SAVQA_LNB(2) SAVQA_LNB(3) SAVQA_LNB(4)
#undef SAVQA_LNB
  }
  if (int rc = check_launch("savqa_ln_bwd")) return rc;
  hipLaunchKernelGGL(ln_bwd_reduce_kernel, dim3((unsigned)((2 * cols + 63) / 64)), dim3(1024), 0, st,
                     ws, (int)cols, (int)blocks, dgamma, dbeta);
  return check_launch("savqa_ln_bwd");
}

extern "C" int savqa_rowflag(void* stream, const float* X, int64_t rows, int64_t cols,
                             int64_t ldx, float* flag) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(rowflag_kernel, dim3((rows + 3) / 4), dim3(256), 0, as_stream(stream), X,
                     rows, cols, ldx, flag);
  return check_launch("savqa_rowflag");
}
