// Bandwidth-bound pieces of the model_v=3 step: graph construction, decoder input,
// row copies (torch.cat), MIL-NCE core, index_put/get, loss, Adam.
#include "common.h"

namespace savqa {

// ------------------------------------------------------------------ graph build
// AttModel_x3.py:103-122 / :229-247. One block per (b, row i), threads over j.
__global__ __launch_bounds__(256) void graph_build_kernel(
    const int32_t* __restrict__ nm, const int32_t* __restrict__ qm, const int32_t* __restrict__ qg,
    const int32_t* __restrict__ ng, int Nn, int Lq, int dec_on, float* __restrict__ gdiag,
    float* __restrict__ graph, float* __restrict__ dec_mask) {
  __shared__ float part[4];
  const int T = Nn + Lq;
  const int b = blockIdx.x / T, i = blockIdx.x % T;
  float rs = 0.f;
  for (int j = threadIdx.x; j < T; j += blockDim.x) {
    float m = 0.f, gd = 0.f, g = 1.f;  // off-diagonal blocks: 1 - 0
    if (i < Nn && j < Nn) {
      m = (float)nm[((int64_t)b * Nn + i) * Nn + j];
      g = ng ? (float)ng[((int64_t)b * Nn + i) * Nn + j] : 1.f;
    } else if (i >= Nn && j >= Nn) {
      const int64_t o = ((int64_t)b * Lq + (i - Nn)) * Lq + (j - Nn);
      m = (float)qm[o];
      gd = m;
      g = (float)qg[o];
    }
    const int64_t o = ((int64_t)b * T + i) * T + j;
    gdiag[o] = gd;
    graph[o] = g;
    rs += m;
  }
  rs = wave_sum(rs);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = rs;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w];
    dec_mask[(int64_t)b * T + i] = (dec_on && t != 0.f) ? 1.f : 0.f;
  }
}

// ------------------------------------------------------------------ decoder input
__global__ void dec_init_kernel(const float* __restrict__ emb, int64_t idx, float scale,
                                const float* __restrict__ pos, int64_t B, int64_t d,
                                DropParam dp, int32_t site, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * d) return;
  const int64_t c = t % d;
  float v = emb[idx * d + c] * scale + pos[c];
  if (site >= 0) v *= drop_mul(dp, site, t);  // dec_dropout (AttModel_x3.py:147, :274)
  out[t] = v;
}

// d emb[idx] += scale * sum_b D'(g[b]), d pos[0] += sum_b D'(g[b]). Block: 32 columns x 8
// row slices (slice r sums rows r, r + 8, ..), folded through LDS in a fixed order -- one
// thread per column looping over all B rows (two workgroups at d = 512, each element a
// SplitMix64 mask) took 69-130 us per launch
constexpr int DIB_COLS = 32, DIB_SLICES = 8;
__global__ __launch_bounds__(256) void dec_init_bwd_kernel(const float* __restrict__ g, int64_t B,
                                                           int64_t d, int64_t idx, float scale,
                                                           DropParam dp, int32_t site,
                                                           float* __restrict__ demb,
                                                           float* __restrict__ dpos) {
  __shared__ float part[DIB_SLICES][DIB_COLS];
  const int cl = threadIdx.x % DIB_COLS, sl = threadIdx.x / DIB_COLS;
  const int64_t c = (int64_t)blockIdx.x * DIB_COLS + cl;
  float ss = 0.f;
  if (c < d) {
    for (int64_t b = sl; b < B; b += DIB_SLICES) {
      float v = g[b * d + c];
      if (site >= 0) v *= drop_mul(dp, site, b * d + c);
      ss += v;
    }
  }
  part[sl][cl] = ss;
  __syncthreads();
  if (sl == 0 && c < d) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < DIB_SLICES; ++r) t += part[r][cl];
    if (demb) demb[idx * d + c] += t * scale;
    if (dpos) dpos[c] += t;
  }
}

// out[t][c] += sum_b X[(b*T + t)*ldx + c]  (gradient of a learned position table)
__global__ void period_sum_kernel(const float* __restrict__ X, int64_t B, int64_t T, int64_t C,
                                  int64_t ldx, float* __restrict__ out) {
  const int64_t t = blockIdx.y;
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int64_t b = 0; b < B; ++b) s += X[(b * T + t) * ldx + c];
  out[t * C + c] += s;
}

// ------------------------------------------------------------------ row copy (cat)
__global__ void copy_rows_kernel(const float* __restrict__ src, int64_t rows, int64_t cols,
                                 int64_t lds, float* __restrict__ dst, int64_t ldd, int64_t group,
                                 int64_t stride, int64_t offset) {
  const int64_t r = blockIdx.x;
  const int64_t dr = (r / group) * stride + (r % group) + offset;
  const float* s = src + r * lds;
  float* d = dst + dr * ldd;
  if ((cols & 3) == 0 && (((uintptr_t)s | (uintptr_t)d) & 15) == 0) {
    for (int64_t c = threadIdx.x; c < cols / 4; c += blockDim.x)
      reinterpret_cast<float4*>(d)[c] = reinterpret_cast<const float4*>(s)[c];
  } else {
    for (int64_t c = threadIdx.x; c < cols; c += blockDim.x) d[c] = s[c];
  }
}

// ------------------------------------------------------------------ MIL-NCE
// one wave per (b, n) row; lanes over H (float4), K (= topN) <= 16 candidates.
constexpr int MIL_KMAX = 16;

__global__ __launch_bounds__(256) void mil_fwd_kernel(const float* __restrict__ Pf,
                                                      const float* __restrict__ Nf,
                                                      const float* __restrict__ v,
                                                      const int32_t* __restrict__ mask,
                                                      int64_t BN, int K, int H, float eps,
                                                      float* __restrict__ obj,
                                                      float* __restrict__ term) {
  const int lane = threadIdx.x & 63;
  const int64_t bn = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bn >= BN) return;
  const int h4 = H / 4;
  const float4* vr = reinterpret_cast<const float4*>(v + bn * H);
  float sp[MIL_KMAX], sn[MIL_KMAX];
  for (int k = 0; k < K; ++k) {
    const float4* pr = reinterpret_cast<const float4*>(Pf + (bn * K + k) * H);
    const float4* nr = reinterpret_cast<const float4*>(Nf + (bn * K + k) * H);
    float a = 0.f, c = 0.f;
    for (int i = lane; i < h4; i += 64) {
      const float4 vv = vr[i], pp = pr[i], qq = nr[i];
      a += (pp.x * vv.x + pp.y * vv.y) + (pp.z * vv.z + pp.w * vv.w);
      c += (qq.x * vv.x + qq.y * vv.y) + (qq.z * vv.z + qq.w * vv.w);
    }
    sp[k] = wave_sum(a);
    sn[k] = wave_sum(c);
  }
  // softmax over k of the raw positive scores (AttModel_x3.py:372-373)
  float mx = -INFINITY;
  for (int k = 0; k < K; ++k) mx = fmaxf(mx, sp[k]);
  float den = 0.f;
  for (int k = 0; k < K; ++k) { sp[k] = expf(sp[k] - mx); den += sp[k]; }
  for (int k = 0; k < K; ++k) sp[k] = sp[k] / den;
  for (int i = lane; i < h4; i += 64) {
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < K; ++k) {
      const float4 pp = reinterpret_cast<const float4*>(Pf + (bn * K + k) * H)[i];
      o.x = fmaf(sp[k], pp.x, o.x); o.y = fmaf(sp[k], pp.y, o.y);
      o.z = fmaf(sp[k], pp.z, o.z); o.w = fmaf(sp[k], pp.w, o.w);
    }
    reinterpret_cast<float4*>(obj + bn * H)[i] = o;
  }
  if (lane == 0) {
    // LSE_k(clamp(mask*s-, eps)) (AttModel_x3.py:367)
    float m2 = -INFINITY;
    for (int k = 0; k < K; ++k) {
      sn[k] = fmaxf((float)mask[bn * K + k] * sn[k], eps);
      m2 = fmaxf(m2, sn[k]);
    }
    float s2 = 0.f;
    for (int k = 0; k < K; ++k) s2 += expf(sn[k] - m2);
    const float lse_neg = m2 + logf(s2);
    const float lse_eps = eps + logf((float)K);
    term[bn] = lse_eps - lse_neg;
  }
}

__global__ void mean_reduce_kernel(const float* __restrict__ x, int64_t n, float scale,
                                   float* __restrict__ out) {
  __shared__ float part[16];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w];
    *out = t * scale;
  }
}

__device__ __forceinline__ void mil_store4(float* p, const float4& v) {
  *reinterpret_cast<float4*>(p) = v;
}
__device__ __forceinline__ void mil_store4(__bf16* p, const float4& v) {
  typedef __bf16 b4 __attribute__((ext_vector_type(4)));
  *reinterpret_cast<b4*>(p) = b4{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
}

// TO: element type of dPf / dNf (float, or bf16 for the low-precision modes' GEMMs)
template <typename TO>
__global__ __launch_bounds__(256) void mil_bwd_kernel(
    const float* __restrict__ Pf, const float* __restrict__ Nf, const float* __restrict__ v,
    const int32_t* __restrict__ mask, int64_t BN, int K, int H, float eps,
    const float* __restrict__ dobj, const float* __restrict__ dmil, TO* __restrict__ dPf,
    TO* __restrict__ dNf, float* __restrict__ dv) {
  const int lane = threadIdx.x & 63;
  const int64_t bn = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bn >= BN) return;
  const int h4 = H / 4;
  const float4* vr = reinterpret_cast<const float4*>(v + bn * H);
  const float4* dor = dobj ? reinterpret_cast<const float4*>(dobj + bn * H) : nullptr;
  float sp[MIL_KMAX], sn[MIL_KMAX], dw[MIL_KMAX];
  for (int k = 0; k < K; ++k) {
    const float4* pr = reinterpret_cast<const float4*>(Pf + (bn * K + k) * H);
    const float4* nr = reinterpret_cast<const float4*>(Nf + (bn * K + k) * H);
    float a = 0.f, c = 0.f, e = 0.f;
    for (int i = lane; i < h4; i += 64) {
      const float4 vv = vr[i], pp = pr[i], qq = nr[i];
      a += (pp.x * vv.x + pp.y * vv.y) + (pp.z * vv.z + pp.w * vv.w);
      c += (qq.x * vv.x + qq.y * vv.y) + (qq.z * vv.z + qq.w * vv.w);
      if (dor) {
        const float4 g = dor[i];
        e += (g.x * pp.x + g.y * pp.y) + (g.z * pp.z + g.w * pp.w);
      }
    }
    sp[k] = wave_sum(a);
    sn[k] = wave_sum(c);
    dw[k] = wave_sum(e);
  }
  // softmax weights w and their backward dsp = w*(dw - sum w dw)
  float mx = -INFINITY;
  for (int k = 0; k < K; ++k) mx = fmaxf(mx, sp[k]);
  float den = 0.f;
  for (int k = 0; k < K; ++k) { sp[k] = expf(sp[k] - mx); den += sp[k]; }
  float wdw = 0.f;
  for (int k = 0; k < K; ++k) { sp[k] = sp[k] / den; wdw += sp[k] * dw[k]; }
  float dsp[MIL_KMAX], dsn[MIL_KMAX];
  for (int k = 0; k < K; ++k) dsp[k] = sp[k] * (dw[k] - wdw);
  // term = LSE(eps) - LSE(snc): d snc_k = -dterm * softmax_k(snc); clamp passes where >= eps
  const float dterm = (*dmil) / (2.f * (float)BN);
  {
    float m2 = -INFINITY;
    float snc[MIL_KMAX];
    for (int k = 0; k < K; ++k) {
      const float mk = (float)mask[bn * K + k];
      snc[k] = fmaxf(mk * sn[k], eps);
      m2 = fmaxf(m2, snc[k]);
    }
    float s2 = 0.f;
    for (int k = 0; k < K; ++k) { dsn[k] = expf(snc[k] - m2); s2 += dsn[k]; }
    for (int k = 0; k < K; ++k) {
      const float mk = (float)mask[bn * K + k];
      const float d_snc = -dterm * (dsn[k] / s2);
      dsn[k] = (mk * sn[k] >= eps) ? d_snc * mk : 0.f;
    }
  }
  for (int i = lane; i < h4; i += 64) {
    const float4 vv = vr[i];
    float4 g = dor ? dor[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < K; ++k) {
      const int64_t off = (bn * K + k) * H;
      const float4 pp = reinterpret_cast<const float4*>(Pf + off)[i];
      const float4 qq = reinterpret_cast<const float4*>(Nf + off)[i];
      float4 dp, dn;
      dp.x = pp.x > 0.f ? sp[k] * g.x + dsp[k] * vv.x : 0.f;
      dp.y = pp.y > 0.f ? sp[k] * g.y + dsp[k] * vv.y : 0.f;
      dp.z = pp.z > 0.f ? sp[k] * g.z + dsp[k] * vv.z : 0.f;
      dp.w = pp.w > 0.f ? sp[k] * g.w + dsp[k] * vv.w : 0.f;
      dn.x = qq.x > 0.f ? dsn[k] * vv.x : 0.f;
      dn.y = qq.y > 0.f ? dsn[k] * vv.y : 0.f;
      dn.z = qq.z > 0.f ? dsn[k] * vv.z : 0.f;
      dn.w = qq.w > 0.f ? dsn[k] * vv.w : 0.f;
      mil_store4(dPf + off + 4 * i, dp);
      mil_store4(dNf + off + 4 * i, dn);
      acc.x += dsp[k] * pp.x + dsn[k] * qq.x;
      acc.y += dsp[k] * pp.y + dsn[k] * qq.y;
      acc.z += dsp[k] * pp.z + dsn[k] * qq.z;
      acc.w += dsp[k] * pp.w + dsn[k] * qq.w;
    }
    float4 o;
    o.x = vv.x > 0.f ? acc.x : 0.f; o.y = vv.y > 0.f ? acc.y : 0.f;
    o.z = vv.z > 0.f ? acc.z : 0.f; o.w = vv.w > 0.f ? acc.w : 0.f;
    reinterpret_cast<float4*>(dv + bn * H)[i] = o;
  }
}

// Single-pass forms (SAVQA_MIL_SPLIT, the default, for H <= 1024 and topN <= 8): one 256-thread
// workgroup per (b, n) row, thread t owning float4 column t of every candidate row, so the P / N
// rows are read once and held in registers from the scores to the outputs (the one-wave kernels
// above read them again for the outputs: P twice forward, P and N twice backward). The per-k dot
// products are summed in exactly the one-wave kernels' order -- lane l adds its columns l,
// l + 64, l + 128, l + 192 in sequence (here: the 4 waves' partials of lane l, exchanged through
// LDS), then the same wave tree -- so the scores, and the forward's object features, are
// bit-identical to theirs (the gradients up to the compiler's FMA-contraction choices), and every
// thread holds the same bits; the softmax / LSE scalars are then formed redundantly per thread.
#ifndef SAVQA_MIL_SPLIT
#define SAVQA_MIL_SPLIT 1
#endif
constexpr int MIL_SPLIT_H = 1024, MIL_SPLIT_K = 8;

template <int NV>
__device__ __forceinline__ void mil_fold(float (&x)[NV], float (*part)[4][64]) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < NV; ++k) part[k][w][lane] = x[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) a += part[k][r][lane];
    x[k] = wave_sum(a);
  }
}

__device__ __forceinline__ float mil_dot4(const float4& a, const float4& b) {
  return (a.x * b.x + a.y * b.y) + (a.z * b.z + a.w * b.w);
}

template <int KC>
__global__ __launch_bounds__(256) void mil_fwd_split_kernel(const float* __restrict__ Pf,
                                                            const float* __restrict__ Nf,
                                                            const float* __restrict__ v,
                                                            const int32_t* __restrict__ mask,
                                                            int H, float eps,
                                                            float* __restrict__ obj,
                                                            float* __restrict__ term) {
  __shared__ float red[2 * KC][4][64];
  const int64_t bn = blockIdx.x;
  const int i = threadIdx.x, h4 = H / 4;
  const bool act = i < h4;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 vv = act ? reinterpret_cast<const float4*>(v + bn * H)[i] : z;
  float4 pp[KC];
  float sc[2 * KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int64_t off = (bn * KC + k) * h4 + i;
    pp[k] = act ? reinterpret_cast<const float4*>(Pf)[off] : z;
    const float4 qq = act ? reinterpret_cast<const float4*>(Nf)[off] : z;
    sc[k] = mil_dot4(pp[k], vv);
    sc[KC + k] = mil_dot4(qq, vv);
  }
  mil_fold<2 * KC>(sc, red);
  // softmax over k of the raw positive scores (AttModel_x3.py:372-373)
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < KC; ++k) mx = fmaxf(mx, sc[k]);
  float den = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k) { sc[k] = expf(sc[k] - mx); den += sc[k]; }
  if (act) {
    float4 o = z;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const float w = sc[k] / den;
      o.x = fmaf(w, pp[k].x, o.x); o.y = fmaf(w, pp[k].y, o.y);
      o.z = fmaf(w, pp[k].z, o.z); o.w = fmaf(w, pp[k].w, o.w);
    }
    reinterpret_cast<float4*>(obj + bn * H)[i] = o;
  }
  if (threadIdx.x == 0) {  // LSE_k(clamp(mask*s-, eps)) (AttModel_x3.py:367)
    float m2 = -INFINITY, sn[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      sn[k] = fmaxf((float)mask[bn * KC + k] * sc[KC + k], eps);
      m2 = fmaxf(m2, sn[k]);
    }
    float s2 = 0.f;
#pragma unroll
    for (int k = 0; k < KC; ++k) s2 += expf(sn[k] - m2);
    term[bn] = (eps + logf((float)KC)) - (m2 + logf(s2));
  }
}

template <int KC, typename TO>
__global__ __launch_bounds__(256) void mil_bwd_split_kernel(
    const float* __restrict__ Pf, const float* __restrict__ Nf, const float* __restrict__ v,
    const int32_t* __restrict__ mask, int64_t BN, int H, float eps,
    const float* __restrict__ dobj, const float* __restrict__ dmil, TO* __restrict__ dPf,
    TO* __restrict__ dNf, float* __restrict__ dv) {
  __shared__ float red[3 * KC][4][64];
  const int64_t bn = blockIdx.x;
  const int i = threadIdx.x, h4 = H / 4;
  const bool act = i < h4;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 vv = act ? reinterpret_cast<const float4*>(v + bn * H)[i] : z;
  const float4 g = act && dobj ? reinterpret_cast<const float4*>(dobj + bn * H)[i] : z;
  float4 pp[KC], qq[KC];
  float sc[3 * KC];  // [0, KC) s+, [KC, 2KC) s-, [2KC, 3KC) dobj . P_k
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int64_t off = (bn * KC + k) * h4 + i;
    pp[k] = act ? reinterpret_cast<const float4*>(Pf)[off] : z;
    qq[k] = act ? reinterpret_cast<const float4*>(Nf)[off] : z;
    sc[k] = mil_dot4(pp[k], vv);
    sc[KC + k] = mil_dot4(qq[k], vv);
    sc[2 * KC + k] = mil_dot4(g, pp[k]);
  }
  mil_fold<3 * KC>(sc, red);
  // softmax weights w and their backward dsp = w*(dw - sum w dw)
  float sp[KC], dsp[KC], dsn[KC];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < KC; ++k) mx = fmaxf(mx, sc[k]);
  float den = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k) { sp[k] = expf(sc[k] - mx); den += sp[k]; }
  float wdw = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k) { sp[k] = sp[k] / den; wdw += sp[k] * sc[2 * KC + k]; }
#pragma unroll
  for (int k = 0; k < KC; ++k) dsp[k] = sp[k] * (sc[2 * KC + k] - wdw);
  // term = LSE(eps) - LSE(snc): d snc_k = -dterm * softmax_k(snc); clamp passes where >= eps
  const float dterm = (*dmil) / (2.f * (float)BN);
  {
    float m2 = -INFINITY, snc[KC], mk[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      mk[k] = (float)mask[bn * KC + k];
      snc[k] = fmaxf(mk[k] * sc[KC + k], eps);
      m2 = fmaxf(m2, snc[k]);
    }
    float s2 = 0.f;
#pragma unroll
    for (int k = 0; k < KC; ++k) { dsn[k] = expf(snc[k] - m2); s2 += dsn[k]; }
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const float d_snc = -dterm * (dsn[k] / s2);
      dsn[k] = (mk[k] * sc[KC + k] >= eps) ? d_snc * mk[k] : 0.f;
    }
  }
  if (!act) return;
  float4 acc = z;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int64_t off = (bn * KC + k) * H + 4 * i;
    const float4 p = pp[k], q = qq[k];
    float4 dp, dn;
    dp.x = p.x > 0.f ? sp[k] * g.x + dsp[k] * vv.x : 0.f;
    dp.y = p.y > 0.f ? sp[k] * g.y + dsp[k] * vv.y : 0.f;
    dp.z = p.z > 0.f ? sp[k] * g.z + dsp[k] * vv.z : 0.f;
    dp.w = p.w > 0.f ? sp[k] * g.w + dsp[k] * vv.w : 0.f;
    dn.x = q.x > 0.f ? dsn[k] * vv.x : 0.f;
    dn.y = q.y > 0.f ? dsn[k] * vv.y : 0.f;
    dn.z = q.z > 0.f ? dsn[k] * vv.z : 0.f;
    dn.w = q.w > 0.f ? dsn[k] * vv.w : 0.f;
    mil_store4(dPf + off, dp);
    mil_store4(dNf + off, dn);
    acc.x += dsp[k] * p.x + dsn[k] * q.x;
    acc.y += dsp[k] * p.y + dsn[k] * q.y;
    acc.z += dsp[k] * p.z + dsn[k] * q.z;
    acc.w += dsp[k] * p.w + dsn[k] * q.w;
  }
  float4 o;
  o.x = vv.x > 0.f ? acc.x : 0.f; o.y = vv.y > 0.f ? acc.y : 0.f;
  o.z = vv.z > 0.f ? acc.z : 0.f; o.w = vv.w > 0.f ? acc.w : 0.f;
  reinterpret_cast<float4*>(dv + bn * H)[i] = o;
}

static bool mil_split_ok(int64_t K, int64_t H) {
  return SAVQA_MIL_SPLIT && K <= MIL_SPLIT_K && H <= MIL_SPLIT_H;
}

#define SAVQA_MIL_K_SWITCH(K, LAUNCH) \
  switch (K) {                        \
    case 1: LAUNCH(1); break;         \
    case 2: LAUNCH(2); break;         \
    case 3: LAUNCH(3); break;         \
    case 4: LAUNCH(4); break;         \
    case 5: LAUNCH(5); break;         \
    case 6: LAUNCH(6); break;         \
    case 7: LAUNCH(7); break;         \
    default: LAUNCH(8); break;        \
  }

// macro[b*Ns + loc[b,n]] = obj[b*Nv + n], n ascending (last write wins, as the
// reference's index_put on CPU); one block per sample keeps that order.
__global__ void index_put_rows_kernel(const int64_t* __restrict__ loc, int64_t Nv, int64_t Ns,
                                      int64_t H, const float* __restrict__ obj,
                                      float* __restrict__ macro) {
  const int64_t b = blockIdx.x;
  for (int64_t n = 0; n < Nv; ++n) {
    const int64_t l = loc[b * Nv + n];
    if (l < 0 || l >= Ns) continue;  // LOC_PAD; an out-of-range location writes nothing
    for (int64_t c = threadIdx.x; c < H; c += blockDim.x)
      macro[(b * Ns + l) * H + c] = obj[(b * Nv + n) * H + c];
    __syncthreads();
  }
}

// Deterministic row scatter-add (savqa_segment_add_rows): one wave per sorted position j;
// the wave at the start of a run of equal ids sums the run's rows of T in run order (the
// stable sort keeps equal ids in their original row order) and adds the sum to the table row
// -- one writer per row, a fixed order, no atomics. Columns in float4s (cols % 4 == 0).
__global__ __launch_bounds__(256) void segment_add_rows_kernel(
    const float* __restrict__ T, int64_t ldt, const int64_t* __restrict__ perm,
    const int64_t* __restrict__ sid, int64_t R, int64_t cols, float* __restrict__ table,
    int64_t ldtab) {
  typedef float v4 __attribute__((ext_vector_type(4)));
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= R) return;
  const int64_t id = sid[j];
  if (j > 0 && sid[j - 1] == id) return;  // not the start of a run (wave-uniform)
  int64_t end = j + 1;
  while (end < R && sid[end] == id) ++end;
  float* dst = table + id * ldtab;
  for (int64_t c = 4 * lane; c < cols; c += 256) {
    v4 acc = *reinterpret_cast<const v4*>(T + perm[j] * ldt + c);
    for (int64_t k = j + 1; k < end; ++k) acc += *reinterpret_cast<const v4*>(T + perm[k] * ldt + c);
    v4* o = reinterpret_cast<v4*>(dst + c);
    *o = *o + acc;
  }
}

__global__ void index_get_rows_kernel(const int64_t* __restrict__ loc, int64_t Nv, int64_t Ns,
                                      int64_t H, const float* __restrict__ dmacro,
                                      float* __restrict__ dobj) {
  const int64_t bn = blockIdx.x;
  const int64_t b = bn / Nv;
  const int64_t l = loc[bn];
  for (int64_t c = threadIdx.x; c < H; c += blockDim.x)
    dobj[bn * H + c] = (l >= 0 && l < Ns) ? dmacro[(b * Ns + l) * H + c] : 0.f;
}

// ------------------------------------------------------------------ loss
// one block per sample; three heads of C logits each.
__global__ __launch_bounds__(256) void loss_kernel(const float* __restrict__ lc,
                                                   const float* __restrict__ lv,
                                                   const float* __restrict__ ls,
                                                   const int64_t* __restrict__ answer, int64_t B,
                                                   int C, float eps, float* __restrict__ dlogits,
                                                   float* __restrict__ lsm_out,
                                                   float* __restrict__ row_loss) {
  __shared__ float red[4];
  __shared__ float stat[6];
  const int64_t b = blockIdx.x;
  const float* heads[3] = {lc + b * C, lv + b * C, ls + b * C};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  auto block_reduce = [&](float v, bool is_max) -> float {
    v = is_max ? wave_max(v) : wave_sum(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < 4; ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
    return r;
  };
  for (int hd = 0; hd < 3; ++hd) {
    float mx = -INFINITY;
    for (int c = threadIdx.x; c < C; c += 256) mx = fmaxf(mx, heads[hd][c]);
    mx = block_reduce(mx, true);
    float s = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) s += expf(heads[hd][c] - mx);
    s = block_reduce(s, false);
    if (threadIdx.x == 0) { stat[2 * hd] = mx; stat[2 * hd + 1] = logf(s); }
  }
  __syncthreads();
  const int64_t ans = answer[b];
  const float off = eps / (float)C;
  float ysum = 0.f, part = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float y = (c == ans ? (1.f - eps) : 0.f) + off;
    // reference order: (vis + syb + concat) / 3
    const float lsv = heads[1][c] - stat[2] - stat[3];
    const float lss = heads[2][c] - stat[4] - stat[5];
    const float lsc = heads[0][c] - stat[0] - stat[1];
    const float l = (lsv + lss + lsc) / 3.f;
    if (lsm_out) lsm_out[b * C + c] = l;
    part += y * l;
    ysum += y;
  }
  part = block_reduce(part, false);
  ysum = block_reduce(ysum, false);
  const float k = -1.f / (3.f * (float)B);
  for (int c = threadIdx.x; c < C; c += 256) {
    const float y = (c == ans ? (1.f - eps) : 0.f) + off;
    for (int hd = 0; hd < 3; ++hd) {
      const float p = expf(heads[hd][c] - stat[2 * hd] - stat[2 * hd + 1]);
      dlogits[((int64_t)hd * B + b) * C + c] = k * (y - p * ysum);
    }
  }
  if (threadIdx.x == 0) row_loss[b] = -part;
}

__global__ void loss_final_kernel(const float* __restrict__ row_loss, int64_t B,
                                  const float* __restrict__ mil, int with_mil,
                                  float* __restrict__ loss) {
  __shared__ float part[4];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < B; i += blockDim.x) s += row_loss[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = part[0] + part[1] + part[2] + part[3];
    t = t / (float)B;
    if (with_mil) t = t + (-(*mil));
    *loss = t;
  }
}

__global__ void scale_by_kernel(const float* __restrict__ in, const float* __restrict__ scale,
                                int64_t n, float* __restrict__ out) {
  const float s = *scale;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = in[i] * s;
}

// out = in * rowscale[row] * (mask > 0)   (ReLU backward of a row-gated activation)
__global__ void rowscale_mask_kernel(const float* __restrict__ in, const float* __restrict__ rs,
                                     const float* __restrict__ mask, int64_t rows, int64_t cols,
                                     float* __restrict__ out) {
  const int64_t n = rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / cols;
    float v = in[i];
    if (rs) v *= rs[r];
    if (mask && !(mask[i] > 0.f)) v = 0.f;
    out[i] = v;
  }
}

// out = a*in + b  (label_smoothing, modules.py:461-463)
__global__ void affine_kernel(const float* __restrict__ in, int64_t n, float a, float b,
                              float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = a * in[i] + b;
}

// out[r][:] = table[idx[r]][:] * scale   (embedding.forward, modules.py:40-43)
__global__ void gather_rows_kernel(const float* __restrict__ table, const int64_t* __restrict__ idx,
                                   int64_t rows, int64_t cols, float scale, float* __restrict__ out) {
  const int64_t r = blockIdx.x;
  const int64_t t = idx[r];
  for (int64_t c = threadIdx.x; c < cols; c += blockDim.x) out[r * cols + c] = table[t * cols + c] * scale;
}

// dtable[idx[r]][:] += g[r][:] * scale, skipping padding_idx rows (F.embedding backward)
__global__ void scatter_rows_kernel(const float* __restrict__ g, const int64_t* __restrict__ idx,
                                    int64_t rows, int64_t cols, float scale, int64_t padding_idx,
                                    float* __restrict__ dtable) {
  const int64_t r = blockIdx.x;
  const int64_t t = idx[r];
  if (t == padding_idx) return;
  for (int64_t c = threadIdx.x; c < cols; c += blockDim.x) atomicAdd(&dtable[t * cols + c], g[r * cols + c] * scale);
}

// ------------------------------------------------------------------ Adam
// torch.optim.Adam (foreach=False, amsgrad=False, maximize=False, weight_decay=0):
// m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2; p -= (lr/bc1) m / (sqrt(v)/sqrt(bc2) + eps).
// Streaming, 28 B/param: each thread moves 2 float4 of p, g, m, v per iteration with
// non-temporal loads/stores (11 GB per step at the cfg-2 arena never fits in cache).
// grid cap of the grid-stride Adam launch (A/B knob; round 3, a since-removed Adam micro-bench over 457M params,
// interleaved runs: 8192 blocks 2.17-2.37 ms, 32768 2.05-2.32 ms, i.e. ~4% within noise)
#ifndef SAVQA_ADAM_BLOCKS
#define SAVQA_ADAM_BLOCKS 32768
#endif
typedef float adam_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void adam4(adam_f4& pp, adam_f4 gg, adam_f4& mm, adam_f4& vv, float b1,
                                      float b2, float eps, float step_size, float sbc2, float gs) {
  // no FMA contraction: every launch site (grid-stride body, its tail, the row kernel) must round
  // identically, so a row-tracked step is bit-identical to the dense one
#pragma clang fp contract(off)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float gx = gg[e] * gs;
    mm[e] = mm[e] + (1.f - b1) * (gx - mm[e]);
    vv[e] = b2 * vv[e] + (1.f - b2) * gx * gx;
    const float den = sqrtf(vv[e]) / sbc2 + eps;
    pp[e] = pp[e] - step_size * (mm[e] / den);
  }
}

__device__ __forceinline__ void adam_sh4(__bf16* q, adam_f4 x) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  typedef float f4_ __attribute__((ext_vector_type(4)));
  const f4_ y = {x[0], x[1], x[2], x[3]};
  *reinterpret_cast<bf16x4*>(q) = __builtin_convertvector(y, bf16x4);
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int64_t n, float lr, float b1, float b2,
                                                   float eps, float step_size, float sbc2,
                                                   float gs, __bf16* __restrict__ sh) {
  // sh (optional): the bf16 image of p (the low-precision modes' weight shadow), written from
  // the updated values in the same pass instead of a separate cast that re-reads p
  (void)lr;
  const int64_t n4 = n / 4;
  adam_f4* P = reinterpret_cast<adam_f4*>(p);
  const adam_f4* Gv = reinterpret_cast<const adam_f4*>(g);
  adam_f4* M = reinterpret_cast<adam_f4*>(m);
  adam_f4* V = reinterpret_cast<adam_f4*>(v);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const int64_t j = i + stride;
    adam_f4 p0 = __builtin_nontemporal_load(P + i), p1 = __builtin_nontemporal_load(P + j);
    const adam_f4 g0 = __builtin_nontemporal_load(Gv + i), g1 = __builtin_nontemporal_load(Gv + j);
    adam_f4 m0 = __builtin_nontemporal_load(M + i), m1 = __builtin_nontemporal_load(M + j);
    adam_f4 v0 = __builtin_nontemporal_load(V + i), v1 = __builtin_nontemporal_load(V + j);
    adam4(p0, g0, m0, v0, b1, b2, eps, step_size, sbc2, gs);
    adam4(p1, g1, m1, v1, b1, b2, eps, step_size, sbc2, gs);
    __builtin_nontemporal_store(p0, P + i); __builtin_nontemporal_store(p1, P + j);
    __builtin_nontemporal_store(m0, M + i); __builtin_nontemporal_store(m1, M + j);
    __builtin_nontemporal_store(v0, V + i); __builtin_nontemporal_store(v1, V + j);
    if (sh) {
      adam_sh4(sh + 4 * i, p0);
      adam_sh4(sh + 4 * j, p1);
    }
  }
  if (i < n4) {
    adam_f4 p0 = P[i], m0 = M[i], v0 = V[i];
    adam4(p0, Gv[i], m0, v0, b1, b2, eps, step_size, sbc2, gs);
    P[i] = p0; M[i] = m0; V[i] = v0;
    if (sh) adam_sh4(sh + 4 * i, p0);
  }
  {  // scalar tail (same roundings as adam4)
#pragma clang fp contract(off)
    for (int64_t k = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
      const float gx = g[k] * gs;
      m[k] = m[k] + (1.f - b1) * (gx - m[k]);
      v[k] = b2 * v[k] + (1.f - b2) * gx * gx;
      const float den = sqrtf(v[k]) / sbc2 + eps;
      p[k] = p[k] - step_size * (m[k] / den);
      if (sh) sh[k] = (__bf16)p[k];
    }
  }
}


// ------------------------------------------------------------------ row-tracked tables
// The three 407000 x 300 GloVe tables (AttModel_x3.py:36-41, :168-171, :295) receive gradient
// rows only for the token ids of the step. Per table row a flag byte: bit 0 = the row has
// Adam state (it was touched at some step), bit 1 = the row was touched since the last
// zero_rows (its gradient may be non-zero). A never-touched row has m = v = 0 and g = 0, so
// torch.optim.Adam leaves p, m and v exactly unchanged there: skipping it is bit-exact. A row
// with state but no gradient this step still decays (g = 0 is not read).
constexpr int ROW_EVER = 1, ROW_CUR = 2;

__global__ __launch_bounds__(256) void mark_rows_kernel(const int64_t* __restrict__ ids, int64_t n,
                                                        int64_t nrows, uint8_t* __restrict__ flags) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = ids[i];
    if (r >= 0 && r < nrows) flags[r] |= ROW_CUR;  // every writer stores old | CUR: no race
  }
}

// One wave per 64 rows: lane l reads flag byte (r0 + l); the wave then walks the flagged rows
// of its group (ballot), each row as `width` floats spread over the 64 lanes (float4 when the
// row is 16-B aligned).
template <bool VEC>
__device__ __forceinline__ void zero_row(float* __restrict__ row, int64_t width, int lane) {
  if (VEC) {
    adam_f4* r4 = reinterpret_cast<adam_f4*>(row);
    for (int64_t c = lane; c < width / 4; c += 64) r4[c] = adam_f4{0.f, 0.f, 0.f, 0.f};
  } else {
    for (int64_t c = lane; c < width; c += 64) row[c] = 0.f;
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void zero_rows_kernel(float* __restrict__ g, int64_t width,
                                                        int64_t nrows, uint8_t* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  if (r0 >= nrows) return;
  const int64_t r = r0 + lane;
  const uint8_t f = r < nrows ? flags[r] : 0;
  uint64_t todo = __ballot((f & ROW_CUR) != 0);
  while (todo) {
    const int l = __builtin_ctzll(todo);
    todo &= todo - 1;
    zero_row<VEC>(g + (r0 + l) * width, width, lane);
  }
  if (f & ROW_CUR) flags[r] = f & ~ROW_CUR;
}

template <bool VEC>
__global__ __launch_bounds__(256) void adam_rows_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        int64_t width, int64_t nrows,
                                                        uint8_t* __restrict__ flags, float b1, float b2,
                                                        float eps, float step_size, float sbc2,
                                                        float gs) {
  const int lane = threadIdx.x & 63;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  if (r0 >= nrows) return;
  const int64_t r = r0 + lane;
  const uint8_t f = r < nrows ? flags[r] : 0;
  uint64_t todo = __ballot(f != 0);
  const uint64_t cur = __ballot((f & ROW_CUR) != 0);
  while (todo) {
    const int l = __builtin_ctzll(todo);
    todo &= todo - 1;
    const int64_t o = (r0 + l) * width;
    const bool has_g = (cur >> l) & 1;
    if (VEC) {
      adam_f4* P = reinterpret_cast<adam_f4*>(p + o);
      const adam_f4* G = reinterpret_cast<const adam_f4*>(g + o);
      adam_f4* M = reinterpret_cast<adam_f4*>(m + o);
      adam_f4* V = reinterpret_cast<adam_f4*>(v + o);
      for (int64_t c = lane; c < width / 4; c += 64) {
        adam_f4 pp = P[c], mm = M[c], vv = V[c];
        const adam_f4 gg = has_g ? G[c] : adam_f4{0.f, 0.f, 0.f, 0.f};
        adam4(pp, gg, mm, vv, b1, b2, eps, step_size, sbc2, gs);
        P[c] = pp; M[c] = mm; V[c] = vv;
      }
    } else {
      for (int64_t c = lane; c < width; c += 64) {
        const float gx = has_g ? g[o + c] * gs : 0.f;
        float mm = m[o + c], vv = v[o + c];
        mm = mm + (1.f - b1) * (gx - mm);
        vv = b2 * vv + (1.f - b2) * gx * gx;
        const float den = sqrtf(vv) / sbc2 + eps;
        m[o + c] = mm; v[o + c] = vv;
        p[o + c] = p[o + c] - step_size * (mm / den);
      }
    }
  }
  if (f & ROW_CUR) flags[r] = f | ROW_EVER;
}
}  // namespace savqa

using namespace savqa;

extern "C" int savqa_graph_build(void* stream, const int32_t* node_mask, const int32_t* q_mask,
                                 const int32_t* q_graph, const int32_t* node_graph, int64_t B,
                                 int64_t Nn, int64_t Lq, int32_t dec_mask_on, float* graph_diag,
                                 float* graph, float* dec_mask) {
  if (B <= 0) return 0;
  if (Nn < 0 || Lq <= 0) return fail(SAVQA_EINVAL, "savqa_graph_build: bad sizes");
  const int64_t T = Nn + Lq;
  hipLaunchKernelGGL(graph_build_kernel, dim3(B * T), dim3(T <= 64 ? 64 : (T <= 128 ? 128 : 256)),
                     0, as_stream(stream), node_mask, q_mask, q_graph, node_graph, (int)Nn,
                     (int)Lq, dec_mask_on, graph_diag, graph, dec_mask);
  return check_launch("savqa_graph_build");
}

extern "C" int savqa_dec_init(void* stream, const float* emb, int64_t idx, float scale,
                              const float* pos, int64_t B, int64_t d, uint64_t seed, int32_t site,
                              float p, float* out) {
  const int64_t n = B * d;
  if (n <= 0) return 0;
  if (p < 0.f || p > 1.f) return fail(SAVQA_EINVAL, "savqa_dec_init: p outside [0,1]");
  hipLaunchKernelGGL(dec_init_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), emb,
                     idx, scale, pos, B, d, make_drop(seed, p), p > 0.f ? site : -1, out);
  return check_launch("savqa_dec_init");
}

extern "C" int savqa_dec_init_bwd(void* stream, const float* g, int64_t B, int64_t d, int64_t idx,
                                  float scale, uint64_t seed, int32_t site, float p, float* demb,
                                  float* dpos) {
  if (B <= 0 || d <= 0) return 0;
  if (p < 0.f || p > 1.f) return fail(SAVQA_EINVAL, "savqa_dec_init_bwd: p outside [0,1]");
  hipLaunchKernelGGL(dec_init_bwd_kernel, dim3((unsigned)((d + DIB_COLS - 1) / DIB_COLS)), dim3(256), 0,
                     as_stream(stream), g,
                     B, d, idx, scale, make_drop(seed, p), p > 0.f ? site : -1, demb, dpos);
  return check_launch("savqa_dec_init_bwd");
}

extern "C" int savqa_period_sum_acc(void* stream, const float* X, int64_t B, int64_t T, int64_t C,
                                    int64_t ldx, float* out) {
  if (B <= 0 || T <= 0 || C <= 0) return 0;
  hipLaunchKernelGGL(period_sum_kernel, dim3((C + 255) / 256, T), dim3(256), 0, as_stream(stream),
                     X, B, T, C, ldx, out);
  return check_launch("savqa_period_sum_acc");
}

extern "C" int savqa_copy_rows(void* stream, const float* src, int64_t rows, int64_t cols,
                               int64_t lds, float* dst, int64_t ldd, int64_t group, int64_t stride,
                               int64_t offset) {
  if (rows <= 0 || cols <= 0) return 0;
  if (group <= 0) { group = rows; stride = rows; }
  hipLaunchKernelGGL(copy_rows_kernel, dim3(rows), dim3(256), 0, as_stream(stream), src, rows, cols,
                     lds, dst, ldd, group, stride, offset);
  return check_launch("savqa_copy_rows");
}

extern "C" int savqa_mil_fwd(void* stream, const float* Pf, const float* Nf, const float* v,
                             const int32_t* mask, int64_t BN, int64_t K, int64_t H, float eps,
                             float* obj, float* ws, float* mil_out) {
  if (BN <= 0) return 0;
  if (K <= 0 || K > MIL_KMAX || H % 4 != 0)
    return fail(SAVQA_EUNSUP, "savqa_mil_fwd: need 1 <= topN <= 16 and H % 4 == 0");
  hipStream_t s = as_stream(stream);
  if (mil_split_ok(K, H)) {
#define SAVQA_MIL_FWD(KC)                                                                     \
  hipLaunchKernelGGL((mil_fwd_split_kernel<KC>), dim3((unsigned)BN), dim3(256), 0, s, Pf, Nf, v, \
                     mask, (int)H, eps, obj, ws)
    SAVQA_MIL_K_SWITCH(K, SAVQA_MIL_FWD)
#undef SAVQA_MIL_FWD
  } else {
    hipLaunchKernelGGL(mil_fwd_kernel, dim3((BN + 3) / 4), dim3(256), 0, s, Pf, Nf, v, mask, BN,
                       (int)K, (int)H, eps, obj, ws);
  }
  hipLaunchKernelGGL(mean_reduce_kernel, dim3(1), dim3(1024), 0, s, ws, BN, 1.f / (2.f * (float)BN),
                     mil_out);
  return check_launch("savqa_mil_fwd");
}

template <typename TO>
static int mil_bwd_launch(hipStream_t s, const float* Pf, const float* Nf, const float* v,
                          const int32_t* mask, int64_t BN, int64_t K, int64_t H, float eps,
                          const float* dobj, const float* dmil, TO* dPf, TO* dNf, float* dv,
                          const char* who) {
  if (mil_split_ok(K, H)) {
#define SAVQA_MIL_BWD(KC)                                                                      \
  hipLaunchKernelGGL((mil_bwd_split_kernel<KC, TO>), dim3((unsigned)BN), dim3(256), 0, s, Pf, Nf, \
                     v, mask, BN, (int)H, eps, dobj, dmil, dPf, dNf, dv)
    SAVQA_MIL_K_SWITCH(K, SAVQA_MIL_BWD)
#undef SAVQA_MIL_BWD
  } else {
    hipLaunchKernelGGL(mil_bwd_kernel<TO>, dim3((BN + 3) / 4), dim3(256), 0, s, Pf, Nf, v, mask, BN,
                       (int)K, (int)H, eps, dobj, dmil, dPf, dNf, dv);
  }
  return check_launch(who);
}

extern "C" int savqa_mil_bwd(void* stream, const float* Pf, const float* Nf, const float* v,
                             const int32_t* mask, int64_t BN, int64_t K, int64_t H, float eps,
                             const float* dobj, const float* dmil, float* dPf, float* dNf,
                             float* dv) {
  if (BN <= 0) return 0;
  if (K <= 0 || K > MIL_KMAX || H % 4 != 0)
    return fail(SAVQA_EUNSUP, "savqa_mil_bwd: need 1 <= topN <= 16 and H % 4 == 0");
  return mil_bwd_launch<float>(as_stream(stream), Pf, Nf, v, mask, BN, K, H, eps, dobj, dmil, dPf,
                               dNf, dv, "savqa_mil_bwd");
}

extern "C" int savqa_mil_bwd_bf16(void* stream, const float* Pf, const float* Nf, const float* v,
                                  const int32_t* mask, int64_t BN, int64_t K, int64_t H, float eps,
                                  const float* dobj, const float* dmil, void* dPf, void* dNf,
                                  float* dv) {
  if (BN <= 0) return 0;
  if (K <= 0 || K > MIL_KMAX || H % 4 != 0)
    return fail(SAVQA_EUNSUP, "savqa_mil_bwd_bf16: need 1 <= topN <= 16 and H % 4 == 0");
  return mil_bwd_launch<__bf16>(as_stream(stream), Pf, Nf, v, mask, BN, K, H, eps, dobj, dmil,
                                static_cast<__bf16*>(dPf), static_cast<__bf16*>(dNf), dv,
                                "savqa_mil_bwd_bf16");
}

extern "C" int savqa_index_put_rows(void* stream, const int64_t* loc, int64_t B, int64_t Nv,
                                    int64_t Ns, int64_t H, const float* obj, float* macro) {
  if (B <= 0 || Nv <= 0) return 0;
  hipLaunchKernelGGL(index_put_rows_kernel, dim3(B), dim3(256), 0, as_stream(stream), loc, Nv, Ns, H,
                     obj, macro);
  return check_launch("savqa_index_put_rows");
}

extern "C" int savqa_segment_add_rows(void* stream, const float* T, int64_t ldt,
                                      const int64_t* perm, const int64_t* sid, int64_t R,
                                      int64_t cols, float* table, int64_t ldtab) {
  if (R <= 0 || cols <= 0) return 0;
  if (cols % 4 || ldt % 4 || ldtab % 4 || ((uintptr_t)T & 15) || ((uintptr_t)table & 15))
    return fail(SAVQA_EUNSUP, "savqa_segment_add_rows: needs 16-B aligned rows (cols, ldt, "
                              "ldtab multiples of 4)");
  hipLaunchKernelGGL(segment_add_rows_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0,
                     as_stream(stream), T, ldt, perm, sid, R, cols, table, ldtab);
  return check_launch("savqa_segment_add_rows");
}

extern "C" int savqa_index_get_rows(void* stream, const int64_t* loc, int64_t B, int64_t Nv,
                                    int64_t Ns, int64_t H, const float* dmacro, float* dobj) {
  if (B <= 0 || Nv <= 0) return 0;
  hipLaunchKernelGGL(index_get_rows_kernel, dim3(B * Nv), dim3(256), 0, as_stream(stream), loc, Nv,
                     Ns, H, dmacro, dobj);
  return check_launch("savqa_index_get_rows");
}

extern "C" int savqa_loss_fwd(void* stream, const float* lc, const float* lv, const float* ls,
                              const int64_t* answer, int64_t B, int64_t C, float eps,
                              const float* mil, int32_t with_mil, float* loss, float* dlogits,
                              float* lsm, float* ws) {
  if (B <= 0) return fail(SAVQA_EINVAL, "savqa_loss_fwd: empty batch");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(loss_kernel, dim3(B), dim3(256), 0, s, lc, lv, ls, answer, B, (int)C, eps,
                     dlogits, lsm, ws);
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, s, ws, B, mil, with_mil, loss);
  return check_launch("savqa_loss_fwd");
}

extern "C" int savqa_scale_by(void* stream, const float* in, const float* scale, int64_t n,
                              float* out) {
  if (n <= 0) return 0;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(scale_by_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), in, scale, n,
                     out);
  return check_launch("savqa_scale_by");
}

extern "C" int savqa_adam_shadow(void* stream, float* p, const float* g, float* m, float* v,
                                 int64_t n, float lr, float beta1, float beta2, float eps,
                                 float bc1, float bc2, float grad_scale, void* shadow) {
  if (n <= 0) return 0;
  if ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) != 0)
    return fail(SAVQA_EINVAL, "savqa_adam: buffers must be 16-B aligned");
  if (((uintptr_t)shadow & 7) != 0)
    return fail(SAVQA_EINVAL, "savqa_adam_shadow: the bf16 shadow must be 8-B aligned");
  const float step_size = lr / bc1;
  const float sbc2 = sqrtf(bc2);
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks > SAVQA_ADAM_BLOCKS) blocks = SAVQA_ADAM_BLOCKS;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), p, g, m, v, n, lr,
                     beta1, beta2, eps, step_size, sbc2, grad_scale, static_cast<__bf16*>(shadow));
  return check_launch("savqa_adam");
}

extern "C" int savqa_adam(void* stream, float* p, const float* g, float* m, float* v, int64_t n,
                          float lr, float beta1, float beta2, float eps, float bc1, float bc2,
                          float grad_scale) {
  return savqa_adam_shadow(stream, p, g, m, v, n, lr, beta1, beta2, eps, bc1, bc2, grad_scale,
                           nullptr);
}

static unsigned rows_grid(int64_t nrows) { return (unsigned)((nrows + 255) / 256); }

extern "C" int savqa_mark_rows(void* stream, const int64_t* ids, int64_t n, int64_t nrows,
                               uint8_t* flags) {
  if (n <= 0) return 0;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(mark_rows_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), ids, n, nrows,
                     flags);
  return check_launch("savqa_mark_rows");
}

extern "C" int savqa_zero_rows(void* stream, float* g, int64_t width, int64_t nrows, uint8_t* flags) {
  if (nrows <= 0) return 0;
  if (width % 4 == 0 && (((uintptr_t)g) & 15) == 0)
    hipLaunchKernelGGL(zero_rows_kernel<true>, dim3(rows_grid(nrows)), dim3(256), 0,
                       as_stream(stream), g, width, nrows, flags);
  else
    hipLaunchKernelGGL(zero_rows_kernel<false>, dim3(rows_grid(nrows)), dim3(256), 0,
                       as_stream(stream), g, width, nrows, flags);
  return check_launch("savqa_zero_rows");
}

extern "C" int savqa_adam_rows(void* stream, float* p, const float* g, float* m, float* v,
                               int64_t width, int64_t nrows, uint8_t* flags, float lr,
                               float beta1, float beta2, float eps, float bc1, float bc2,
                               float grad_scale) {
  if (nrows <= 0) return 0;
  const float step_size = lr / bc1, sbc2 = sqrtf(bc2);
  const bool vec = width % 4 == 0 && ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) |
                                        ((uintptr_t)v)) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(adam_rows_kernel<true>, dim3(rows_grid(nrows)), dim3(256), 0,
                       as_stream(stream), p, g, m, v, width, nrows, flags, beta1, beta2, eps,
                       step_size, sbc2, grad_scale);
  else
    hipLaunchKernelGGL(adam_rows_kernel<false>, dim3(rows_grid(nrows)), dim3(256), 0,
                       as_stream(stream), p, g, m, v, width, nrows, flags, beta1, beta2, eps,
                       step_size, sbc2, grad_scale);
  return check_launch("savqa_adam_rows");
}

extern "C" int savqa_rowscale_mask(void* stream, const float* in, const float* rowscale,
                                   const float* mask, int64_t rows, int64_t cols, float* out) {
  const int64_t n = rows * cols;
  if (n <= 0) return 0;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(rowscale_mask_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), in,
                     rowscale, mask, rows, cols, out);
  return check_launch("savqa_rowscale_mask");
}

namespace savqa {
__global__ void axpby_kernel(const float* __restrict__ x, const float* __restrict__ y, int64_t n,
                             float a, float b, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a * x[i] + b * y[i];
}
}  // namespace savqa

extern "C" int savqa_axpby(void* stream, const float* x, const float* y, int64_t n, float a,
                           float b, float* out) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(axpby_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), x, y, n, a, b, out);
  return check_launch("savqa_axpby");
}

extern "C" int savqa_affine(void* stream, const float* in, int64_t n, float a, float b, float* out) {
  if (n <= 0) return 0;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(affine_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), in, n, a, b, out);
  return check_launch("savqa_affine");
}

extern "C" int savqa_gather_rows(void* stream, const float* table, const int64_t* idx, int64_t rows,
                                 int64_t cols, float scale, float* out) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(rows), dim3(cols >= 256 ? 256 : 64), 0,
                     as_stream(stream), table, idx, rows, cols, scale, out);
  return check_launch("savqa_gather_rows");
}

extern "C" int savqa_scatter_rows(void* stream, const float* g, const int64_t* idx, int64_t rows,
                                  int64_t cols, float scale, int64_t padding_idx, float* dtable) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(scatter_rows_kernel, dim3(rows), dim3(cols >= 256 ? 256 : 64), 0,
                     as_stream(stream), g, idx, rows, cols, scale, padding_idx, dtable);
  return check_launch("savqa_scatter_rows");
}
