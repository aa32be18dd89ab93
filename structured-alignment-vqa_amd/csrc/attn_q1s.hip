// Single-query graph attention over long key sequences, split over keys: the decoder's
// cross-attention (models/AttModel_x3.py:279, new_multihead_attention modules.py:236-311 with
// T_q = 1) at T_k > 128 -- the super-node relation workload (T_k = 1314) and cfg 4 (449).
// The key-tiled kernels (attn_flash.hip) tile 64 queries, so with one query they ran one
// workgroup per (sample, head): 32 workgroups on 256 CUs at B = 4. Here every wave takes 64
// keys of one (sample, head), so a launch has B * H * ceil(T_k / 64) waves.
//
// Forward, per (b, h) with scores x_j = q.k_j / 8 (ATT_MASKED where the key row is masked),
// graph weights g_j, key split s:
//   partial: m_s = max x, Z_s = sum e^(x - m_s), W_s = sum |g| e^(x - m_s),
//            U_s = sum g e^(x - m_s) v_j                                    (q1s_fwd_part)
//   combine: m = max m_s, Z = sum Z_s e^(m_s - m), W, U likewise;
//            nrm = W / Z (= sum_j |g_j P_j|, P the softmax over ALL keys), O = U / Z /
//            max(nrm, 1e-12) * qflag; (m, Z, nrm) saved for the backward    (q1s_fwd_combine)
// Backward (the single-query kernel's chain, attn.hip gattn_bwd_q1_kernel, with its two
// whole-row sums taken over the splits): dn_j = (dO.v_j) qflag, bm_j = g_j P_j,
//   t1 = sum_j dn_j bm_j (fp64, fixed order over the splits); dV_j        (q1s_bwd_dv)
//   dnrm = -t1 / sden^2 (0 in F.normalize's clamped branch), da_j = g_j (dn_j / sden + dnrm
//   sgn bm_j), t2 = sum_j da_j P_j = t1 / sden + dnrm nrm (closed form), ds_j = P_j (da_j -
//   t2) / 8; dK_j = ds_j q, dV_j = (bm_j / sden) qflag dO, dQ = sum_j ds_j k_j, each through
//   its ReLU mask (Q / K / V are ReLU outputs)                              (q1s_bwd_main,
//   q1s_bwd_dq: the per-split dQ partials summed in a fixed order)
// Lane layout (as attn.hip's single-query kernels): lane (kk = lane >> 4, c = lane & 15)
// holds float4 c of key row 4 it + kk, so each K / V load instruction reads 4 whole 256-B
// rows, and a 16-lane DPP reduction finishes each dot product.
#include "attn_common.h"

#include <algorithm>
#include <string>

namespace savqa {

#ifndef SAVQA_Q1S_KEYS
#define SAVQA_Q1S_KEYS 64
#endif
constexpr int QS_KEYS = SAVQA_Q1S_KEYS;  // keys per wave (one split)
constexpr int QS_IT = QS_KEYS / 4;     // 4 key rows per load instruction
constexpr int QS_PART = 4 + ATT_DK;    // floats per forward partial: m, Z, W, pad, U[64]

struct Q1sArgs {
  AttnArgs a;
  int ns;             // splits per (b, h)
  float* stats;       // [B * H][4]: m, Z, nrm
  float* part;        // forward partials [B * H * ns][QS_PART]
  double* t1;         // backward: [B * H * ns]
  float* dqp;         // backward: dQ partials [B * H * ns][64]
  float* pdn;         // backward: (P_j, dn_j) of every key [B * H * ns][QS_KEYS][2]
};

__device__ __forceinline__ float rows4_max_s(float v) {
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}
__device__ __forceinline__ float rows4_sum_s(float v) {
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ f4v xrow_sum_s(f4v v) {  // sum over the 4 key rows of a lane's c
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] += __shfl_xor(v[e], 16);
    v[e] += __shfl_xor(v[e], 32);
  }
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// the wave's (b, h, split) from the grid: blocks of 4 waves over consecutive splits
__device__ __forceinline__ bool q1s_unit(const Q1sArgs& p, int& b, int& h, int& s) {
  const int w = threadIdx.x >> 6;
  const int nsb = (p.ns + 3) >> 2;
  const int bh = blockIdx.x / nsb;
  s = (blockIdx.x - bh * nsb) * 4 + w;
  b = bh / p.a.H;
  h = bh - b * p.a.H;
  return s < p.ns;
}

// scores of the wave's 64 keys (-inf past T_k)
__device__ __forceinline__ void q1s_scores(const AttnArgs& a, int64_t kb, int j0, int hd, int kk,
                                           int c, f4v q4, float (&x)[QS_IT]) {
#pragma unroll
  for (int it = 0; it < QS_IT; ++it) {
    const int j = j0 + 4 * it + kk;
    const f4v k4 = ld4(a.k + (kb + min(j, a.Tk - 1)) * a.ldk + hd + 4 * c);
    const float d = row16_sum((q4.x * k4.x + q4.y * k4.y) + (q4.z * k4.z + q4.w * k4.w));
    x[it] = j < a.Tk ? (a.kflag[kb + j] == 0.f ? ATT_MASKED : d * 0.125f) : -INFINITY;
  }
}

__global__ __launch_bounds__(256) void q1s_fwd_part_kernel(Q1sArgs p) {
  int b, h, s;
  if (!q1s_unit(p, b, h, s)) return;  // wave-uniform
  const AttnArgs& a = p.a;
  const int lane = threadIdx.x & 63, kk = lane >> 4, c = lane & 15, hd = h * ATT_DK;
  const int64_t kb = (int64_t)b * a.Tk;
  const int j0 = s * QS_KEYS;
  const f4v q4 = ld4(a.q + (int64_t)b * a.ldq + hd + 4 * c);
  f4v v4[QS_IT];  // V rows issued with the K rows: one memory round trip per wave
#pragma unroll
  for (int it = 0; it < QS_IT; ++it)
    v4[it] = ld4(a.v + (kb + min(j0 + 4 * it + kk, a.Tk - 1)) * a.ldv + hd + 4 * c);
  float x[QS_IT];
  q1s_scores(a, kb, j0, hd, kk, c, q4, x);
  float mx = -INFINITY;
#pragma unroll
  for (int it = 0; it < QS_IT; ++it) mx = fmaxf(mx, x[it]);
  mx = rows4_max_s(mx);
  float z = 0.f, w = 0.f;
  f4v u = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < QS_IT; ++it) {
    const int j = j0 + 4 * it + kk;
    const float e = j < a.Tk ? expf(x[it] - mx) : 0.f;
    const float gj = j < a.Tk ? a.G[kb + j] : 0.f;
    z += e;
    w += fabsf(gj) * e;
    u += (gj * e) * v4[it];
  }
  z = rows4_sum_s(z);
  w = rows4_sum_s(w);
  u = xrow_sum_s(u);
  float* rec = p.part + ((int64_t)(b * a.H + h) * p.ns + s) * QS_PART;
  if (lane == 0) *reinterpret_cast<f4v*>(rec) = f4v{mx, z, w, 0.f};
  if (kk == 0) *reinterpret_cast<f4v*>(rec + 4 + 4 * c) = u;
}

// one wave per (b, h): the split statistics a lane per split (64 at a time), then lane d
// combines dimension d of U -- every load of a pass issued before its sums (latency-bound
// otherwise: one dependent L2 round trip per split)
__global__ __launch_bounds__(256) void q1s_fwd_combine_kernel(Q1sArgs p) {
  const AttnArgs& a = p.a;
  const int bh = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bh >= a.B * a.H) return;
  const int lane = threadIdx.x & 63;
  const int b = bh / a.H, h = bh - b * a.H;
  const float* rec = p.part + (int64_t)bh * p.ns * QS_PART;
  float m = -INFINITY;
  for (int s0 = 0; s0 < p.ns; s0 += 64)
    if (s0 + lane < p.ns) m = fmaxf(m, rec[(s0 + lane) * QS_PART]);
  m = wave_max(m);
  float z = 0.f, w = 0.f, u = 0.f;
  for (int s0 = 0; s0 < p.ns; s0 += 64) {
    float sc = 0.f;
    if (s0 + lane < p.ns) {
      const f4v st = *reinterpret_cast<const f4v*>(rec + (s0 + lane) * QS_PART);
      sc = expf(st[0] - m);
      z += st[1] * sc;
      w += st[2] * sc;
    }
    const int n = min(64, p.ns - s0);
    for (int r0 = 0; r0 < n; r0 += 16) {
      float uv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float x = rec[(s0 + min(r0 + r, n - 1)) * QS_PART + 4 + lane];
        uv[r] = r0 + r < n ? x : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) u += uv[r] * __shfl(sc, r0 + r);
    }
  }
  z = wave_sum(z);
  w = wave_sum(w);
  const float nrm = w / z;
  const float sden = fmaxf(nrm, 1e-12f);
  a.o[(int64_t)b * a.ldo + h * ATT_DK + lane] = u / z / sden * a.qflag[b];
  if (lane == 0) *reinterpret_cast<f4v*>(p.stats + 4 * bh) = f4v{m, z, nrm, 0.f};
}

// per split: P_j (the forward's row max and denominator), dn_j = (dO . v_j) qflag, dV_j =
// (g_j P_j / sden) qflag dO through V's ReLU mask (needs only forward statistics), the partial
// of t1 = sum_j dn_j g_j P_j (fp64), and (P_j, dn_j) kept for q1s_bwd_main
__global__ __launch_bounds__(256) void q1s_bwd_dv_kernel(Q1sArgs p) {
  int b, h, s;
  if (!q1s_unit(p, b, h, s)) return;
  const AttnArgs& a = p.a;
  const int lane = threadIdx.x & 63, kk = lane >> 4, c = lane & 15, hd = h * ATT_DK;
  const int bh = b * a.H + h;
  const int64_t kb = (int64_t)b * a.Tk;
  const int j0 = s * QS_KEYS;
  const f4v st = *reinterpret_cast<const f4v*>(p.stats + 4 * bh);
  const float sden = fmaxf(st[2], 1e-12f);
  const float qf = a.qflag[b];
  const f4v q4 = ld4(a.q + (int64_t)b * a.ldq + hd + 4 * c);
  const f4v do4 = ld4(a.dout + (int64_t)b * a.lddo + hd + 4 * c);
  f4v v4[QS_IT];
#pragma unroll
  for (int it = 0; it < QS_IT; ++it)
    v4[it] = ld4(a.v + (kb + min(j0 + 4 * it + kk, a.Tk - 1)) * a.ldv + hd + 4 * c);
  float x[QS_IT];
  q1s_scores(a, kb, j0, hd, kk, c, q4, x);
  const bool vv = vec_rows(a.dv, a.lddv);
  float* pdn = p.pdn + ((int64_t)bh * p.ns + s) * QS_KEYS * 2;
  double t = 0.0;
#pragma unroll
  for (int it = 0; it < QS_IT; ++it) {
    const int j = j0 + 4 * it + kk;
    const float dn =
        row16_sum((do4.x * v4[it].x + do4.y * v4[it].y) + (do4.z * v4[it].z + do4.w * v4[it].w)) * qf;
    if (j < a.Tk) {
      const float P = expf(x[it] - st[0]) / st[1];
      const float bm = a.G[kb + j] * P;
      if (c == 0) {
        t += (double)dn * (double)bm;
        *reinterpret_cast<float2*>(pdn + 2 * (4 * it + kk)) = make_float2(P, dn);
      }
      const float pj = bm / sden * qf;
      f4v gv;
#pragma unroll
      for (int e = 0; e < 4; ++e) gv[e] = v4[it][e] > 0.f ? pj * do4[e] : 0.f;
      stx4(a.dv + (kb + j) * a.lddv + hd + 4 * c, gv, vv);
    }
  }
  t = wave_sum_d(t);
  if (lane == 0) p.t1[(int64_t)bh * p.ns + s] = t;
}

// per split: ds_j from (P_j, dn_j) and the whole-row t1, dK_j = ds_j q through K's ReLU mask,
// and the split's dQ partial sum_j ds_j k_j
__global__ __launch_bounds__(256) void q1s_bwd_main_kernel(Q1sArgs p) {
  int b, h, s;
  if (!q1s_unit(p, b, h, s)) return;
  const AttnArgs& a = p.a;
  const int lane = threadIdx.x & 63, kk = lane >> 4, c = lane & 15, hd = h * ATT_DK;
  const int bh = b * a.H + h;
  const int64_t kb = (int64_t)b * a.Tk;
  const int j0 = s * QS_KEYS;
  f4v k4[QS_IT];
#pragma unroll
  for (int it = 0; it < QS_IT; ++it)
    k4[it] = ld4(a.k + (kb + min(j0 + 4 * it + kk, a.Tk - 1)) * a.ldk + hd + 4 * c);
  const float nrm = p.stats[4 * bh + 2], sden = fmaxf(nrm, 1e-12f);
  double t1 = 0.0;  // lane r holds split r (64 at a time); the butterfly sum is the same in
  for (int r0 = 0; r0 < p.ns; r0 += 64)  // every wave of (b, h)
    if (r0 + lane < p.ns) t1 += p.t1[(int64_t)bh * p.ns + r0 + lane];
  t1 = wave_sum_d(t1);
  const double dnrm_d = nrm >= 1e-12f ? -t1 / ((double)sden * (double)sden) : 0.0;
  const float dnrm = (float)dnrm_d;
  const float t2 = (float)(t1 / (double)sden + dnrm_d * (double)nrm);
  const f4v q4 = ld4(a.q + (int64_t)b * a.ldq + hd + 4 * c);
  const float* pdn = p.pdn + ((int64_t)bh * p.ns + s) * QS_KEYS * 2;
  const bool vk = vec_rows(a.dk, a.lddk);
  f4v dq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < QS_IT; ++it) {
    const int j = j0 + 4 * it + kk;
    if (j >= a.Tk) continue;
    const float2 pd = *reinterpret_cast<const float2*>(pdn + 2 * (4 * it + kk));
    const float gj = a.G[kb + j];
    const float bm = gj * pd.x;
    const float sg = bm > 0.f ? 1.f : (bm < 0.f ? -1.f : 0.f);
    const float da = (pd.y / sden + dnrm * sg) * gj;
    float ds = pd.x * (da - t2);
    if (a.kflag[kb + j] == 0.f) ds = 0.f;
    ds *= 0.125f;
    dq += ds * k4[it];
    f4v gk;
#pragma unroll
    for (int e = 0; e < 4; ++e) gk[e] = k4[it][e] > 0.f ? ds * q4[e] : 0.f;
    stx4(a.dk + (kb + j) * a.lddk + hd + 4 * c, gk, vk);
  }
  dq = xrow_sum_s(dq);
  if (kk == 0) *reinterpret_cast<f4v*>(p.dqp + ((int64_t)bh * p.ns + s) * ATT_DK + 4 * c) = dq;
}

__global__ __launch_bounds__(256) void q1s_bwd_dq_kernel(Q1sArgs p) {
  const AttnArgs& a = p.a;
  const int bh = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bh >= a.B * a.H) return;
  const int lane = threadIdx.x & 63;
  const int b = bh / a.H, h = bh - b * a.H;
  float v = 0.f;
  const float* src = p.dqp + (int64_t)bh * p.ns * ATT_DK + lane;
  for (int r0 = 0; r0 < p.ns; r0 += 16) {
    float x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float y = src[(int64_t)min(r0 + r, p.ns - 1) * ATT_DK];
      x[r] = r0 + r < p.ns ? y : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) v += x[r];
  }
  const int64_t qi = (int64_t)b * a.ldq + h * ATT_DK + lane;
  a.dq[(int64_t)b * a.lddq + h * ATT_DK + lane] = a.q[qi] > 0.f ? v : 0.f;
}

static int q1s_ns(int64_t Tk) { return (int)((Tk + QS_KEYS - 1) / QS_KEYS); }

static int q1s_check(const AttnArgs& a, int64_t dk, const char* who) {
  if (dk != ATT_DK) return fail(SAVQA_EUNSUP, std::string(who) + ": head dim must be 64");
  if (a.Tk <= 0 || a.B <= 0 || a.H <= 0) return fail(SAVQA_EINVAL, std::string(who) + ": empty");
  const uintptr_t al = (uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v;
  if ((al & 15) || (a.ldq & 3) || (a.ldk & 3) || (a.ldv & 3))
    return fail(SAVQA_EINVAL, std::string(who) + ": Q/K/V must be 16-B aligned with ld % 4 == 0");
  return 0;
}

}  // namespace savqa

using namespace savqa;

extern "C" int64_t savqa_gattn_q1s_ws_bytes(int64_t B, int64_t H, int64_t Tk) {
  const int64_t units = B * H * (int64_t)q1s_ns(Tk);
  const int64_t fwd = units * QS_PART * (int64_t)sizeof(float);
  const int64_t bwd = units * (int64_t)sizeof(double) + units * ATT_DK * (int64_t)sizeof(float) +
                      units * QS_KEYS * 2 * (int64_t)sizeof(float);
  return std::max(fwd, bwd) + 256;
}

static int q1s_ws(Q1sArgs& p, void* ws, int64_t ws_bytes, bool fwd, const char* who) {
  const int64_t units = (int64_t)p.a.B * p.a.H * p.ns;
  if (!ws || ws_bytes < savqa_gattn_q1s_ws_bytes(p.a.B, p.a.H, p.a.Tk) || ((uintptr_t)ws & 15))
    return fail(SAVQA_EINVAL, std::string(who) + ": workspace missing, too small or not 16-B aligned");
  char* w = static_cast<char*>(ws);
  if (fwd) {
    p.part = reinterpret_cast<float*>(w);
  } else {
    p.t1 = reinterpret_cast<double*>(w);
    p.dqp = reinterpret_cast<float*>(w + ((units * (int64_t)sizeof(double) + 15) & ~(int64_t)15));
    p.pdn = p.dqp + units * ATT_DK;
  }
  return 0;
}

extern "C" int savqa_gattn_fwd_q1s(void* stream, const float* q, int64_t ldq, const float* k,
                                   int64_t ldk, const float* v, int64_t ldv, const float* G,
                                   const float* kflag, const float* qflag, int64_t B, int64_t Tk,
                                   int64_t H, int64_t dk, float* o, int64_t ldo, float* stats,
                                   void* ws, int64_t ws_bytes) {
  Q1sArgs p{};
  AttnArgs& a = p.a;
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv; a.G = G;
  a.kflag = kflag; a.qflag = qflag; a.B = (int)B; a.Tq = 1; a.Tk = (int)Tk; a.H = (int)H;
  a.o = o; a.ldo = ldo;
  if (int rc = q1s_check(a, dk, "savqa_gattn_fwd_q1s")) return rc;
  if (!stats || ((uintptr_t)stats & 15))
    return fail(SAVQA_EINVAL, "savqa_gattn_fwd_q1s: 16-B aligned stats [B*H*4] required");
  p.ns = q1s_ns(Tk);
  p.stats = stats;
  if (int rc = q1s_ws(p, ws, ws_bytes, true, "savqa_gattn_fwd_q1s")) return rc;
  hipStream_t s = as_stream(stream);
  const unsigned blocks = (unsigned)(B * H * ((p.ns + 3) / 4));
  hipLaunchKernelGGL(q1s_fwd_part_kernel, dim3(blocks), dim3(256), 0, s, p);
  if (int rc = check_launch("savqa_gattn_fwd_q1s(part)")) return rc;
  hipLaunchKernelGGL(q1s_fwd_combine_kernel, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0, s, p);
  return check_launch("savqa_gattn_fwd_q1s(combine)");
}

extern "C" int savqa_gattn_bwd_q1s(void* stream, const float* q, int64_t ldq, const float* k,
                                   int64_t ldk, const float* v, int64_t ldv, const float* G,
                                   const float* kflag, const float* qflag, int64_t B, int64_t Tk,
                                   int64_t H, int64_t dk, const float* dout, int64_t lddo,
                                   const float* stats, float* dq, int64_t lddq, float* dk_,
                                   int64_t lddk, float* dv, int64_t lddv, void* ws,
                                   int64_t ws_bytes) {
  Q1sArgs p{};
  AttnArgs& a = p.a;
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv; a.G = G;
  a.kflag = kflag; a.qflag = qflag; a.B = (int)B; a.Tq = 1; a.Tk = (int)Tk; a.H = (int)H;
  a.dout = dout; a.lddo = lddo; a.dq = dq; a.lddq = lddq; a.dk = dk_; a.lddk = lddk;
  a.dv = dv; a.lddv = lddv;
  if (int rc = q1s_check(a, dk, "savqa_gattn_bwd_q1s")) return rc;
  if (!stats || ((uintptr_t)stats & 15) || (((uintptr_t)dout) & 15) || (lddo & 3))
    return fail(SAVQA_EINVAL, "savqa_gattn_bwd_q1s: stats / dO must be 16-B aligned, ld % 4 == 0");
  p.ns = q1s_ns(Tk);
  p.stats = const_cast<float*>(stats);
  if (int rc = q1s_ws(p, ws, ws_bytes, false, "savqa_gattn_bwd_q1s")) return rc;
  hipStream_t s = as_stream(stream);
  const unsigned blocks = (unsigned)(B * H * ((p.ns + 3) / 4));
  hipLaunchKernelGGL(q1s_bwd_dv_kernel, dim3(blocks), dim3(256), 0, s, p);
  if (int rc = check_launch("savqa_gattn_bwd_q1s(dv)")) return rc;
  hipLaunchKernelGGL(q1s_bwd_main_kernel, dim3(blocks), dim3(256), 0, s, p);
  if (int rc = check_launch("savqa_gattn_bwd_q1s(main)")) return rc;
  hipLaunchKernelGGL(q1s_bwd_dq_kernel, dim3((unsigned)((B * H + 3) / 4)), dim3(256), 0, s, p);
  return check_launch("savqa_gattn_bwd_q1s(dq)");
}
