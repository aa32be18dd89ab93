// Graph-guided multi-head attention core (forward + backward), gfx950.
//
// Reference: new_multihead_attention.forward, models/modules.py:246-301, i.e. after
// the ReLU'd Q/K/V projections (done by the GEMM) and before the residual + LN
// (done by ln.hip). Per (sample b, head h):
//   S = Q_h K_h^T / 8                              (:251-254, dk = 64)
//   S[:, j] = -4294967296 where kflag[b,j] == 0    (:257-263, blend of a -2^32+1 pad)
//   A = softmax over ALL keys                      (:278)
//   Bm = A * G[b]  (graph broadcast over heads)    (:280-284)
//   N = Bm / max(sum|Bm|, 1e-12)                   (:285, F.normalize p=1)
//   P = N * qflag[b,i]                             (:289-292)
//   O_h = P V_h                                    (:298-301)
// The encoder self-attention (Tq = Tk = T <= 100) and the decoder cross-attention
// (Tq = 1, keys = encoder output) are the same kernel with different strides.
//
// Layout: one 256-thread workgroup (4 waves) per (b, h). K_h and V_h (Tk x 64 fp32)
// are staged once into LDS with 68-float rows so a lane-per-key float4 read is
// bank-conflict-free; each wave processes 4 query rows at a time (register blocking:
// one K float4 read feeds 16 FMAs). Softmax / normalise use 64-lane shuffles.
// The backward recomputes P (no T x T tensor is saved) and keeps P and dS rows in LDS
// for the column sums dV = P^T dO and dK = dS^T Q.
#include "common.h"

namespace savqa {

constexpr int ATT_DK = 64;
constexpr int ATT_KLD = 68;  // padded K/V row (floats), 16-B aligned
constexpr int ATT_RB = 4;    // query rows per wave per pass
constexpr float ATT_MASKED = -4294967296.0f;  // fp32(-2**32 + 1)

struct AttnArgs {
  const float* q; int64_t ldq;
  const float* k; int64_t ldk;
  const float* v; int64_t ldv;
  const float* G;
  const float* kflag;
  const float* qflag;
  int B, Tq, Tk, H;
  float* o; int64_t ldo;
  float* att;
  // backward
  const float* dout; int64_t lddo;
  float* dq; int64_t lddq;
  float* dk; int64_t lddk;
  float* dv; int64_t lddv;
};

// Stage K_h, V_h rows [0,Tk) of sample b into LDS (row stride ATT_KLD).
__device__ __forceinline__ void stage_kv(const AttnArgs& a, int b, int h, float* Ks, float* Vs) {
  for (int idx = threadIdx.x; idx < a.Tk * 16; idx += blockDim.x) {
    const int j = idx >> 4, c4 = (idx & 15) * 4;
    const int64_t row = (int64_t)b * a.Tk + j;
    const float4 kv = *reinterpret_cast<const float4*>(a.k + row * a.ldk + h * ATT_DK + c4);
    const float4 vv = *reinterpret_cast<const float4*>(a.v + row * a.ldv + h * ATT_DK + c4);
    *reinterpret_cast<float4*>(&Ks[j * ATT_KLD + c4]) = kv;
    *reinterpret_cast<float4*>(&Vs[j * ATT_KLD + c4]) = vv;
  }
}

// Scores for ATT_RB query rows held in LDS (qs: [ATT_RB][64]) against key j (this lane,
// key block kb): s[r] = q_r . K_j
template <int KB>
__device__ __forceinline__ void row_dots(const float* qs, const float* Ks, int Tk, int lane,
                                         float (&s)[ATT_RB][KB]) {
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int j = kb * 64 + lane;
    const int jj = j < Tk ? j : Tk - 1;
    float acc[ATT_RB] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int d = 0; d < ATT_DK; d += 4) {
      const float4 kv = *reinterpret_cast<const float4*>(&Ks[jj * ATT_KLD + d]);
#pragma unroll
      for (int r = 0; r < ATT_RB; ++r) {
        const float4 qv = *reinterpret_cast<const float4*>(&qs[r * ATT_DK + d]);
        acc[r] = fmaf(qv.x, kv.x, acc[r]);
        acc[r] = fmaf(qv.y, kv.y, acc[r]);
        acc[r] = fmaf(qv.z, kv.z, acc[r]);
        acc[r] = fmaf(qv.w, kv.w, acc[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < ATT_RB; ++r) s[r][kb] = acc[r];
  }
}

// Forward quantities of one query row (given raw dots s[kb] of this lane's keys):
// a (softmax), bm (= a*G), inv (1/max(sum|bm|,eps)), nrm (sum|bm|), p (= bm*inv*qf).
template <int KB>
struct RowState {
  float a[KB], bm[KB], g[KB];
  float nrm, inv;
};

template <int KB>
__device__ __forceinline__ void row_forward(const AttnArgs& a, int b, int i, int lane,
                                            const float (&s)[KB], RowState<KB>& st) {
  float mx = -INFINITY;
  float sv[KB];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int j = kb * 64 + lane;
    float x = -INFINITY;
    if (j < a.Tk) {
      x = s[kb] * 0.125f;
      if (a.kflag[(int64_t)b * a.Tk + j] == 0.f) x = ATT_MASKED;
    }
    sv[kb] = x;
    mx = fmaxf(mx, x);
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int j = kb * 64 + lane;
    const float e = j < a.Tk ? expf(sv[kb] - mx) : 0.f;
    sv[kb] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  float nrm = 0.f;
  const float* grow = a.G + ((int64_t)b * a.Tq + i) * a.Tk;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int j = kb * 64 + lane;
    const float aa = sv[kb] / sum;
    const float gg = j < a.Tk ? grow[j] : 0.f;
    st.a[kb] = aa;
    st.g[kb] = gg;
    st.bm[kb] = gg * aa;
    nrm += fabsf(st.bm[kb]);
  }
  nrm = wave_sum(nrm);
  st.nrm = nrm;
  st.inv = 1.f / fmaxf(nrm, 1e-12f);
}

template <int KB>
__global__ __launch_bounds__(256) void gattn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int bh = blockIdx.x;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* Ks = sm;
  float* Vs = Ks + a.Tk * ATT_KLD;
  float* Ps = Vs + a.Tk * ATT_KLD;                     // [4 waves][ATT_RB][KB*64]
  float* Qs = Ps + 4 * ATT_RB * KB * 64;               // [4 waves][ATT_RB][64]
  float* P = Ps + w * ATT_RB * KB * 64;
  float* qs = Qs + w * ATT_RB * ATT_DK;
  stage_kv(a, b, h, Ks, Vs);
  __syncthreads();

  for (int i0 = w * ATT_RB; i0 < a.Tq; i0 += 4 * ATT_RB) {
#pragma unroll
    for (int r = 0; r < ATT_RB; ++r) {
      const int i = i0 + r < a.Tq ? i0 + r : a.Tq - 1;
      qs[r * ATT_DK + lane] = a.q[((int64_t)b * a.Tq + i) * a.ldq + h * ATT_DK + lane];
    }
    __builtin_amdgcn_wave_barrier();
    float s[ATT_RB][KB];
    row_dots<KB>(qs, Ks, a.Tk, lane, s);
#pragma unroll
    for (int r = 0; r < ATT_RB; ++r) {
      const int i = i0 + r;
      if (i >= a.Tq) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) P[r * KB * 64 + kb * 64 + lane] = 0.f;
        continue;
      }
      RowState<KB> st;
      row_forward<KB>(a, b, i, lane, s[r], st);
      const float qf = a.qflag[(int64_t)b * a.Tq + i];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int j = kb * 64 + lane;
        const float n = st.bm[kb] / fmaxf(st.nrm, 1e-12f);
        if (a.att && j < a.Tk)
          a.att[(((int64_t)h * a.B + b) * a.Tq + i) * a.Tk + j] = n;
        P[r * KB * 64 + kb * 64 + lane] = j < a.Tk ? n * qf : 0.f;
      }
    }
    __builtin_amdgcn_wave_barrier();
    // O_r[d] = sum_j P[r][j] V[j][d]   (lane = d)
    float o[ATT_RB] = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < a.Tk; ++j) {
      const float vv = Vs[j * ATT_KLD + lane];
#pragma unroll
      for (int r = 0; r < ATT_RB; ++r) o[r] = fmaf(P[r * KB * 64 + j], vv, o[r]);
    }
#pragma unroll
    for (int r = 0; r < ATT_RB; ++r) {
      const int i = i0 + r;
      if (i < a.Tq) a.o[((int64_t)b * a.Tq + i) * a.ldo + h * ATT_DK + lane] = o[r];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <int KB>
__global__ __launch_bounds__(256) void gattn_bwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int bh = blockIdx.x;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int PLD = a.Tk + 1;
  const int TQP = (a.Tq + ATT_RB - 1) / ATT_RB * ATT_RB;  // rows padded to the row block
  float* Ks = sm;
  float* Vs = Ks + a.Tk * ATT_KLD;
  float* Pst = Vs + a.Tk * ATT_KLD;          // [Tq][Tk+1]  P
  float* dSt = Pst + a.Tq * PLD;             // [Tq][Tk+1]  dS (pre-scale, masked)
  float* Qs = dSt + a.Tq * PLD;              // [TQP][64]   Q_h rows (staged once)
  float* dOs = Qs + TQP * ATT_DK;            // [TQP][64]   dO_h rows
  stage_kv(a, b, h, Ks, Vs);
  for (int idx = threadIdx.x; idx < TQP * 16; idx += blockDim.x) {
    const int i = idx >> 4, c4 = (idx & 15) * 4;
    float4 qv = make_float4(0.f, 0.f, 0.f, 0.f), dv4 = qv;
    if (i < a.Tq) {
      const int64_t row = (int64_t)b * a.Tq + i;
      qv = *reinterpret_cast<const float4*>(a.q + row * a.ldq + h * ATT_DK + c4);
      dv4 = *reinterpret_cast<const float4*>(a.dout + row * a.lddo + h * ATT_DK + c4);
    }
    *reinterpret_cast<float4*>(&Qs[i * ATT_DK + c4]) = qv;
    *reinterpret_cast<float4*>(&dOs[i * ATT_DK + c4]) = dv4;
  }
  __syncthreads();

  for (int i0 = w * ATT_RB; i0 < a.Tq; i0 += 4 * ATT_RB) {
    const float* qs = Qs + i0 * ATT_DK;
    const float* dos = dOs + i0 * ATT_DK;
    __builtin_amdgcn_wave_barrier();
    float s[ATT_RB][KB], dp[ATT_RB][KB];
    row_dots<KB>(qs, Ks, a.Tk, lane, s);
    row_dots<KB>(dos, Vs, a.Tk, lane, dp);   // dP_ij = dO_i . V_j
#pragma unroll
    for (int r = 0; r < ATT_RB; ++r) {
      const int i = i0 + r;
      if (i >= a.Tq) continue;
      RowState<KB> st;
      row_forward<KB>(a, b, i, lane, s[r], st);
      const float qf = a.qflag[(int64_t)b * a.Tq + i];
      const float sden = fmaxf(st.nrm, 1e-12f);
      // dN = dP * qf ;  n = bm / sden
      float dn[KB], t1 = 0.f;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        dn[kb] = dp[r][kb] * qf;
        t1 += dn[kb] * st.bm[kb];
      }
      t1 = wave_sum(t1);
      // d sden = -sum dn*bm / sden^2 ; passes through clamp_min where nrm >= eps
      const float dnrm = st.nrm >= 1e-12f ? -t1 / (sden * sden) : 0.f;
      float da[KB], t2 = 0.f;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const float sg = st.bm[kb] > 0.f ? 1.f : (st.bm[kb] < 0.f ? -1.f : 0.f);
        const float dbm = dn[kb] / sden + dnrm * sg;
        da[kb] = dbm * st.g[kb];
        t2 += da[kb] * st.a[kb];
      }
      t2 = wave_sum(t2);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int j = kb * 64 + lane;
        if (j < a.Tk) {
          float ds = st.a[kb] * (da[kb] - t2);
          if (a.kflag[(int64_t)b * a.Tk + j] == 0.f) ds = 0.f;
          dSt[i * PLD + j] = ds * 0.125f;
          Pst[i * PLD + j] = st.bm[kb] / sden * qf;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    // dQ_r[d] = sum_j dS[r][j] K[j][d]  (lane = d), then the ReLU mask of Q
    float dq[ATT_RB] = {0.f, 0.f, 0.f, 0.f};
    const int nr = min(ATT_RB, a.Tq - i0);
    for (int j = 0; j < a.Tk; ++j) {
      const float kv = Ks[j * ATT_KLD + lane];
#pragma unroll
      for (int r = 0; r < ATT_RB; ++r)
        if (r < nr) dq[r] = fmaf(dSt[(i0 + r) * PLD + j], kv, dq[r]);
    }
#pragma unroll
    for (int r = 0; r < ATT_RB; ++r) {
      if (r < nr) {
        const int64_t row = (int64_t)b * a.Tq + i0 + r;
        a.dq[row * a.lddq + h * ATT_DK + lane] = qs[r * ATT_DK + lane] > 0.f ? dq[r] : 0.f;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // column pass: dV[j] = sum_i P[i][j] dO[i], dK[j] = sum_i dS[i][j] Q[i]  (lane = d)
  for (int j0 = w * 4; j0 < a.Tk; j0 += 16) {
    float dvv[4] = {0.f, 0.f, 0.f, 0.f}, dkk[4] = {0.f, 0.f, 0.f, 0.f};
    const int nj = min(4, a.Tk - j0);
    for (int i = 0; i < a.Tq; ++i) {
      const float dov = dOs[i * ATT_DK + lane];
      const float qv = Qs[i * ATT_DK + lane];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c < nj) {
          dvv[c] = fmaf(Pst[i * PLD + j0 + c], dov, dvv[c]);
          dkk[c] = fmaf(dSt[i * PLD + j0 + c], qv, dkk[c]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c < nj) {
        const int j = j0 + c;
        const int64_t row = (int64_t)b * a.Tk + j;
        a.dv[row * a.lddv + h * ATT_DK + lane] = Vs[j * ATT_KLD + lane] > 0.f ? dvv[c] : 0.f;
        a.dk[row * a.lddk + h * ATT_DK + lane] = Ks[j * ATT_KLD + lane] > 0.f ? dkk[c] : 0.f;
      }
    }
  }
}

static size_t fwd_lds(int Tk, int KB) {
  return sizeof(float) * ((size_t)2 * Tk * ATT_KLD + 4 * ATT_RB * KB * 64 + 4 * ATT_RB * ATT_DK);
}
static size_t bwd_lds(int Tq, int Tk) {
  const size_t tqp = (size_t)(Tq + ATT_RB - 1) / ATT_RB * ATT_RB;
  return sizeof(float) * ((size_t)2 * Tk * ATT_KLD + 2 * (size_t)Tq * (Tk + 1) + 2 * tqp * ATT_DK);
}
constexpr size_t kMaxLds = 160 * 1024;

static int validate(const AttnArgs& a, int64_t dk, const char* who) {
  if (dk != ATT_DK) return fail(SAVQA_EUNSUP, std::string(who) + ": head dim must be 64");
  if (a.Tk <= 0 || a.Tq <= 0 || a.B <= 0 || a.H <= 0) return fail(SAVQA_EINVAL, std::string(who) + ": empty");
  if (a.Tk > 128) return fail(SAVQA_EUNSUP, std::string(who) + ": Tk > 128 not supported yet");
  const uintptr_t al = (uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v;
  if ((al & 15) || (a.ldk & 3) || (a.ldv & 3))
    return fail(SAVQA_EINVAL, std::string(who) + ": K/V must be 16-B aligned with ld % 4 == 0");
  return 0;
}

}  // namespace savqa

using namespace savqa;

extern "C" int savqa_gattn_fwd(void* stream, const float* q, int64_t ldq, const float* k,
                               int64_t ldk, const float* v, int64_t ldv, const float* G,
                               const float* kflag, const float* qflag, int64_t B, int64_t Tq,
                               int64_t Tk, int64_t H, int64_t dk, float* o, int64_t ldo,
                               float* att) {
  AttnArgs a{};
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv; a.G = G;
  a.kflag = kflag; a.qflag = qflag; a.B = (int)B; a.Tq = (int)Tq; a.Tk = (int)Tk; a.H = (int)H;
  a.o = o; a.ldo = ldo; a.att = att;
  if (int rc = validate(a, dk, "savqa_gattn_fwd")) return rc;
  hipStream_t s = as_stream(stream);
  if (Tk <= 64) {
    const size_t lds = fwd_lds((int)Tk, 1);
    hipLaunchKernelGGL(gattn_fwd_kernel<1>, dim3(B * H), dim3(256), lds, s, a);
  } else {
    const size_t lds = fwd_lds((int)Tk, 2);
    hipLaunchKernelGGL(gattn_fwd_kernel<2>, dim3(B * H), dim3(256), lds, s, a);
  }
  return check_launch("savqa_gattn_fwd");
}

extern "C" int savqa_gattn_bwd(void* stream, const float* q, int64_t ldq, const float* k,
                               int64_t ldk, const float* v, int64_t ldv, const float* G,
                               const float* kflag, const float* qflag, int64_t B, int64_t Tq,
                               int64_t Tk, int64_t H, int64_t dk, const float* dout, int64_t lddo,
                               float* dq, int64_t lddq, float* dk_, int64_t lddk, float* dv,
                               int64_t lddv) {
  AttnArgs a{};
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv; a.G = G;
  a.kflag = kflag; a.qflag = qflag; a.B = (int)B; a.Tq = (int)Tq; a.Tk = (int)Tk; a.H = (int)H;
  a.dout = dout; a.lddo = lddo; a.dq = dq; a.lddq = lddq; a.dk = dk_; a.lddk = lddk;
  a.dv = dv; a.lddv = lddv;
  if (int rc = validate(a, dk, "savqa_gattn_bwd")) return rc;
  const size_t lds = bwd_lds((int)Tq, (int)Tk);
  if (lds > kMaxLds) return fail(SAVQA_EUNSUP, "savqa_gattn_bwd: Tq*Tk too large for the LDS path");
  hipStream_t s = as_stream(stream);
  if (Tk <= 64)
    hipLaunchKernelGGL(gattn_bwd_kernel<1>, dim3(B * H), dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL(gattn_bwd_kernel<2>, dim3(B * H), dim3(256), lds, s, a);
  return check_launch("savqa_gattn_bwd");
}
