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
// Two kernel families: T_q > 1 (encoder self-attention, and any multi-query block call):
// the MFMA strip kernels (gattn_*_mfma_kernel, one wave per 16-query strip; a partial strip
// is masked); T_q = 1 (decoder cross-attention): the single-query kernels
// (gattn_*_q1_kernel). The backward recomputes P (no T x T tensor is saved).
#include "attn_common.h"

#include <type_traits>

#ifndef SAVQA_ATT_BWD2
#define SAVQA_ATT_BWD2 1
#endif

namespace savqa {

// ---------------------------------------------------------------------------------------
// MFMA path (v_mfma_f32_16x16x4_f32, exact fp32 products). One workgroup per (b, h) with
// one wave per 16-row query strip (nw = ceil(Tq/16) <= 8 waves); NJT = ceil(Tk/16) key
// tiles. 16x16x4 operand maps: lane l supplies A[m = l&15][k = l>>4] and B[k = l>>4]
// [n = l&15]; the accumulator holds D[4(l>>4) + r][l&15], r = 0..3. Inner products over
// d take 4 consecutive d per lane (one b128 load) and consume them as 4 k-steps, so
// lane group g covers d = 16c + 4g + t: the same permutation on A and B.
//
// Backward, phase 1 (per wave, registers only): S and dP strips (16 x 16*NJT), the row
// softmax / graph / L1-normalise chain and its adjoint with 16-lane DPP row reductions
// (an accumulator row lives in one 16-lane DPP row), then P and dS are written to LDS
// transposed ([key][query], one b128 per lane per tile).
// Phase 2 (after one barrier), 16x16 output tiles in contiguous runs per wave:
//   dV = P^T dO and dK = dS^T Q  (A = b128 rows of the transposed LDS images),
//   dQ = dS K                     (A = 4 scalar LDS reads, conflict-free, see PLD).
// The B operands (dO, Q, K column blocks) come straight from global memory (L1/L2 hits:
// the workgroup just streamed the same rows in phase 1) into registers, once per
// (tensor, column block) group.
// LDS: 2 * 16*NJT * (16*nw + 4) floats  (53.7 KB at T = 73, 2 workgroups / CU).
// PLD = 16*nw + 4 makes both the b128 row reads (16 lanes -> 16 disjoint bank quads)
// and the scalar column reads (4 lane groups at bank offsets 16g) conflict-free.
// acc[jt] = X_strip . Y_tile(jt)^T over d = 64: X rows (i0 + col), Y rows (16 jt + col)
template <int NJT>
__device__ __forceinline__ void strip_dots(const f4v (&x)[4], const float* y, int64_t ldy,
                                           int64_t ybase, int Tk, int col, int g,
                                           f4v (&acc)[NJT]) {
#pragma unroll
  for (int jt = 0; jt < NJT; ++jt) {
    const int j = min(jt * 16 + col, Tk - 1);
    const float* yr = y + (ybase + j) * ldy + 4 * g;
    f4v yv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) yv[c] = ld4(yr + 16 * c);
    f4v s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      s = mfma16(x[c].x, yv[c].x, s);
      s = mfma16(x[c].y, yv[c].y, s);
      s = mfma16(x[c].z, yv[c].z, s);
      s = mfma16(x[c].w, yv[c].w, s);
    }
    acc[jt] = s;
  }
}

// Cooperative stage of K_h and V_h rows [0, TK) into LDS (zero rows past Tk) through the
// (sample, head) views: thread t moves 16-B chunk t % 16 of rows t / 16 + 4 nw u' (one 32-bit
// lane offset; the row block of each load is its soffset). Batches of SKV_BATCH loads per
// thread are issued back to back and only then stored, so a batch costs one memory latency.
constexpr int SKV_BATCH = 4;
template <int TK>
__device__ __forceinline__ void stage_kv_tiles(const BView& K, const BView& V, int Tk, float* Ks,
                                               float* Vs) {
  const int t = threadIdx.x, rstep = blockDim.x >> 4;
  const uint32_t kvo = (uint32_t)(t >> 4) * K.ld + 16u * (t & 15);
  const uint32_t vvo = (uint32_t)(t >> 4) * V.ld + 16u * (t & 15);
  for (int r0 = 0; r0 < TK; r0 += SKV_BATCH * rstep) {
    f4v kv[SKV_BATCH], vv[SKV_BATCH];
#pragma unroll
    for (int u = 0; u < SKV_BATCH; ++u) {
      const uint32_t row = (uint32_t)(r0 + u * rstep);
      kv[u] = bld16b<f4v>(K, kvo, row * K.ld);
      vv[u] = bld16b<f4v>(V, vvo, row * V.ld);
    }
#pragma unroll
    for (int u = 0; u < SKV_BATCH; ++u) {
      const int j = r0 + u * rstep + (t >> 4), c4 = (t & 15) * 4;
      if (j < TK) {
        const bool ok = j < Tk;
        const f4v z = {0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f4v*>(&Ks[j * ATT_KLD + c4]) = ok ? kv[u] : z;
        *reinterpret_cast<f4v*>(&Vs[j * ATT_KLD + c4]) = ok ? vv[u] : z;
      }
    }
  }
}

// Forward row chain for accumulator row r of this lane (query i, keys 16 jt + col):
// a = softmax, gg = graph, bm = a*gg, nrm = sum|bm| (all keys < Tk). The exponent runs in
// base 2 (attn_common.h ATT_SCALE2: one v_exp_f32 per element).
template <int NJT>
__device__ __forceinline__ float strip_row_forward(const f4v (&s)[NJT], int r, const float (&kf)[NJT],
                                                   const float (&gpre)[NJT], int Tk, int col,
                                                   float (&aa)[NJT], float (&gg)[NJT],
                                                   float (&bm)[NJT]) {
  float x[NJT];
  float mx = -INFINITY;
#pragma unroll
  for (int jt = 0; jt < NJT; ++jt) {
    const int j = jt * 16 + col;
    float v = -INFINITY;
    if (j < Tk) v = kf[jt] == 0.f ? ATT_MASKED : s[jt][r] * ATT_SCALE2;
    x[jt] = v;
    mx = fmaxf(mx, v);
  }
  mx = row16_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int jt = 0; jt < NJT; ++jt) {
    const int j = jt * 16 + col;
    const float e = j < Tk ? att_exp2(x[jt] - mx) : 0.f;
    x[jt] = e;
    sum += e;
  }
  sum = row16_sum(sum);
  const float rsum = __builtin_amdgcn_rcpf(sum);  // one reciprocal per row (the elements multiply)
  float nrm = 0.f;
#pragma unroll
  for (int jt = 0; jt < NJT; ++jt) {
    const int j = jt * 16 + col;
    aa[jt] = x[jt] * rsum;
    gg[jt] = j < Tk ? gpre[jt] : 0.f;
    bm[jt] = gg[jt] * aa[jt];
    nrm += fabsf(bm[jt]);
  }
  return row16_sum(nrm);
}

// graph values of this lane's 4 accumulator rows (queries i0+4g+r) x keys 16 jt + col, and the
// key / query flags of the strip, loaded up front (their latency overlaps the MFMA strip
// products instead of serialising inside the row chain): one lane offset, the (r, jt) parts in
// soffset. Rows / columns past T read neighbouring (or zero) values that the chain masks.
template <int NJT>
__device__ __forceinline__ void preload_graph(const BView& G, int Tk, int i0, int g, int col,
                                              float (&gp)[4][NJT]) {
  const uint32_t vo = (uint32_t)((i0 + 4 * g) * Tk + col) * 4u;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int jt = 0; jt < NJT; ++jt) gp[r][jt] = bld1(G, vo, (uint32_t)(r * Tk + jt * 16) * 4u);
}
template <int NJT>
__device__ __forceinline__ void preload_flags(const BView& KF, const BView& QF, int i0, int g,
                                              int col, float (&kf)[NJT], float (&qf)[4]) {
#pragma unroll
  for (int jt = 0; jt < NJT; ++jt) kf[jt] = bld1(KF, 4u * col, 64u * jt);
#pragma unroll
  for (int r = 0; r < 4; ++r) qf[r] = bld1(QF, 4u * (i0 + 4 * g), 4u * r);
}

template <int NJT, typename T>
__global__ __launch_bounds__(512) void gattn_fwd_mfma_kernel(AttnArgsT<T> a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  // XCD-aware (common.h xcd_remap): the H heads of a sample run on one XCD, so its graph
  // rows come from HBM once per L2 instead of once per head
  const int bh = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int i0 = w * 16;
  constexpr int TK = NJT * 16;
  constexpr int WLD = 20;                   // per-wave P^T image [TK][16 + 4]
  constexpr uint32_t ES = sizeof(T);
  // V first, then K; the per-wave P^T images reuse K's space once S is computed (one
  // block barrier), so the block needs V + max(K, P) instead of V + K + P (T=73: 54 KB,
  // 3 workgroups per CU instead of 2)
  float* Vs = sm;                           // [TK][ATT_KLD]
  float* Ks = Vs + TK * ATT_KLD;            // [TK][ATT_KLD]
  float* Pw = Ks + w * TK * WLD;
  const StripViews<AttnArgsT<T>> sv(a, b, h);
  // strip operands, graph and flags first, then the K/V staging: every load of the
  // workgroup's first phase is in flight together (rows past Tq: masked outputs)
  f4v qa[4];
  {
    const uint32_t vo = (uint32_t)(i0 + col) * sv.q.ld + 4 * ES * g;
#pragma unroll
    for (int c = 0; c < 4; ++c) qa[c] = bldx4<T>(sv.q, vo, 16 * ES * c);
  }
  float gp[4][NJT], kf[NJT], qf[4];
  preload_graph<NJT>(sv.g, a.Tk, i0, g, col, gp);
  preload_flags<NJT>(sv.kf, sv.qf, i0, g, col, kf, qf);
  stage_kv_tiles<TK>(sv.k, sv.v, a.Tk, Ks, Vs);
  __syncthreads();  // K/V staged
  f4v s[NJT];
  strip_dots_lds<NJT>(qa, Ks, col, g, s);
  __syncthreads();  // every wave is done with K before the P images overwrite it

  f4v pv[NJT];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    float aa[NJT], gg[NJT], bm[NJT];
    const float nrm = strip_row_forward<NJT>(s, r, kf, gp[r], a.Tk, col, aa, gg, bm);
    const float rsd = __builtin_amdgcn_rcpf(fmaxf(nrm, 1e-12f));
#pragma unroll
    for (int jt = 0; jt < NJT; ++jt) {
      const int j = jt * 16 + col;
      const float n = bm[jt] * rsd;
      const bool ok = i < a.Tq && j < a.Tk;
      if (a.att && ok) a.att[(((int64_t)h * a.B + b) * a.Tq + i) * a.Tk + j] = n;
      pv[jt][r] = ok ? n * qf[r] : 0.f;
    }
  }
#pragma unroll
  for (int jt = 0; jt < NJT; ++jt)
    *reinterpret_cast<f4v*>(&Pw[(jt * 16 + col) * WLD + 4 * g]) = pv[jt];
  __builtin_amdgcn_wave_barrier();  // this wave's P^T strip written (wave-private image)
  // O strip = P V: A[m = i][k = j] = P^T[j][i], B[k = j][n = d] = V[j][d]
  f4v o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int jc = 0; jc < NJT; ++jc) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = jc * 16 + 4 * g + t;
      const float pa = Pw[j * WLD + col];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] = mfma16(pa, Vs[j * ATT_KLD + dt * 16 + col], o[dt]);
    }
  }
  const BView O = head_view(a.o, a.ldo, (int64_t)a.B * a.Tq, (int64_t)b * a.Tq, h * ATT_DK);
  const uint32_t ovo = (uint32_t)(i0 + 4 * g) * O.ld + 4u * col;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (i0 + 4 * g + r < a.Tq) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) bst32(O, o[dt][r], ovo, r * O.ld + 64u * dt);
    }
  }
}

template <int NJT, typename T>
__global__ __launch_bounds__(512) void gattn_bwd_mfma_kernel(AttnArgsT<T> a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  // XCD-aware (common.h xcd_remap): the H heads of a sample run on one XCD, so its graph
  // rows come from HBM once per L2 instead of once per head
  const int bh = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bh / a.H, h = bh % a.H;
  const int nw = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int i0 = w * 16;
  constexpr int TK = NJT * 16;
  const int PLD = 16 * nw + 4;
  float* Pt = sm;             // [TK][PLD]  P^T                      (phase 2)
  float* dSt = sm + TK * PLD; // [TK][PLD]  dS^T (scaled by 1/8, masked)
  float* Ks = sm;             // [TK][ATT_KLD] K_h, V_h staged for phase 1 (aliases Pt/dSt)
  float* Vs = sm + TK * ATT_KLD;
  const int64_t qb = (int64_t)b * a.Tq, kb = (int64_t)b * a.Tk;
  const int hd = h * ATT_DK;

  // ---- phase 1: strips (strip operands, graph and flags are loaded before the K/V
  // staging, so all of the phase's loads are in flight together)
  {
    f4v qa[4], oa[4];
    const int iq = min(i0 + col, a.Tq - 1);
    const T* qr = a.q + (qb + iq) * a.ldq + hd + 4 * g;
    const float* orr = a.dout + (qb + iq) * a.lddo + hd + 4 * g;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      qa[c] = ldx4(qr + 16 * c);
      oa[c] = ld4(orr + 16 * c);
    }
    float gp[4][NJT];
    const StripViews<std::remove_reference_t<decltype(a)>> sv(a, b, h);
    preload_graph<NJT>(sv.g, a.Tk, i0, g, col, gp);
    float kf[NJT];
#pragma unroll
    for (int jt = 0; jt < NJT; ++jt) kf[jt] = a.kflag[kb + min(jt * 16 + col, a.Tk - 1)];
    stage_kv_tiles<TK>(sv.k, sv.v, a.Tk, Ks, Vs);
    __syncthreads();  // K/V staged
    f4v s[NJT], dp[NJT];
    strip_dots_lds<NJT>(qa, Ks, col, g, s);
    strip_dots_lds<NJT>(oa, Vs, col, g, dp);
    __syncthreads();  // every wave is done with K/V: the region becomes P^T / dS^T
    f4v pv[NJT], dsv[NJT];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * g + r;
      const int ic = min(i, a.Tq - 1);
      float aa[NJT], gg[NJT], bm[NJT];
      const float nrm = strip_row_forward<NJT>(s, r, kf, gp[r], a.Tk, col, aa, gg, bm);
      const float sden = fmaxf(nrm, 1e-12f);
      const float rsd = 1.f / sden;
      const float qf = a.qflag[qb + ic];
      float dn[NJT], t1 = 0.f;
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        dn[jt] = dp[jt][r] * qf;
        t1 += dn[jt] * bm[jt];
      }
      t1 = row16_sum(t1);
      const float dnrm = nrm >= 1e-12f ? -t1 * (rsd * rsd) : 0.f;
      float da[NJT], t2 = 0.f;
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        const float sg = bm[jt] > 0.f ? 1.f : (bm[jt] < 0.f ? -1.f : 0.f);
        const float dbm = dn[jt] * rsd + dnrm * sg;
        da[jt] = dbm * gg[jt];
        t2 += da[jt] * aa[jt];
      }
      t2 = row16_sum(t2);
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        const int j = jt * 16 + col;
        const bool ok = i < a.Tq && j < a.Tk;
        float ds = aa[jt] * (da[jt] - t2);
        if (kf[jt] == 0.f) ds = 0.f;
        dsv[jt][r] = ok ? ds * 0.125f : 0.f;
        pv[jt][r] = ok ? bm[jt] * rsd * qf : 0.f;
      }
    }
#pragma unroll
    for (int jt = 0; jt < NJT; ++jt) {
      *reinterpret_cast<f4v*>(&Pt[(jt * 16 + col) * PLD + i0 + 4 * g]) = pv[jt];
      *reinterpret_cast<f4v*>(&dSt[(jt * 16 + col) * PLD + i0 + 4 * g]) = dsv[jt];
    }
  }
  __syncthreads();

  // ---- phase 2: 16x16 output tiles, grouped (tensor, 16-column block dt):
  //   groups [0,4): dV = P^T dO, [4,8): dK = dS^T Q  (NJT key tiles each, k = query),
  //   groups [8,12): dQ = dS K                        (nw query tiles each, k = key).
  // Each wave takes a CONTIGUOUS run of tiles, so consecutive tiles share the group's
  // B column block (dO / Q / K[:, dt]), loaded once into registers per group.
  const int nitems = 8 * NJT + 4 * nw;
  const int it0 = nitems * w / nw, it1 = nitems * (w + 1) / nw;
  int cur = -1;
  float bcol[8][4];  // B rows k = 16 kc + 4g + t of column dt*16 + col (kc < 8)
  for (int it = it0; it < it1; ++it) {
    int grp, tile;
    if (it < 8 * NJT) {
      grp = it / NJT;
      tile = it - grp * NJT;
    } else {
      grp = 8 + (it - 8 * NJT) / nw;
      tile = (it - 8 * NJT) % nw;
    }
    const int dt = grp & 3;
    const int dcol = hd + dt * 16 + col;
    if (grp != cur) {  // wave-uniform
      cur = grp;
      const T* src = grp < 8 ? a.q : a.k;  // dO (fp32) for grp < 4
      const int64_t ld = grp < 4 ? a.lddo : (grp < 8 ? a.ldq : a.ldk);
      const int64_t base = grp < 8 ? qb : kb;
      const int lim = grp < 8 ? a.Tq : a.Tk;
      const int nk = grp < 8 ? nw : NJT;
#pragma unroll
      for (int kc = 0; kc < 8; ++kc) {
        if (kc < nk) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int64_t off = (base + min(kc * 16 + 4 * g + t, lim - 1)) * ld + dcol;
            bcol[kc][t] = grp < 4 ? a.dout[off] : ldx1(src + off);
          }
        }
      }
    }
    // ReLU-mask values of this tile's 4 output rows, fetched before the MFMAs (clamped rows)
    float mk[4];
    {
      const T* msrc = grp < 4 ? a.v : (grp < 8 ? a.k : a.q);
      const int64_t mld = grp < 4 ? a.ldv : (grp < 8 ? a.ldk : a.ldq);
      const int64_t base = grp < 8 ? kb : qb;
      const int lim = grp < 8 ? a.Tk : a.Tq;
#pragma unroll
      for (int r = 0; r < 4; ++r) mk[r] = ldx1(msrc + (base + min(tile * 16 + 4 * g + r, lim - 1)) * mld + dcol);
    }
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    if (grp < 8) {
      const bool isv = grp < 4;
      const float* arow = (isv ? Pt : dSt) + (tile * 16 + col) * PLD + 4 * g;
#pragma unroll
      for (int kc = 0; kc < 8; ++kc) {
        if (kc < nw) {
          const f4v av = ld4(arow + kc * 16);
          acc = mfma16(av.x, bcol[kc][0], acc);
          acc = mfma16(av.y, bcol[kc][1], acc);
          acc = mfma16(av.z, bcol[kc][2], acc);
          acc = mfma16(av.w, bcol[kc][3], acc);
        }
      }
      // dV / dK rows j = 16 tile + 4g + r, ReLU mask of the saved V / K
      T* dst = isv ? a.dv : a.dk;
      const int64_t dld = isv ? a.lddv : a.lddk;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = tile * 16 + 4 * g + r;
        if (j < a.Tk) stx1(dst + (kb + j) * dld + dcol, mk[r] > 0.f ? acc[r] : 0.f);
      }
    } else {
#pragma unroll
      for (int kc = 0; kc < NJT; ++kc) {
        float av[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) av[t] = dSt[(kc * 16 + 4 * g + t) * PLD + tile * 16 + col];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc = mfma16(av[t], bcol[kc][t], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = tile * 16 + 4 * g + r;
        if (i < a.Tq) stx1(a.dq + (qb + i) * a.lddq + dcol, mk[r] > 0.f ? acc[r] : 0.f);
      }
    }
  }
}

// fp32 backward, second structure (SAVQA_ATT_BWD2; the bf16 twin gattn_bwd_mfma_bf2_kernel
// below explains the restructuring): dQ = dS K in phase 1 from the wave's own dS^T columns and
// the staged K, then dV^T = dO^T P and dK^T = Q^T dS as 16x16 tiles whose B operand is one b128
// read of a P^T / dS^T row and whose 4 outputs per lane are one 16-B store. LDS: K stays
// staged through the kernel (dQ's B operand, dK's ReLU mask); P^T takes V's place once every
// wave has its dP; dS^T has its own region: 75 KB at T = 73 (2 workgroups per CU, as before).
template <int NJT, typename T>
__global__ __launch_bounds__(512) void gattn_bwd_mfma2_kernel(AttnArgsT<T> a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int bh = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bh / a.H, h = bh % a.H;
  const int nw = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int i0 = w * 16;
  constexpr int TK = NJT * 16;
  constexpr uint32_t ES = sizeof(T);
  const int PLD = 16 * nw + 4;
  const int VREG = TK * ATT_KLD > TK * PLD ? TK * ATT_KLD : TK * PLD;
  float* Ks = sm;                   // [TK][ATT_KLD] K_h (whole kernel)
  float* Vs = sm + TK * ATT_KLD;    // [TK][ATT_KLD] V_h (phase 1a), then
  float* Pt = Vs;                   // [TK][PLD]     P^T
  float* dSt = Vs + VREG;           // [TK][PLD]     dS^T (scaled by 1/8, masked)
  const StripViews<AttnArgsT<T>> sv(a, b, h);
  const int64_t nq = (int64_t)a.B * a.Tq, nk = (int64_t)a.B * a.Tk;
  const int64_t qb = (int64_t)b * a.Tq, kb = (int64_t)b * a.Tk;
  const BView DO = head_view(a.dout, a.lddo, nq, qb, h * ATT_DK);
  {
    f4v qa[4], oa[4];
    const uint32_t qvo = (uint32_t)(i0 + col) * sv.q.ld + 4 * ES * g;
    const uint32_t ovo = (uint32_t)(i0 + col) * DO.ld + 16u * g;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      qa[c] = bldx4<T>(sv.q, qvo, 16 * ES * c);
      oa[c] = bld16b<f4v>(DO, ovo, 64u * c);
    }
    float gp[4][NJT], kf[NJT], qf[4];
    preload_graph<NJT>(sv.g, a.Tk, i0, g, col, gp);
    preload_flags<NJT>(sv.kf, sv.qf, i0, g, col, kf, qf);
    stage_kv_tiles<TK>(sv.k, sv.v, a.Tk, Ks, Vs);
    __syncthreads();  // K/V staged
    f4v s[NJT], dp[NJT];
    strip_dots_lds<NJT>(qa, Ks, col, g, s);
    strip_dots_lds<NJT>(oa, Vs, col, g, dp);
    __syncthreads();  // every wave is done with V: its region becomes P^T
    f4v pv[NJT], dsv[NJT];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * g + r;
      float aa[NJT], gg[NJT], bm[NJT];
      const float nrm = strip_row_forward<NJT>(s, r, kf, gp[r], a.Tk, col, aa, gg, bm);
      const float rsd = __builtin_amdgcn_rcpf(fmaxf(nrm, 1e-12f));
      float dn[NJT], t1 = 0.f;
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        dn[jt] = dp[jt][r] * qf[r];
        t1 += dn[jt] * bm[jt];
      }
      t1 = row16_sum(t1);
      const float dnrm = nrm >= 1e-12f ? -t1 * (rsd * rsd) : 0.f;
      float da[NJT], t2 = 0.f;
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        const float sg = bm[jt] > 0.f ? 1.f : (bm[jt] < 0.f ? -1.f : 0.f);
        const float dbm = dn[jt] * rsd + dnrm * sg;
        da[jt] = dbm * gg[jt];
        t2 += da[jt] * aa[jt];
      }
      t2 = row16_sum(t2);
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        const int j = jt * 16 + col;
        const bool ok = i < a.Tq && j < a.Tk;
        float ds = aa[jt] * (da[jt] - t2);
        if (kf[jt] == 0.f) ds = 0.f;
        dsv[jt][r] = ok ? ds * 0.125f : 0.f;
        pv[jt][r] = ok ? bm[jt] * rsd * qf[r] : 0.f;
      }
    }
#pragma unroll
    for (int jt = 0; jt < NJT; ++jt) {
      *reinterpret_cast<f4v*>(&Pt[(jt * 16 + col) * PLD + i0 + 4 * g]) = pv[jt];
      *reinterpret_cast<f4v*>(&dSt[(jt * 16 + col) * PLD + i0 + 4 * g]) = dsv[jt];
    }
  }
  {
    // dQ ReLU masks (rows i0 + 4g + r, columns 16 dt + col), under the dQ products
    const uint32_t mvo = (uint32_t)(i0 + 4 * g) * sv.q.ld + ES * col;
    float qm[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) qm[r][dt] = bldx1<T>(sv.q, mvo, r * sv.q.ld + 16 * ES * dt);
    __builtin_amdgcn_wave_barrier();  // this wave's dS^T columns are written (in-order LDS)
    // dQ strip = dS K: A[m = i][k = j] = dS^T[j][i0 + i], B[k = j][n = d] = K[j][16 dt + d]
    f4v dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < NJT; ++kc) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int j = kc * 16 + 4 * g + t;
        const float av = dSt[j * PLD + i0 + col];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma16(av, Ks[j * ATT_KLD + dt * 16 + col], dq[dt]);
      }
    }
    const BView DQ = head_view(a.dq, a.lddq, nq, qb, h * ATT_DK);
    const uint32_t dvo = (uint32_t)(i0 + 4 * g) * DQ.ld + ES * col;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (i0 + 4 * g + r < a.Tq) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          bstx1<T>(DQ, qm[r][dt] > 0.f ? dq[dt][r] : 0.f, dvo, r * DQ.ld + 16 * ES * dt);
      }
    }
  }
  __syncthreads();

  // ---- phase 2: dV^T = dO^T P, dK^T = Q^T dS (item = grp * NJT + jt, grp < 4 dV, >= 4 dK);
  //   A[m = d][k = i] = X[i][16 dt + d] (preloaded per group; query rows past Tq read as 0),
  //   B[k = i][n = j] = Y^T[j][i] (one b128 per 16 queries: lane group g feeds k = 16 kc + 4g + t
  //   at MFMA step t), D[m = 4g + r][n = col] = out[j = 16 jt + col][d = 16 dt + 4g + r]: one
  //   16-B store
  const int nitems = 8 * NJT;
  const int it0 = nitems * w / nw, it1 = nitems * (w + 1) / nw;
  constexpr int MAXG = 3;
  const int g0 = it0 / NJT;
  const uint32_t avo_o = (uint32_t)(4 * g) * DO.ld + 4u * col;
  const uint32_t avo_q = (uint32_t)(4 * g) * sv.q.ld + ES * col;
  float acol[MAXG][NJT][4];  // (query tiles: nw == NJT, host check)
#pragma unroll
  for (int u = 0; u < MAXG; ++u) {
    const int grp = g0 + u;
    if (grp * NJT < it1 && grp < 8) {  // wave-uniform
      const int dt = grp & 3;
#pragma unroll
      for (int kc = 0; kc < NJT; ++kc)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint32_t row = (uint32_t)(kc * 16 + t);
          const float x = grp < 4 ? bld1(DO, avo_o, row * DO.ld + 64u * dt)
                                  : bldx1<T>(sv.q, avo_q, row * sv.q.ld + 16 * ES * dt);
          acol[u][kc][t] = kc * 16 + 4 * g + t < a.Tq ? x : 0.f;
        }
    }
  }
  const BView DK = head_view(a.dk, a.lddk, nk, kb, h * ATT_DK);
  const BView DV = head_view(a.dv, a.lddv, nk, kb, h * ATT_DK);
  const bool vk = vec_rows(a.dk, a.lddk), vv = vec_rows(a.dv, a.lddv);
#pragma unroll
  for (int u = 0; u < MAXG; ++u) {
    const int grp = g0 + u;
    const int lo = max(it0, grp * NJT), hi = min(it1, (grp + 1) * NJT);
    if (grp >= 8 || lo >= hi) continue;  // wave-uniform
    const bool isv = grp < 4;
    const int dt = grp & 3;
    const float* Yt = isv ? Pt : dSt;
    const BView& D = isv ? DV : DK;
    const uint32_t svo = (uint32_t)col * D.ld + 4 * ES * g;
    const uint32_t vvo = (uint32_t)col * sv.v.ld + 4 * ES * g;
    for (int it = lo; it < hi; ++it) {
      const int jt = it - grp * NJT;
      const int j = jt * 16 + col;
      // ReLU mask: V from global (its LDS image is now P^T), K from its staged image
      const f4v mk = isv ? bldx4<T>(sv.v, vvo, (uint32_t)(jt * 16) * sv.v.ld + 16 * ES * dt)
                         : ld4(Ks + j * ATT_KLD + dt * 16 + 4 * g);
      f4v acc = {0.f, 0.f, 0.f, 0.f};
      const float* yrow = Yt + j * PLD + 4 * g;
#pragma unroll
      for (int kc = 0; kc < NJT; ++kc) {
        const f4v yv = ld4(yrow + kc * 16);
        acc = mfma16(acol[u][kc][0], yv.x, acc);
        acc = mfma16(acol[u][kc][1], yv.y, acc);
        acc = mfma16(acol[u][kc][2], yv.z, acc);
        acc = mfma16(acol[u][kc][3], yv.w, acc);
      }
      if (j < a.Tk) {
        f4v o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = mk[r] > 0.f ? acc[r] : 0.f;
        bstx4<T>(D, o, svo, (uint32_t)(jt * 16) * D.ld + 16 * ES * dt, isv ? vv : vk);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// bf16 MFMA strip kernels (bf16 training modes, cfg 3 / cfg 5). Same workgroup / wave /
// strip structure and the same fp32 softmax -> graph -> L1 chain (and adjoint) as the fp32
// kernels above, but the products run on bf16 matrix cores and every LDS image is bf16:
//   S = Q K^T, dP = dO V^T     v_mfma_f32_16x16x32_bf16, 2 per 16x16 tile (Q, K, V are bf16
//                              already: exact products, fp32 sums; dO is rounded to bf16);
//   O = P V, dV = P^T dO,      v_mfma_f32_16x16x16_bf16, one per 16 k (P and dS rounded to
//   dK = dS^T Q, dQ = dS K     bf16, as a bf16 attention's second GEMM does).
// The fp32 kernels issue 8x (S) / 4x (phase 2) as many 16x16x4 MFMAs. bf16 LDS images halve
// the footprint, which buys both more workgroups per CU (T = 73 backward: 3 instead of 2,
// VGPR-limited) and keeping K / V staged through the backward's phase 2 (50 KB).
// Both MFMA forms take operand k-sets by lane group (A[m = l&15][k in set(l>>4)],
// B[k in set(l>>4)][n = l&15], D[4(l>>4)+r][l&15]); A and B always use the same set, so the
// inner products are exact whatever the hardware's k order inside a set.
typedef __bf16 att_bf16x8 __attribute__((ext_vector_type(8)));
typedef short att_s4 __attribute__((ext_vector_type(4)));
constexpr int ATT_KLB = 72;  // staged K/V row (bf16): 144 B, conflict-free 16-B reads by 16 rows

__device__ __forceinline__ f4v mfma_bf32(att_bf16x8 a, att_bf16x8 b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4v mfma_bf16(att_bf16x4 a, att_bf16x4 b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(att_s4, a),
                                                   __builtin_bit_cast(att_s4, b), c, 0, 0, 0);
}
__device__ __forceinline__ att_bf16x8 cat8(att_bf16x4 lo, att_bf16x4 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ att_bf16x4 ldb4(const __bf16* p) {
  return *reinterpret_cast<const att_bf16x4*>(p);
}
__device__ __forceinline__ att_bf16x8 ldb8_lds(const __bf16* p) {
  return *reinterpret_cast<const att_bf16x8*>(p);
}
// strip operand: 8 consecutive d (32c + 8g ..) of a bf16 row / of an fp32 row rounded to bf16
__device__ __forceinline__ att_bf16x8 strip8(const __bf16* p) { return cat8(ldb4(p), ldb4(p + 4)); }
__device__ __forceinline__ att_bf16x8 strip8(const float* p) {
  return cat8(__builtin_convertvector(ld4(p), att_bf16x4), __builtin_convertvector(ld4(p + 4), att_bf16x4));
}

// K_h, V_h rows [0, TK) of sample b into bf16 LDS images [TK][ATT_KLB] (zero rows past Tk):
// thread t moves 16-B chunk t % 8 of rows t / 8 + 8 nw u' (one lane offset per view, the row
// block in soffset); batched like stage_kv_tiles (all loads of a batch issued before any store)
template <int TK>
__device__ __forceinline__ void stage_kv_bf(const BView& K, const BView& V, int Tk, __bf16* Ks,
                                            __bf16* Vs) {
  const int t = threadIdx.x, rstep = blockDim.x >> 3;
  const uint32_t kvo = (uint32_t)(t >> 3) * K.ld + 16u * (t & 7);
  const uint32_t vvo = (uint32_t)(t >> 3) * V.ld + 16u * (t & 7);
  for (int r0 = 0; r0 < TK; r0 += SKV_BATCH * rstep) {
    att_bf16x8 kv[SKV_BATCH], vv[SKV_BATCH];
#pragma unroll
    for (int u = 0; u < SKV_BATCH; ++u) {
      const uint32_t row = (uint32_t)(r0 + u * rstep);
      kv[u] = bld16b<att_bf16x8>(K, kvo, row * K.ld);
      vv[u] = bld16b<att_bf16x8>(V, vvo, row * V.ld);
    }
#pragma unroll
    for (int u = 0; u < SKV_BATCH; ++u) {
      const int j = r0 + u * rstep + (t >> 3), c8 = (t & 7) * 8;
      if (j < TK) {
        const bool ok = j < Tk;
        const att_bf16x8 z = {};
        *reinterpret_cast<att_bf16x8*>(&Ks[j * ATT_KLB + c8]) = ok ? kv[u] : z;
        *reinterpret_cast<att_bf16x8*>(&Vs[j * ATT_KLB + c8]) = ok ? vv[u] : z;
      }
    }
  }
}

// acc[jt] = X_strip . Y_tile(jt)^T over d = 64 (Y staged bf16 in LDS)
template <int NJT>
__device__ __forceinline__ void strip_dots_bf(const att_bf16x8 (&x)[2], const __bf16* Ys, int col,
                                              int g, f4v (&acc)[NJT]) {
#pragma unroll
  for (int jt = 0; jt < NJT; ++jt) {
    const __bf16* yr = Ys + (jt * 16 + col) * ATT_KLB + 8 * g;
    f4v s = {0.f, 0.f, 0.f, 0.f};
    s = mfma_bf32(x[0], ldb8_lds(yr), s);
    s = mfma_bf32(x[1], ldb8_lds(yr + 32), s);
    acc[jt] = s;
  }
}

__device__ __forceinline__ att_bf16x4 pack4(f4v v) { return __builtin_convertvector(v, att_bf16x4); }

template <int NJT>
__global__ __launch_bounds__(512) void gattn_fwd_mfma_bf_kernel(AttnArgsT<__bf16> a) {
  extern __shared__ __attribute__((aligned(16))) __bf16 smb[];
  const int bh = xcd_remap(blockIdx.x, gridDim.x);  // heads of a sample on one XCD
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int i0 = w * 16;
  constexpr int TK = NJT * 16;
  constexpr int WLB = 20;                  // per-wave P^T image [TK][16 + 4] bf16
  __bf16* Ks = smb;                        // [TK][ATT_KLB]
  __bf16* Vs = Ks + TK * ATT_KLB;          // [TK][ATT_KLB]
  __bf16* Pw = Vs + TK * ATT_KLB + w * TK * WLB;
  const StripViews<AttnArgsT<__bf16>> sv(a, b, h);
  att_bf16x8 qa[2];
  {
    const uint32_t vo = (uint32_t)(i0 + col) * sv.q.ld + 16u * g;
    qa[0] = bld16b<att_bf16x8>(sv.q, vo, 0);
    qa[1] = bld16b<att_bf16x8>(sv.q, vo, 64);
  }
  float gp[4][NJT], kf[NJT], qf[4];
  preload_graph<NJT>(sv.g, a.Tk, i0, g, col, gp);
  preload_flags<NJT>(sv.kf, sv.qf, i0, g, col, kf, qf);
  stage_kv_bf<TK>(sv.k, sv.v, a.Tk, Ks, Vs);
  __syncthreads();  // K/V staged
  f4v s[NJT];
  strip_dots_bf<NJT>(qa, Ks, col, g, s);
  f4v pv[NJT];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    float aa[NJT], gg[NJT], bm[NJT];
    const float nrm = strip_row_forward<NJT>(s, r, kf, gp[r], a.Tk, col, aa, gg, bm);
    const float rsd = __builtin_amdgcn_rcpf(fmaxf(nrm, 1e-12f));
#pragma unroll
    for (int jt = 0; jt < NJT; ++jt) {
      const int j = jt * 16 + col;
      const float n = bm[jt] * rsd;
      const bool ok = i < a.Tq && j < a.Tk;
      if (a.att && ok) a.att[(((int64_t)h * a.B + b) * a.Tq + i) * a.Tk + j] = n;
      pv[jt][r] = ok ? n * qf[r] : 0.f;
    }
  }
#pragma unroll
  for (int jt = 0; jt < NJT; ++jt)
    *reinterpret_cast<att_bf16x4*>(&Pw[(jt * 16 + col) * WLB + 4 * g]) = pack4(pv[jt]);
  __builtin_amdgcn_wave_barrier();  // this wave's P^T strip written (wave-private image)
  // O strip = P V: A[m = i][k = j] = P^T[j][i], B[k = j][n = d] = V[j][d]; k = 16 jc + 4g + t
  f4v o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int jc = 0; jc < NJT; ++jc) {
    const int j = jc * 16 + 4 * g;
    const att_bf16x4 pa = {Pw[j * WLB + col], Pw[(j + 1) * WLB + col], Pw[(j + 2) * WLB + col],
                           Pw[(j + 3) * WLB + col]};
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const __bf16* vc = Vs + j * ATT_KLB + dt * 16 + col;
      const att_bf16x4 vb = {vc[0], vc[ATT_KLB], vc[2 * ATT_KLB], vc[3 * ATT_KLB]};
      o[dt] = mfma_bf16(pa, vb, o[dt]);
    }
  }
  const BView O = head_view(a.o, a.ldo, (int64_t)a.B * a.Tq, (int64_t)b * a.Tq, h * ATT_DK);
  const uint32_t ovo = (uint32_t)(i0 + 4 * g) * O.ld + 4u * col;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (i0 + 4 * g + r < a.Tq) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) bst32(O, o[dt][r], ovo, r * O.ld + 64u * dt);
    }
  }
}

template <int NJT>
__global__ __launch_bounds__(512) void gattn_bwd_mfma_bf_kernel(AttnArgsT<__bf16> a) {
  extern __shared__ __attribute__((aligned(16))) __bf16 smb[];
  const int bh = xcd_remap(blockIdx.x, gridDim.x);  // heads of a sample on one XCD
  const int b = bh / a.H, h = bh % a.H;
  const int nw = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int i0 = w * 16;
  constexpr int TK = NJT * 16;
  // P^T / dS^T row stride (bf16): 16 nw + 8 keeps the 8-B row reads of 16 rows on disjoint
  // bank pairs and the scalar column reads of the 4 lane groups on disjoint bank ranges
  const int PLB = 16 * nw + 8;
  // K_h / V_h stay staged through phase 2 (not aliased by the P^T / dS^T images): dQ's B
  // operand and the dK / dV ReLU masks are LDS reads instead of global round trips (T = 73:
  // 50 KB, still 3 workgroups per CU, which the 114 VGPRs limit anyway; -17 % vs aliasing)
  __bf16* Ks = smb;                // [TK][ATT_KLB]
  __bf16* Vs = smb + TK * ATT_KLB;
  __bf16* Pt = Vs + TK * ATT_KLB;  // [TK][PLB]  P^T
  __bf16* dSt = Pt + TK * PLB;     // [TK][PLB]  dS^T (scaled by 1/8, masked)
  const int64_t qb = (int64_t)b * a.Tq, kb = (int64_t)b * a.Tk;
  const int hd = h * ATT_DK;

  // ---- phase 1: strips
  {
    att_bf16x8 qa[2], oa[2];
    const int iq = min(i0 + col, a.Tq - 1);
    const __bf16* qr = a.q + (qb + iq) * a.ldq + hd + 8 * g;
    const float* orr = a.dout + (qb + iq) * a.lddo + hd + 8 * g;
    qa[0] = strip8(qr);
    qa[1] = strip8(qr + 32);
    oa[0] = strip8(orr);
    oa[1] = strip8(orr + 32);
    float gp[4][NJT];
    const StripViews<std::remove_reference_t<decltype(a)>> sv(a, b, h);
    preload_graph<NJT>(sv.g, a.Tk, i0, g, col, gp);
    float kf[NJT];
#pragma unroll
    for (int jt = 0; jt < NJT; ++jt) kf[jt] = a.kflag[kb + min(jt * 16 + col, a.Tk - 1)];
    stage_kv_bf<TK>(sv.k, sv.v, a.Tk, Ks, Vs);
    __syncthreads();  // K/V staged
    f4v s[NJT], dp[NJT];
    strip_dots_bf<NJT>(qa, Ks, col, g, s);
    strip_dots_bf<NJT>(oa, Vs, col, g, dp);
    f4v pv[NJT], dsv[NJT];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * g + r;
      const int ic = min(i, a.Tq - 1);
      float aa[NJT], gg[NJT], bm[NJT];
      const float nrm = strip_row_forward<NJT>(s, r, kf, gp[r], a.Tk, col, aa, gg, bm);
      const float sden = fmaxf(nrm, 1e-12f);
      const float rsd = 1.f / sden;
      const float qf = a.qflag[qb + ic];
      float dn[NJT], t1 = 0.f;
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        dn[jt] = dp[jt][r] * qf;
        t1 += dn[jt] * bm[jt];
      }
      t1 = row16_sum(t1);
      const float dnrm = nrm >= 1e-12f ? -t1 * (rsd * rsd) : 0.f;
      float da[NJT], t2 = 0.f;
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        const float sg = bm[jt] > 0.f ? 1.f : (bm[jt] < 0.f ? -1.f : 0.f);
        const float dbm = dn[jt] * rsd + dnrm * sg;
        da[jt] = dbm * gg[jt];
        t2 += da[jt] * aa[jt];
      }
      t2 = row16_sum(t2);
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        const int j = jt * 16 + col;
        const bool ok = i < a.Tq && j < a.Tk;
        float ds = aa[jt] * (da[jt] - t2);
        if (kf[jt] == 0.f) ds = 0.f;
        dsv[jt][r] = ok ? ds * 0.125f : 0.f;
        pv[jt][r] = ok ? bm[jt] * rsd * qf : 0.f;
      }
    }
#pragma unroll
    for (int jt = 0; jt < NJT; ++jt) {
      *reinterpret_cast<att_bf16x4*>(&Pt[(jt * 16 + col) * PLB + i0 + 4 * g]) = pack4(pv[jt]);
      *reinterpret_cast<att_bf16x4*>(&dSt[(jt * 16 + col) * PLB + i0 + 4 * g]) = pack4(dsv[jt]);
    }
  }
  __syncthreads();

  // ---- phase 2: 16x16 output tiles, grouped (tensor, 16-column block dt) as in the fp32
  // kernel: [0,4) dV = P^T dO, [4,8) dK = dS^T Q (k = query), [8,12) dQ = dS K (k = key);
  // one 16x16x16 MFMA per 16 k, k = 16 kc + 4g + t
  const int nitems = 8 * NJT + 4 * nw;
  const int it0 = nitems * w / nw, it1 = nitems * (w + 1) / nw;
  int cur = -1;
  att_bf16x4 bcol[8];  // B rows k = 16 kc + 4g + t of column dt*16 + col (kc < 8)
  for (int it = it0; it < it1; ++it) {
    int grp, tile;
    if (it < 8 * NJT) {
      grp = it / NJT;
      tile = it - grp * NJT;
    } else {
      grp = 8 + (it - 8 * NJT) / nw;
      tile = (it - 8 * NJT) % nw;
    }
    const int dt = grp & 3;
    const int dcol = hd + dt * 16 + col;
    if (grp != cur) {  // wave-uniform
      cur = grp;
      const __bf16* src = grp < 8 ? a.q : a.k;  // dO (fp32) for grp < 4
      const int64_t ld = grp < 4 ? a.lddo : (grp < 8 ? a.ldq : a.ldk);
      const int64_t base = grp < 8 ? qb : kb;
      const int lim = grp < 8 ? a.Tq : a.Tk;
      const int nk = grp < 8 ? nw : NJT;
      if (grp >= 8) {  // dQ = dS K: K columns from the staged image
#pragma unroll
        for (int kc = 0; kc < NJT; ++kc) {
          const __bf16* kcp = Ks + (kc * 16 + 4 * g) * ATT_KLB + dt * 16 + col;
          bcol[kc] = att_bf16x4{kcp[0], kcp[ATT_KLB], kcp[2 * ATT_KLB], kcp[3 * ATT_KLB]};
        }
      } else
#pragma unroll
      for (int kc = 0; kc < 8; ++kc) {
        if (kc < nk) {
          float t4[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int64_t off = (base + min(kc * 16 + 4 * g + t, lim - 1)) * ld + dcol;
            t4[t] = grp < 4 ? a.dout[off] : (float)src[off];
          }
          bcol[kc] = pack4(f4v{t4[0], t4[1], t4[2], t4[3]});
        }
      }
    }
    // ReLU-mask values of this tile's 4 output rows, fetched before the MFMAs (clamped rows)
    float mk[4];
    {
      const __bf16* msrc = grp < 4 ? a.v : (grp < 8 ? a.k : a.q);
      const int64_t mld = grp < 4 ? a.ldv : (grp < 8 ? a.ldk : a.ldq);
      const int64_t base = grp < 8 ? kb : qb;
      const int lim = grp < 8 ? a.Tk : a.Tq;
      if (grp < 8) {  // dV / dK rows: masks of the staged V / K
        const __bf16* mc = (grp < 4 ? Vs : Ks) + (tile * 16 + 4 * g) * ATT_KLB + dt * 16 + col;
#pragma unroll
        for (int r = 0; r < 4; ++r) mk[r] = (float)mc[r * ATT_KLB];
      } else
#pragma unroll
      for (int r = 0; r < 4; ++r) mk[r] = (float)msrc[(base + min(tile * 16 + 4 * g + r, lim - 1)) * mld + dcol];
    }
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    if (grp < 8) {
      const bool isv = grp < 4;
      const __bf16* arow = (isv ? Pt : dSt) + (tile * 16 + col) * PLB + 4 * g;
#pragma unroll
      for (int kc = 0; kc < 8; ++kc)
        if (kc < nw) acc = mfma_bf16(ldb4(arow + kc * 16), bcol[kc], acc);
      __bf16* dst = isv ? a.dv : a.dk;
      const int64_t dld = isv ? a.lddv : a.lddk;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = tile * 16 + 4 * g + r;
        if (j < a.Tk) dst[(kb + j) * dld + dcol] = (__bf16)(mk[r] > 0.f ? acc[r] : 0.f);
      }
    } else {
#pragma unroll
      for (int kc = 0; kc < NJT; ++kc) {
        const __bf16* ac = dSt + (kc * 16 + 4 * g) * PLB + tile * 16 + col;
        const att_bf16x4 av = {ac[0], ac[PLB], ac[2 * PLB], ac[3 * PLB]};
        acc = mfma_bf16(av, bcol[kc], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = tile * 16 + 4 * g + r;
        if (i < a.Tq) a.dq[(qb + i) * a.lddq + dcol] = (__bf16)(mk[r] > 0.f ? acc[r] : 0.f);
      }
    }
  }
}

// Backward, second structure (SAVQA_ATT_BWD2): the round-2 kernel above spends its phase 2 on
// 8 NJT + 4 nw 16x16 tiles per workgroup whose B operands come from global memory per
// (tensor, column block) and whose 4 mask loads per tile are issued after the previous
// tile's stores (vmcnt counts stores: each tile waits for a store round trip), writing
// scalar bf16 elements. Here
//   * dQ = dS K moves into phase 1: each wave multiplies its own dS strip (read back from the
//     block dS^T image it just wrote, no barrier needed) by the staged K; the dQ masks
//     (Q > 0) are loaded before any store;
//   * phase 2 computes dV and dK TRANSPOSED, dV^T = dO^T P and dK^T = Q^T dS: the B operand is
//     then a contiguous 4-query run of a P^T / dS^T row (one 8-B LDS read), the ReLU mask a
//     4-column run of the staged V / K row (8-B LDS read), and each lane's 4 outputs are 4
//     consecutive d of one key row: one 8-B store instead of four 2-B ones;
//   * the A operands (dO / Q columns, k = query) of every (tensor, column block) group a wave
//     touches are loaded at the start of phase 2, before its first store.
template <int NJT>
__global__ __launch_bounds__(512) void gattn_bwd_mfma_bf2_kernel(AttnArgsT<__bf16> a) {
  extern __shared__ __attribute__((aligned(16))) __bf16 smb[];
  const int bh = xcd_remap(blockIdx.x, gridDim.x);  // heads of a sample on one XCD
  const int b = bh / a.H, h = bh % a.H;
  const int nw = blockDim.x >> 6;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int i0 = w * 16;
  constexpr int TK = NJT * 16;
  const int PLB = 16 * nw + 8;
  __bf16* Ks = smb;                // [TK][ATT_KLB]
  __bf16* Vs = smb + TK * ATT_KLB;
  // phase 2 overlays the K / V images with Q^T and dO^T ([64 d][PLB] each)
  __bf16* Pt = smb + max(2 * TK * ATT_KLB, 2 * ATT_DK * PLB);  // [TK][PLB]  P^T
  __bf16* dSt = Pt + TK * PLB;     // [TK][PLB]  dS^T (scaled by 1/8, masked)
  const StripViews<AttnArgsT<__bf16>> sv(a, b, h);
  const int64_t nq = (int64_t)a.B * a.Tq, nk = (int64_t)a.B * a.Tk;
  const int64_t qb = (int64_t)b * a.Tq, kb = (int64_t)b * a.Tk;
  const BView DO = head_view(a.dout, a.lddo, nq, qb, h * ATT_DK);

  // ---- phase 1: strips, then dQ of the strip
  att_bf16x8 qa[2], oa[2];  // Q / dO of this lane's strip row (kept for phase 2's images)
  {
    {
      const uint32_t qvo = (uint32_t)(i0 + col) * sv.q.ld + 16u * g;
      const uint32_t ovo = (uint32_t)(i0 + col) * DO.ld + 32u * g;
      qa[0] = bld16b<att_bf16x8>(sv.q, qvo, 0);
      qa[1] = bld16b<att_bf16x8>(sv.q, qvo, 64);
      f4v o4[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) o4[c] = bld16b<f4v>(DO, ovo, (c >> 1) * 128u + (c & 1) * 16u);
      oa[0] = cat8(pack4(o4[0]), pack4(o4[1]));
      oa[1] = cat8(pack4(o4[2]), pack4(o4[3]));
    }
    float gp[4][NJT], kf[NJT], qf[4];
    preload_graph<NJT>(sv.g, a.Tk, i0, g, col, gp);
    preload_flags<NJT>(sv.kf, sv.qf, i0, g, col, kf, qf);
    stage_kv_bf<TK>(sv.k, sv.v, a.Tk, Ks, Vs);
    __syncthreads();  // K/V staged
    f4v s[NJT], dp[NJT];
    strip_dots_bf<NJT>(qa, Ks, col, g, s);
    strip_dots_bf<NJT>(oa, Vs, col, g, dp);
    f4v pv[NJT], dsv[NJT];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 4 * g + r;
      float aa[NJT], gg[NJT], bm[NJT];
      const float nrm = strip_row_forward<NJT>(s, r, kf, gp[r], a.Tk, col, aa, gg, bm);
      const float rsd = __builtin_amdgcn_rcpf(fmaxf(nrm, 1e-12f));
      float dn[NJT], t1 = 0.f;
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        dn[jt] = dp[jt][r] * qf[r];
        t1 += dn[jt] * bm[jt];
      }
      t1 = row16_sum(t1);
      const float dnrm = nrm >= 1e-12f ? -t1 * (rsd * rsd) : 0.f;
      float da[NJT], t2 = 0.f;
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        const float sg = bm[jt] > 0.f ? 1.f : (bm[jt] < 0.f ? -1.f : 0.f);
        const float dbm = dn[jt] * rsd + dnrm * sg;
        da[jt] = dbm * gg[jt];
        t2 += da[jt] * aa[jt];
      }
      t2 = row16_sum(t2);
#pragma unroll
      for (int jt = 0; jt < NJT; ++jt) {
        const int j = jt * 16 + col;
        const bool ok = i < a.Tq && j < a.Tk;
        float ds = aa[jt] * (da[jt] - t2);
        if (kf[jt] == 0.f) ds = 0.f;
        dsv[jt][r] = ok ? ds * 0.125f : 0.f;
        pv[jt][r] = ok ? bm[jt] * rsd * qf[r] : 0.f;
      }
    }
#pragma unroll
    for (int jt = 0; jt < NJT; ++jt) {
      *reinterpret_cast<att_bf16x4*>(&Pt[(jt * 16 + col) * PLB + i0 + 4 * g]) = pack4(pv[jt]);
      *reinterpret_cast<att_bf16x4*>(&dSt[(jt * 16 + col) * PLB + i0 + 4 * g]) = pack4(dsv[jt]);
    }
    // dQ ReLU masks of this lane's outputs (rows i0 + 4g + r, columns 16 dt + col): loaded
    // here, where the strip registers are dead, under the dQ products below
    const uint32_t mvo = (uint32_t)(i0 + 4 * g) * sv.q.ld + 2u * col;
    unsigned short qm[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) qm[r][dt] = bld16(sv.q, mvo, r * sv.q.ld + 32u * dt);
    __builtin_amdgcn_wave_barrier();  // this wave's dS^T columns are written (in-order LDS)
    // dQ strip = dS K: A[m = i][k = j] = dS^T[j][i0 + i], B[k = j][n = d] = K[j][16 dt + d]
    f4v dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < NJT; ++kc) {
      const __bf16* ac = dSt + (kc * 16 + 4 * g) * PLB + i0 + col;
      const att_bf16x4 av = {ac[0], ac[PLB], ac[2 * PLB], ac[3 * PLB]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const __bf16* kcp = Ks + (kc * 16 + 4 * g) * ATT_KLB + dt * 16 + col;
        const att_bf16x4 kv = {kcp[0], kcp[ATT_KLB], kcp[2 * ATT_KLB], kcp[3 * ATT_KLB]};
        dq[dt] = mfma_bf16(av, kv, dq[dt]);
      }
    }
    const BView DQ = head_view(a.dq, a.lddq, nq, qb, h * ATT_DK);
    const uint32_t dvo = (uint32_t)(i0 + 4 * g) * DQ.ld + 2u * col;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (i0 + 4 * g + r < a.Tq) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const float m = (float)__builtin_bit_cast(__bf16, qm[r][dt]);
          bstx1<__bf16>(DQ, m > 0.f ? dq[dt][r] : 0.f, dvo, r * DQ.ld + 32u * dt);
        }
      }
    }
  }
  __syncthreads();

  // ---- Q^T and dO^T of every query over the K / V images (phase 2 reads K / V only for its
  // ReLU masks, which it loads from memory): each phase-2 A operand is then one 8-B LDS read
  // instead of four scattered global loads (the per-lane loads were ~20 % of the kernel)
  __bf16* Qt = smb;
  __bf16* Ot = smb + ATT_DK * PLB;
  {
    const int i = i0 + col;
    const bool ok = i < a.Tq;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int dd = 32 * hf + 8 * g + e;
        Qt[dd * PLB + i] = ok ? qa[hf][e] : (__bf16)0.f;
        Ot[dd * PLB + i] = ok ? oa[hf][e] : (__bf16)0.f;
      }
  }
  // ---- phase 2: dV^T = dO^T P and dK^T = Q^T dS, 16x16 tiles (key tile jt, column block dt),
  // grouped (tensor, dt): item = grp * NJT + jt, grp < 4 dV, grp >= 4 dK; k = query.
  //   A[m = d][k = i] = X^T[16 dt + d][i]   (X = dO rounded to bf16, or Q; rows i >= Tq zero)
  //   B[k = i][n = j] = Y^T[j][i]           (Y^T = P^T or dS^T)
  //   D[m = 4g + r][n = col] = out[j = 16 jt + col][d = 16 dt + 4g + r]
  const int nitems = 8 * NJT;
  const int it0 = nitems * w / nw, it1 = nitems * (w + 1) / nw;
  constexpr int MAXI = 8;  // items per wave (nw == NJT: checked on the host)
  // this wave's ReLU masks (K / V > 0 at its outputs), all loaded before its first store
  att_bf16x4 mkv[MAXI];
#pragma unroll
  for (int q = 0; q < MAXI; ++q) {
    const int it = it0 + q;
    mkv[q] = att_bf16x4{(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
    if (it < it1) {  // wave-uniform
      const int grp = it / NJT, jt = it - grp * NJT;
      const BView& M = grp < 4 ? sv.v : sv.k;
      mkv[q] = bld8b<att_bf16x4>(M, (uint32_t)(jt * 16 + col) * M.ld + 8u * g, 32u * (grp & 3));
    }
  }
  __syncthreads();  // Q^T / dO^T written
  const BView DK = head_view(a.dk, a.lddk, nk, kb, h * ATT_DK);
  const BView DV = head_view(a.dv, a.lddv, nk, kb, h * ATT_DK);
  const bool vk = vec_rows(a.dk, a.lddk), vv = vec_rows(a.dv, a.lddv);
#pragma unroll
  for (int q = 0; q < MAXI; ++q) {
    const int it = it0 + q;
    if (it >= it1) break;  // wave-uniform
    const int grp = it / NJT, jt = it - grp * NJT, dt = grp & 3;
    const bool isv = grp < 4;
    const __bf16* xcol = (isv ? Ot : Qt) + (16 * dt + col) * PLB + 4 * g;
    const int j = jt * 16 + col;
    const __bf16* yrow = (isv ? Pt : dSt) + j * PLB + 4 * g;
    f4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < NJT; ++kc) acc = mfma_bf16(ldb4(xcol + kc * 16), ldb4(yrow + kc * 16), acc);
    if (j < a.Tk) {
      f4v o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (float)mkv[q][r] > 0.f ? acc[r] : 0.f;
      const BView& D = isv ? DV : DK;
      bstx4<__bf16>(D, o, (uint32_t)col * D.ld + 8u * g, (uint32_t)(jt * 16) * D.ld + 32u * dt,
                    isv ? vv : vk);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Single-query path (T_q = 1: the decoder cross-attention, one query token per sample).
// One wave per (b, h); 16 lanes per key row (lane = (key slot kk = lane>>4, float4 chunk
// c = lane&15)), so every K/V load instruction reads 4 whole 256-B rows (coalesced) and
// a 16-lane DPP row reduction finishes each dot product. NIT = ceil(Tk/4) rounded up to
// a multiple of 8 (register arrays, compile-time indexed).
__device__ __forceinline__ float rows4_max(float v) {  // one value per 16-lane row -> all
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}
__device__ __forceinline__ float rows4_sum(float v) {
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ f4v xrow_sum(f4v v) {  // sum over the 4 rows, lane c keeps col c
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] += __shfl_xor(v[e], 16);
    v[e] += __shfl_xor(v[e], 32);
  }
  return v;
}

// s[it] (scaled, masked; -inf past Tk) and the forward chain for the single query of (b,h)
template <int NIT, class A>
__device__ __forceinline__ void q1_forward(const A& a, int b, int hd, int kk, int c,
                                           const f4v q4, float (&s)[NIT], float (&aa)[NIT],
                                           float (&gg)[NIT], float (&bm)[NIT], float& nrm) {
  const int64_t kb = (int64_t)b * a.Tk;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    float x = -INFINITY;
    if (4 * it < a.Tk) {
      const int j = 4 * it + kk;
      const f4v k4 = ldx4(a.k + (kb + min(j, a.Tk - 1)) * a.ldk + hd + 4 * c);
      const float d = row16_sum((q4.x * k4.x + q4.y * k4.y) + (q4.z * k4.z + q4.w * k4.w));
      if (j < a.Tk) x = a.kflag[kb + j] == 0.f ? ATT_MASKED : d * 0.125f;
    }
    s[it] = x;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int it = 0; it < NIT; ++it) mx = fmaxf(mx, s[it]);
  mx = rows4_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const float e = 4 * it + kk < a.Tk ? expf(s[it] - mx) : 0.f;
    aa[it] = e;
    sum += e;
  }
  sum = rows4_sum(sum);
  const float* grow = a.G + (int64_t)b * a.Tk;
  float nr = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int j = 4 * it + kk;
    aa[it] = aa[it] / sum;
    gg[it] = j < a.Tk ? grow[j] : 0.f;
    bm[it] = gg[it] * aa[it];
    nr += fabsf(bm[it]);
  }
  nrm = rows4_sum(nr);
}


template <int NIT, typename TQ, typename TKV>
__global__ __launch_bounds__(256) void gattn_fwd_q1_kernel(AttnArgsT<TQ, TKV> a) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.x * 4 + w;
  if (bh >= a.B * a.H) return;  // wave-uniform
  const int b = bh / a.H, h = bh % a.H, hd = h * ATT_DK;
  const int kk = lane >> 4, c = lane & 15;
  const f4v q4 = ldx4(a.q + (int64_t)b * a.ldq + hd + 4 * c);
  float s[NIT], aa[NIT], gg[NIT], bm[NIT], nrm;
  q1_forward<NIT>(a, b, hd, kk, c, q4, s, aa, gg, bm, nrm);
  const float sden = fmaxf(nrm, 1e-12f);
  const float qf = a.qflag[b];
  const int64_t kb = (int64_t)b * a.Tk;
  f4v o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    if (4 * it < a.Tk) {
      const int j = 4 * it + kk;
      const float n = bm[it] / sden;
      if (a.att && c == 0 && j < a.Tk) a.att[((int64_t)h * a.B + b) * a.Tk + j] = n;
      const float pj = j < a.Tk ? n * qf : 0.f;
      const f4v v4 = ldx4(a.v + (kb + min(j, a.Tk - 1)) * a.ldv + hd + 4 * c);
      o += pj * v4;
    }
  }
  o = xrow_sum(o);
  if (kk == 0) stx4(a.o + (int64_t)b * a.ldo + hd + 4 * c, o, vec_rows(a.o, a.ldo));
}

// bf16 K/V: capped at 128 VGPRs (4 waves per SIMD, so all B*H waves of cfg 3 are resident at
// once instead of 1.33 rounds at 3 per SIMD); the cap's spills are cheaper than the lost
// occupancy there (bf16 T = 73: 94 -> 72 us) but not for fp32 K/V (55 -> 65 us: uncapped)
template <int NIT, typename TQ, typename TKV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sizeof(TKV) == 2 ? 4 : 1)))
void gattn_bwd_q1_kernel(AttnArgsT<TQ, TKV> a) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.x * 4 + w;
  if (bh >= a.B * a.H) return;
  const int b = bh / a.H, h = bh % a.H, hd = h * ATT_DK;
  const int kk = lane >> 4, c = lane & 15;
  const int64_t kb = (int64_t)b * a.Tk;
  const f4v q4 = ldx4(a.q + (int64_t)b * a.ldq + hd + 4 * c);
  const f4v do4 = ld4(a.dout + (int64_t)b * a.lddo + hd + 4 * c);
  float s[NIT], aa[NIT], gg[NIT], bm[NIT], nrm;
  q1_forward<NIT>(a, b, hd, kk, c, q4, s, aa, gg, bm, nrm);
  const float sden = fmaxf(nrm, 1e-12f);
  const float qf = a.qflag[b];
  // dP_j = dO . V_j ; dN = dP * qf
  float dn[NIT], t1 = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    float x = 0.f;
    if (4 * it < a.Tk) {
      const int j = 4 * it + kk;
      const f4v v4 = ldx4(a.v + (kb + min(j, a.Tk - 1)) * a.ldv + hd + 4 * c);
      x = row16_sum((do4.x * v4.x + do4.y * v4.y) + (do4.z * v4.z + do4.w * v4.w)) * qf;
      if (j >= a.Tk) x = 0.f;
    }
    dn[it] = x;
    t1 += x * bm[it];
  }
  t1 = rows4_sum(t1);
  const float dnrm = nrm >= 1e-12f ? -t1 / (sden * sden) : 0.f;
  float t2 = 0.f;
  const bool vk = vec_rows(a.dk, a.lddk), vv = vec_rows(a.dv, a.lddv);
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const float sg = bm[it] > 0.f ? 1.f : (bm[it] < 0.f ? -1.f : 0.f);
    const float dbm = dn[it] / sden + dnrm * sg;
    dn[it] = dbm * gg[it];  // da
    t2 += dn[it] * aa[it];
  }
  t2 = rows4_sum(t2);
  f4v dq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    if (4 * it < a.Tk) {
      const int j = 4 * it + kk;
      const bool ok = j < a.Tk;
      float ds = aa[it] * (dn[it] - t2);
      if (!ok || a.kflag[kb + min(j, a.Tk - 1)] == 0.f) ds = 0.f;
      ds *= 0.125f;
      const float pj = ok ? bm[it] / sden * qf : 0.f;
      const int64_t row = kb + min(j, a.Tk - 1);
      const f4v k4 = ldx4(a.k + row * a.ldk + hd + 4 * c);
      const f4v v4 = ldx4(a.v + row * a.ldv + hd + 4 * c);
      dq += ds * k4;
      if (ok) {
        f4v gk, gv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gk[e] = k4[e] > 0.f ? ds * q4[e] : 0.f;
          gv[e] = v4[e] > 0.f ? pj * do4[e] : 0.f;
        }
        stx4(a.dk + row * a.lddk + hd + 4 * c, gk, vk);
        stx4(a.dv + row * a.lddv + hd + 4 * c, gv, vv);
      }
    }
  }
  dq = xrow_sum(dq);
  if (kk == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) dq[e] = q4[e] > 0.f ? dq[e] : 0.f;
    stx4(a.dq + (int64_t)b * a.lddq + hd + 4 * c, dq, vec_rows(a.dq, a.lddq));
  }
}

// Single-query path split over the 4 waves of a workgroup (SAVQA_ATT_Q1W, the default): one
// workgroup per (b, h); wave w takes keys [4 NI w, 4 NI (w + 1)) as NI iterations of 4 key
// rows (lane = (key slot kk, float4 chunk c) as above) and keeps its K / V rows in registers
// from the first load to the last use. The softmax max and sum, the L1 norm, the adjoint's
// t1 / t2 and the output / dQ partials cross the waves through LDS, one slot per wave (and per
// exchange: no slot is reused, so each exchange costs one barrier), folded in wave order: every
// lane and every rerun sees the same bits. One (b, h) is then one load round trip for 16 NI
// keys spread over 4 waves, where the one-wave kernels above walk ceil(T_k / 4) iterations and
// read K / V twice (their register arrays do not hold the rows between the passes).
#ifndef SAVQA_ATT_Q1W
#define SAVQA_ATT_Q1W 1
#endif

__device__ __forceinline__ float q1w_sum4(const float* r) { return (r[0] + r[1]) + (r[2] + r[3]); }
__device__ __forceinline__ float q1w_max4(const float* r) {
  return fmaxf(fmaxf(r[0], r[1]), fmaxf(r[2], r[3]));
}

// K / V rows, graph weights and key flags of this wave's keys (rows past T_k clamped to the
// last one: valid addresses, masked at use)
template <int NI, typename TQ, typename TKV>
__device__ __forceinline__ void q1w_load(const AttnArgsT<TQ, TKV>& a, int b, int hd, int j0, int kk,
                                         int c, f4v (&k4)[NI], f4v (&v4)[NI], float (&gg)[NI],
                                         float (&kf)[NI]) {
  const int64_t kb = (int64_t)b * a.Tk;
  const float* grow = a.G + kb;
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    const int j = j0 + 4 * it + kk;
    const int64_t row = kb + min(j, a.Tk - 1);
    k4[it] = ldx4(a.k + row * a.ldk + hd + 4 * c);
    v4[it] = ldx4(a.v + row * a.ldv + hd + 4 * c);
    gg[it] = j < a.Tk ? grow[min(j, a.Tk - 1)] : 0.f;
    kf[it] = a.kflag[row];
  }
}

// softmax over all 4 waves' keys -> aa (0 past T_k), bm = g * aa; red: 2 x 4 LDS slots
template <int NI>
__device__ __forceinline__ void q1w_softmax(const f4v q4, const f4v (&k4)[NI], const float (&gg)[NI],
                                            const float (&kf)[NI], int j0, int kk, int Tk, int w,
                                            int lane, float (*red)[4], float (&aa)[NI],
                                            float (&bm)[NI]) {
  float s[NI], mx = -INFINITY;
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    const f4v k = k4[it];
    const float d = row16_sum((q4.x * k.x + q4.y * k.y) + (q4.z * k.z + q4.w * k.w));
    const int j = j0 + 4 * it + kk;
    s[it] = j < Tk ? (kf[it] == 0.f ? ATT_MASKED : d * 0.125f) : -INFINITY;
    mx = fmaxf(mx, s[it]);
  }
  mx = rows4_max(mx);
  if (lane == 0) red[0][w] = mx;
  __syncthreads();
  const float M = q1w_max4(red[0]);
  float sum = 0.f;
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    aa[it] = j0 + 4 * it + kk < Tk ? expf(s[it] - M) : 0.f;
    sum += aa[it];
  }
  sum = rows4_sum(sum);
  if (lane == 0) red[1][w] = sum;
  __syncthreads();
  const float Z = q1w_sum4(red[1]);
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    aa[it] = aa[it] / Z;
    bm[it] = gg[it] * aa[it];
  }
}

template <int NI, typename TQ, typename TKV>
__global__ __launch_bounds__(256) void gattn_fwd_q1w_kernel(AttnArgsT<TQ, TKV> a) {
  __shared__ float red[3][4];
  __shared__ f4v ured[4][16];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int bh = xcd_remap(blockIdx.x, gridDim.x);  // the heads of a sample on one XCD
  const int b = bh / a.H, h = bh % a.H, hd = h * ATT_DK;
  const int kk = lane >> 4, c = lane & 15;
  const int j0 = 4 * NI * w;
  const f4v q4 = ldx4(a.q + (int64_t)b * a.ldq + hd + 4 * c);
  f4v k4[NI], v4[NI];
  float gg[NI], kf[NI], aa[NI], bm[NI];
  q1w_load<NI>(a, b, hd, j0, kk, c, k4, v4, gg, kf);
  q1w_softmax<NI>(q4, k4, gg, kf, j0, kk, a.Tk, w, lane, red, aa, bm);
  float nr = 0.f;
  f4v u = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    nr += fabsf(bm[it]);
    u += bm[it] * v4[it];  // 0 past T_k (g = 0 there)
  }
  nr = rows4_sum(nr);
  u = xrow_sum(u);
  if (lane == 0) red[2][w] = nr;
  if (kk == 0) ured[w][c] = u;
  __syncthreads();
  const float sden = fmaxf(q1w_sum4(red[2]), 1e-12f);
  if (a.att && c == 0) {
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int j = j0 + 4 * it + kk;
      if (j < a.Tk) a.att[((int64_t)h * a.B + b) * a.Tk + j] = bm[it] / sden;
    }
  }
  if (w == 0 && kk == 0) {
    const f4v o = ((ured[0][c] + ured[1][c]) + (ured[2][c] + ured[3][c])) * (a.qflag[b] / sden);
    stx4(a.o + (int64_t)b * a.ldo + hd + 4 * c, o, vec_rows(a.o, a.ldo));
  }
}

template <int NI, typename TQ, typename TKV>
__global__ __launch_bounds__(256) void gattn_bwd_q1w_kernel(AttnArgsT<TQ, TKV> a) {
  __shared__ float red[5][4];
  __shared__ f4v qred[4][16];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int bh = xcd_remap(blockIdx.x, gridDim.x);
  const int b = bh / a.H, h = bh % a.H, hd = h * ATT_DK;
  const int kk = lane >> 4, c = lane & 15;
  const int j0 = 4 * NI * w;
  const int64_t kb = (int64_t)b * a.Tk;
  const f4v q4 = ldx4(a.q + (int64_t)b * a.ldq + hd + 4 * c);
  const f4v do4 = ld4(a.dout + (int64_t)b * a.lddo + hd + 4 * c);
  const float qf = a.qflag[b];
  f4v k4[NI], v4[NI];
  float gg[NI], kf[NI], aa[NI], bm[NI];
  q1w_load<NI>(a, b, hd, j0, kk, c, k4, v4, gg, kf);
  q1w_softmax<NI>(q4, k4, gg, kf, j0, kk, a.Tk, w, lane, red, aa, bm);
  // dP_j = dO . V_j ; dN = dP * qf ; t1 = sum dN bm, with the L1 norm in the same exchange
  float dn[NI], t1 = 0.f, nr = 0.f;
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    const f4v v = v4[it];
    const float x = row16_sum((do4.x * v.x + do4.y * v.y) + (do4.z * v.z + do4.w * v.w)) * qf;
    dn[it] = j0 + 4 * it + kk < a.Tk ? x : 0.f;
    t1 += dn[it] * bm[it];
    nr += fabsf(bm[it]);
  }
  t1 = rows4_sum(t1);
  nr = rows4_sum(nr);
  if (lane == 0) {
    red[2][w] = nr;
    red[3][w] = t1;
  }
  __syncthreads();
  const float nrm = q1w_sum4(red[2]);
  const float sden = fmaxf(nrm, 1e-12f);
  const float dnrm = nrm >= 1e-12f ? -q1w_sum4(red[3]) / (sden * sden) : 0.f;
  float t2 = 0.f;
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    const float sg = bm[it] > 0.f ? 1.f : (bm[it] < 0.f ? -1.f : 0.f);
    dn[it] = (dn[it] / sden + dnrm * sg) * gg[it];  // da
    t2 += dn[it] * aa[it];
  }
  t2 = rows4_sum(t2);
  if (lane == 0) red[4][w] = t2;
  __syncthreads();
  t2 = q1w_sum4(red[4]);
  const bool vk = vec_rows(a.dk, a.lddk), vv = vec_rows(a.dv, a.lddv);
  f4v dq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    const int j = j0 + 4 * it + kk;
    const bool ok = j < a.Tk;
    float ds = aa[it] * (dn[it] - t2);
    if (!ok || kf[it] == 0.f) ds = 0.f;
    ds *= 0.125f;
    const float pj = ok ? bm[it] / sden * qf : 0.f;
    dq += ds * k4[it];
    if (ok) {
      f4v gk, gv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gk[e] = k4[it][e] > 0.f ? ds * q4[e] : 0.f;
        gv[e] = v4[it][e] > 0.f ? pj * do4[e] : 0.f;
      }
      const int64_t row = kb + j;
      stx4(a.dk + row * a.lddk + hd + 4 * c, gk, vk);
      stx4(a.dv + row * a.lddv + hd + 4 * c, gv, vv);
    }
  }
  dq = xrow_sum(dq);
  if (kk == 0) qred[w][c] = dq;
  __syncthreads();
  if (w == 0 && kk == 0) {
    f4v r = (qred[0][c] + qred[1][c]) + (qred[2][c] + qred[3][c]);
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = q4[e] > 0.f ? r[e] : 0.f;
    stx4(a.dq + (int64_t)b * a.lddq + hd + 4 * c, r, vec_rows(a.dq, a.lddq));
  }
}

template <typename TQ, typename TKV>
static int validate(const AttnArgsT<TQ, TKV>& a, int64_t dk, const char* who) {
  constexpr uintptr_t AQ = sizeof(TQ) * 4 - 1, AK = sizeof(TKV) * 4 - 1;  // 4-element vector loads
  if (dk != ATT_DK) return fail(SAVQA_EUNSUP, std::string(who) + ": head dim must be 64");
  if (a.Tk <= 0 || a.Tq <= 0 || a.B <= 0 || a.H <= 0) return fail(SAVQA_EINVAL, std::string(who) + ": empty");
  if (a.Tk > 128) return fail(SAVQA_EUNSUP, std::string(who) + ": Tk > 128 not supported yet");
  if ((((uintptr_t)a.q) & AQ) || ((((uintptr_t)a.k) | ((uintptr_t)a.v)) & AK) || (a.ldk & 3) ||
      (a.ldv & 3) || (a.ldq & 3))
    return fail(SAVQA_EINVAL, std::string(who) + ": Q/K/V must be vector-aligned with ld % 4 == 0");
  if (a.Tq > 128) return fail(SAVQA_EUNSUP, std::string(who) + ": Tq > 128 not supported yet");
  return 0;
}

// Path choice: 2 = single-query kernels (T_q = 1), 1 = MFMA strip kernels (T_q > 1).
template <typename TQ, typename TKV>
static int attn_path(const AttnArgsT<TQ, TKV>& a) {
  return a.Tq == 1 ? 2 : 1;
}

static int q1_nit(int Tk) { return ((Tk + 3) / 4 + 7) / 8 * 8; }

template <typename TQ, typename TKV>
static int launch_fwd(AttnArgsT<TQ, TKV>& a, int64_t dk, hipStream_t s, const char* who) {
  if (int rc = validate(a, dk, who)) return rc;
  const int B = a.B, H = a.H, Tq = a.Tq, Tk = a.Tk;
  const int path = attn_path(a);
  if (path != 2 && !std::is_same<TQ, TKV>::value)
    return fail(SAVQA_EUNSUP, std::string(who) + ": fp32 Q with bf16 K/V needs T_q = 1");
  if (path == 2 && SAVQA_ATT_Q1W) {
    const dim3 g((unsigned)(B * H));
    switch ((Tk + 15) / 16) {
#define SAVQA_Q1W_CASE(N)                                                                      \
  case N: hipLaunchKernelGGL((gattn_fwd_q1w_kernel<N, TQ, TKV>), g, dim3(256), 0, s, a); break;
      SAVQA_Q1W_CASE(1) SAVQA_Q1W_CASE(2) SAVQA_Q1W_CASE(3) SAVQA_Q1W_CASE(4)
      SAVQA_Q1W_CASE(5) SAVQA_Q1W_CASE(6) SAVQA_Q1W_CASE(7) SAVQA_Q1W_CASE(8)
#undef SAVQA_Q1W_CASE
    }
  } else if (path == 2) {
    const dim3 g((unsigned)((B * H + 3) / 4));
    switch (q1_nit(Tk)) {
      case 8: hipLaunchKernelGGL((gattn_fwd_q1_kernel<8, TQ, TKV>), g, dim3(256), 0, s, a); break;
      case 16: hipLaunchKernelGGL((gattn_fwd_q1_kernel<16, TQ, TKV>), g, dim3(256), 0, s, a); break;
      case 24: hipLaunchKernelGGL((gattn_fwd_q1_kernel<24, TQ, TKV>), g, dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL((gattn_fwd_q1_kernel<32, TQ, TKV>), g, dim3(256), 0, s, a); break;
    }
  } else if (path == 1) {
    if constexpr (std::is_same<TQ, TKV>::value) {
    using T = TKV;
    const int njt = (Tk + 15) / 16, nw = (Tq + 15) / 16;
    const size_t lds = sizeof(float) * ((size_t)njt * 16 * ATT_KLD +
                                        std::max((size_t)njt * 16 * ATT_KLD, (size_t)nw * njt * 16 * 20));
    if constexpr (sizeof(T) == 2) {
      // bf16 MFMA kernels: bf16 K/V images + per-wave bf16 P^T images
      const size_t ldsb = 2 * ((size_t)2 * njt * 16 * ATT_KLB + (size_t)nw * njt * 16 * 20);
      switch (njt) {
#define SAVQA_FWD_CASE(N)                                                                       \
  case N:                                                                                       \
    hipLaunchKernelGGL((gattn_fwd_mfma_bf_kernel<N>), dim3(B * H), dim3(64 * nw), ldsb, s, a);  \
    break;
        SAVQA_FWD_CASE(1) SAVQA_FWD_CASE(2) SAVQA_FWD_CASE(3) SAVQA_FWD_CASE(4)
        SAVQA_FWD_CASE(5) SAVQA_FWD_CASE(6) SAVQA_FWD_CASE(7) SAVQA_FWD_CASE(8)
#undef SAVQA_FWD_CASE
      }
    } else {
    switch (njt) {
#define SAVQA_FWD_CASE(N)                                                                      \
  case N:                                                                                      \
    hipLaunchKernelGGL((gattn_fwd_mfma_kernel<N, T>), dim3(B * H), dim3(64 * nw), lds, s, a);  \
    break;
      SAVQA_FWD_CASE(1) SAVQA_FWD_CASE(2) SAVQA_FWD_CASE(3) SAVQA_FWD_CASE(4)
      SAVQA_FWD_CASE(5) SAVQA_FWD_CASE(6) SAVQA_FWD_CASE(7) SAVQA_FWD_CASE(8)
#undef SAVQA_FWD_CASE
    }
    }
    }
  }
  return check_launch(who);
}

template <typename TQ, typename TKV>
static int launch_bwd(AttnArgsT<TQ, TKV>& a, int64_t dk, hipStream_t s, const char* who) {
  if (int rc = validate(a, dk, who)) return rc;
  const int B = a.B, H = a.H, Tq = a.Tq, Tk = a.Tk;
  const int path = attn_path(a);
  if (path != 2 && !std::is_same<TQ, TKV>::value)
    return fail(SAVQA_EUNSUP, std::string(who) + ": fp32 Q with bf16 K/V needs T_q = 1");
  if (((a.lddo & 3) || (((uintptr_t)a.dout) & 15)))
    return fail(SAVQA_EINVAL, std::string(who) + ": dO must be 16-B aligned with ld % 4 == 0");
  if (path == 2 && SAVQA_ATT_Q1W) {
    const dim3 g((unsigned)(B * H));
    switch ((Tk + 15) / 16) {
#define SAVQA_Q1W_CASE(N)                                                                      \
  case N: hipLaunchKernelGGL((gattn_bwd_q1w_kernel<N, TQ, TKV>), g, dim3(256), 0, s, a); break;
      SAVQA_Q1W_CASE(1) SAVQA_Q1W_CASE(2) SAVQA_Q1W_CASE(3) SAVQA_Q1W_CASE(4)
      SAVQA_Q1W_CASE(5) SAVQA_Q1W_CASE(6) SAVQA_Q1W_CASE(7) SAVQA_Q1W_CASE(8)
#undef SAVQA_Q1W_CASE
    }
    return check_launch(who);
  }
  if (path == 2) {
    const dim3 g((unsigned)((B * H + 3) / 4));
    switch (q1_nit(Tk)) {
      case 8: hipLaunchKernelGGL((gattn_bwd_q1_kernel<8, TQ, TKV>), g, dim3(256), 0, s, a); break;
      case 16: hipLaunchKernelGGL((gattn_bwd_q1_kernel<16, TQ, TKV>), g, dim3(256), 0, s, a); break;
      case 24: hipLaunchKernelGGL((gattn_bwd_q1_kernel<24, TQ, TKV>), g, dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL((gattn_bwd_q1_kernel<32, TQ, TKV>), g, dim3(256), 0, s, a); break;
    }
    return check_launch(who);
  }
  if (path == 1) {
    if constexpr (std::is_same<TQ, TKV>::value) {
    using T = TKV;
    const int njt = (Tk + 15) / 16, nw = (Tq + 15) / 16;
    if constexpr (sizeof(T) == 2) {
      // bf16 MFMA kernels: bf16 K/V images kept next to the bf16 P^T / dS^T images
      const size_t ldsb = 2 * 2 * (size_t)njt * 16 * (size_t)(16 * nw + 8 + ATT_KLB);
      // second structure: phase 2 overlays the K / V images with Q^T / dO^T [64][16 nw + 8]
      const size_t ldsb2 = 2 * (std::max(2 * (size_t)njt * 16 * ATT_KLB, 2 * (size_t)ATT_DK * (16 * nw + 8)) +
                                2 * (size_t)njt * 16 * (size_t)(16 * nw + 8));
      // second structure (transposed dV / dK, dQ in phase 1): as many query as key tiles (the
      // self-attention shape), so a wave's phase-2 item run is 8 NJT / nw = 8 items
      const bool v2 = SAVQA_ATT_BWD2 && nw == njt;
      switch (njt) {
#define SAVQA_BWD_CASE(N)                                                                       \
  case N:                                                                                       \
    if (v2) hipLaunchKernelGGL((gattn_bwd_mfma_bf2_kernel<N>), dim3(B * H), dim3(64 * nw), ldsb2, s, a); \
    else hipLaunchKernelGGL((gattn_bwd_mfma_bf_kernel<N>), dim3(B * H), dim3(64 * nw), ldsb, s, a); \
    break;
        SAVQA_BWD_CASE(1) SAVQA_BWD_CASE(2) SAVQA_BWD_CASE(3) SAVQA_BWD_CASE(4)
        SAVQA_BWD_CASE(5) SAVQA_BWD_CASE(6) SAVQA_BWD_CASE(7) SAVQA_BWD_CASE(8)
#undef SAVQA_BWD_CASE
      }
    } else {
    const size_t lds = sizeof(float) * 2 * (size_t)njt * 16 * (size_t)std::max(16 * nw + 4, ATT_KLD);
    // v2: K [TK][ATT_KLD] + max(V, P^T) + dS^T [TK][16 nw + 4] (over the 160 KB of a CU at
    // TK = 128: the round-2 structure then)
    const size_t lds2 = sizeof(float) * (size_t)njt * 16 *
                        ((size_t)ATT_KLD + std::max(16 * nw + 4, ATT_KLD) + (size_t)(16 * nw + 4));
    const bool v2 = SAVQA_ATT_BWD2 && nw == njt && (8 * njt + nw - 1) / nw <= 2 * njt &&
                    lds2 <= 160 * 1024;
    switch (njt) {
#define SAVQA_BWD_CASE(N)                                                                      \
  case N:                                                                                      \
    if (v2) hipLaunchKernelGGL((gattn_bwd_mfma2_kernel<N, T>), dim3(B * H), dim3(64 * nw), lds2, s, a); \
    else hipLaunchKernelGGL((gattn_bwd_mfma_kernel<N, T>), dim3(B * H), dim3(64 * nw), lds, s, a);  \
    break;
      SAVQA_BWD_CASE(1) SAVQA_BWD_CASE(2) SAVQA_BWD_CASE(3) SAVQA_BWD_CASE(4)
      SAVQA_BWD_CASE(5) SAVQA_BWD_CASE(6) SAVQA_BWD_CASE(7) SAVQA_BWD_CASE(8)
#undef SAVQA_BWD_CASE
    }
    }
    }
  }
  return check_launch(who);
}

template <typename TQ, typename TKV>
static AttnArgsT<TQ, TKV> make_args(const void* q, int64_t ldq, const void* k, int64_t ldk,
                                    const void* v, int64_t ldv, const float* G, const float* kflag,
                                    const float* qflag, int64_t B, int64_t Tq, int64_t Tk,
                                    int64_t H) {
  AttnArgsT<TQ, TKV> a{};
  a.q = static_cast<const TQ*>(q); a.ldq = ldq;
  a.k = static_cast<const TKV*>(k); a.ldk = ldk;
  a.v = static_cast<const TKV*>(v); a.ldv = ldv;
  a.G = G; a.kflag = kflag; a.qflag = qflag;
  a.B = (int)B; a.Tq = (int)Tq; a.Tk = (int)Tk; a.H = (int)H;
  return a;
}

}  // namespace savqa

using namespace savqa;

extern "C" int savqa_gattn_fwd(void* stream, const float* q, int64_t ldq, const float* k,
                               int64_t ldk, const float* v, int64_t ldv, const float* G,
                               const float* kflag, const float* qflag, int64_t B, int64_t Tq,
                               int64_t Tk, int64_t H, int64_t dk, float* o, int64_t ldo,
                               float* att) {
  AttnArgs a = make_args<float, float>(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H);
  a.o = o; a.ldo = ldo; a.att = att;
  return launch_fwd(a, dk, as_stream(stream), "savqa_gattn_fwd");
}

extern "C" int savqa_gattn_bwd(void* stream, const float* q, int64_t ldq, const float* k,
                               int64_t ldk, const float* v, int64_t ldv, const float* G,
                               const float* kflag, const float* qflag, int64_t B, int64_t Tq,
                               int64_t Tk, int64_t H, int64_t dk, const float* dout, int64_t lddo,
                               float* dq, int64_t lddq, float* dk_, int64_t lddk, float* dv,
                               int64_t lddv) {
  AttnArgs a = make_args<float, float>(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H);
  a.dout = dout; a.lddo = lddo; a.dq = dq; a.lddq = lddq; a.dk = dk_; a.lddk = lddk;
  a.dv = dv; a.lddv = lddv;
  return launch_bwd(a, dk, as_stream(stream), "savqa_gattn_bwd");
}

template <typename TQ>
static int fwd_bf16(void* stream, const void* q, int64_t ldq, const void* k, int64_t ldk,
                    const void* v, int64_t ldv, const float* G, const float* kflag,
                    const float* qflag, int64_t B, int64_t Tq, int64_t Tk, int64_t H, int64_t dk,
                    float* o, int64_t ldo, float* att) {
  auto a = make_args<TQ, __bf16>(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H);
  a.o = o; a.ldo = ldo; a.att = att;
  return launch_fwd(a, dk, as_stream(stream), "savqa_gattn_fwd_bf16");
}

template <typename TQ>
static int bwd_bf16(void* stream, const void* q, int64_t ldq, const void* k, int64_t ldk,
                    const void* v, int64_t ldv, const float* G, const float* kflag,
                    const float* qflag, int64_t B, int64_t Tq, int64_t Tk, int64_t H, int64_t dk,
                    const float* dout, int64_t lddo, void* dq, int64_t lddq, void* dk_,
                    int64_t lddk, void* dv, int64_t lddv) {
  auto a = make_args<TQ, __bf16>(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H);
  a.dout = dout; a.lddo = lddo;
  a.dq = static_cast<TQ*>(dq); a.lddq = lddq;
  a.dk = static_cast<__bf16*>(dk_); a.lddk = lddk;
  a.dv = static_cast<__bf16*>(dv); a.lddv = lddv;
  return launch_bwd(a, dk, as_stream(stream), "savqa_gattn_bwd_bf16");
}

extern "C" int savqa_gattn_fwd_bf16(void* stream, int32_t q_bf16, const void* q, int64_t ldq,
                                    const void* k, int64_t ldk, const void* v, int64_t ldv,
                                    const float* G, const float* kflag, const float* qflag,
                                    int64_t B, int64_t Tq, int64_t Tk, int64_t H, int64_t dk,
                                    float* o, int64_t ldo, float* att) {
  return q_bf16 ? fwd_bf16<__bf16>(stream, q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H,
                                   dk, o, ldo, att)
                : fwd_bf16<float>(stream, q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H,
                                  dk, o, ldo, att);
}

extern "C" int savqa_gattn_bwd_bf16(void* stream, int32_t q_bf16, const void* q, int64_t ldq,
                                    const void* k, int64_t ldk, const void* v, int64_t ldv,
                                    const float* G, const float* kflag, const float* qflag,
                                    int64_t B, int64_t Tq, int64_t Tk, int64_t H, int64_t dk,
                                    const float* dout, int64_t lddo, void* dq, int64_t lddq,
                                    void* dk_, int64_t lddk, void* dv, int64_t lddv) {
  return q_bf16 ? bwd_bf16<__bf16>(stream, q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H,
                                   dk, dout, lddo, dq, lddq, dk_, lddk, dv, lddv)
                : bwd_bf16<float>(stream, q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H,
                                  dk, dout, lddo, dq, lddq, dk_, lddk, dv, lddv);
}
