// Key-tiled ("flash") graph-guided attention for long sequences, gfx950.
//
// Same operator as attn.hip (new_multihead_attention.forward, models/modules.py:246-301):
//   S = Q_h K_h^T / 8, masked keys -> -4294967296, A = softmax over ALL keys,
//   N = (A*G) / max(sum|A*G|, 1e-12), P = N * qflag, O_h = P V_h
// but without holding a whole score row: keys stream through LDS in tiles of 64 and
// every query row keeps running statistics (online softmax):
//   m = max_j s_j,  Z = sum_j e_j,  W = sum_j e_j |g_j|,  acc = sum_j e_j g_j v_j,
//   e_j = exp(s_j - m)  (rescaled by exp(m_old - m_new) when m grows)
// and O = acc * qflag / D with D = max(W, 1e-12 Z)  ( == (e g / Z) / max(W / Z, 1e-12) ).
// Used for T_k > 128 (cfg 4's 114/449-token stacks, super-node relation graphs up to
// T = 1600) where the full-row kernels' registers/LDS do not fit.
//
// Backward (per row i, with c_i = [W_i >= 1e-12 Z_i], n = e g / D, P = e / Z):
//   delta_i = sum_j n_ij dN_ij,  dN_ij = qflag_i dO_i . V_j   (= dO_i . O_i analytically;
//             computed from the dN values themselves, and n from W, Z re-summed over the
//             backward's own e values, so sum_j dS_ij = 0 holds to rounding)
//   dS_ij = n_ij (dN_ij - c_i sgn(g_ij) delta_i) - (1 - c_i) P_ij delta_i   (0 on masked keys)
// i.e. the softmax / L1-normalise adjoints collapse to per-row scalars, so the backward
// is three tiled kernels: delta (workgroup per query tile, one sweep over the key tiles),
// dQ (the same tiles, a second sweep: dS and dQ) and dK, dV (workgroup per key tile, loop
// over query tiles), all recomputing S from the saved (m, Z, W). stats = [B*H*Tq][4]
// floats: m, Z, W, delta. The delta sweep is its own kernel so that neither sweep holds
// the other's registers (three and four workgroups per CU instead of two for the fused one).
#include "attn_common.h"

namespace savqa {

constexpr int FL_KT = 64;   // keys (or queries) per staged tile
constexpr int FL_WLD = 16;  // per-wave transposed image, [64][16] floats, rows placed by fl_img

// Float offset of element (r, f) of a per-wave [64][16] image. Unpadded (64 B rows), so the
// 4-wave forward workgroup takes 51200 B of LDS and three fit a CU (55296 B with 20-float
// padded rows: two). Rows are placed so that the 16-B column-group writes (lanes: 16
// consecutive rows r, one group f = 4g) and the row reads of fl_accum (lanes: 16 columns of
// the 4 rows j, j+4, j+8, j+12) both fall on distinct banks: the row's 64-B window is
// (r + r/4) mod 4 of its 4-row block, and the column group is XORed with (r/4) mod 4.
__device__ __forceinline__ int fl_img(int r, int f) {
  const int h = (r >> 2) & 3;
  return (((r & ~3) | ((r + h) & 3)) << 4) + (f ^ (h << 2));
}

// Cooperative stage of rows [r0, r0 + 64) of X and Y (head slice hd) into LDS, zero past lim.
__device__ __forceinline__ void fl_stage2(const float* X, int64_t ldx, const float* Y, int64_t ldy,
                                          int64_t base, int r0, int lim, int hd, float* Xs,
                                          float* Ys) {
  for (int idx = threadIdx.x; idx < FL_KT * 16; idx += blockDim.x) {
    const int j = idx >> 4, c4 = (idx & 15) * 4;
    f4v xv = {0.f, 0.f, 0.f, 0.f}, yv = xv;
    if (r0 + j < lim) {
      const int64_t row = base + r0 + j;
      xv = ld4(X + row * ldx + hd + c4);
      yv = ld4(Y + row * ldy + hd + c4);
    }
    *reinterpret_cast<f4v*>(&Xs[j * ATT_KLD + c4]) = xv;
    *reinterpret_cast<f4v*>(&Ys[j * ATT_KLD + c4]) = yv;
  }
}

__device__ __forceinline__ void fl_load_strip(const float* X, int64_t ldx, int64_t row, int hd,
                                              int g, f4v (&x)[4]) {
  const float* p = X + row * ldx + hd + 4 * g;
#pragma unroll
  for (int c = 0; c < 4; ++c) x[c] = ld4(p + 16 * c);
}

// acc[dt] += sum over the 64 rows j of the tile: img[j][col] (A: m = col, k = j) * Ys[j][16dt+col]
__device__ __forceinline__ void fl_accum(const float* img, const float* Ys, int col, int g,
                                         f4v (&acc)[4]) {
#pragma unroll
  for (int jc = 0; jc < 4; ++jc) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = jc * 16 + 4 * g + t;
      const float av = img[fl_img(j, col)];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma16(av, Ys[j * ATT_KLD + dt * 16 + col], acc[dt]);
    }
  }
}

// ---------------------------------------------------------------------------------- fwd
// grid = B*H*nqt, block = 64*nw (wave w: query strip qt*16nw + 16w)
__global__ __launch_bounds__(256) void gattn_fwd_flash_kernel(AttnArgs a, float* __restrict__ stats,
                                                             int nqt) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nw = blockDim.x >> 6;
  // XCD-aware: the tiles of a (sample, head) and the heads of a sample share an XCD's L2
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = bid % nqt, bh = bid / nqt;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int i0 = qt * 16 * nw + w * 16;
  float* Ks = sm;
  float* Vs = Ks + FL_KT * ATT_KLD;
  float* Pw = Vs + FL_KT * ATT_KLD + w * FL_KT * FL_WLD;
  const int64_t qb = (int64_t)b * a.Tq, kb = (int64_t)b * a.Tk;
  const int hd = h * ATT_DK;

  f4v qa[4];
  fl_load_strip(a.q, a.ldq, qb + min(i0 + col, a.Tq - 1), hd, g, qa);
  const float* grow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) grow[r] = a.G + (qb + min(i0 + 4 * g + r, a.Tq - 1)) * a.Tk;
  float m[4], Z[4], W[4];
  f4v o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = -INFINITY;
    Z[r] = 0.f;
    W[r] = 0.f;
    o[r] = f4v{0.f, 0.f, 0.f, 0.f};
  }
  const int nkt = (a.Tk + FL_KT - 1) / FL_KT;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * FL_KT;
    __syncthreads();  // every wave is done with the previous tile
    fl_stage2(a.k, a.ldk, a.v, a.ldv, kb, k0, a.Tk, hd, Ks, Vs);
    float kf[4], gv[4][4];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const int jc = min(k0 + jt * 16 + col, a.Tk - 1);
      kf[jt] = a.kflag[kb + jc];
#pragma unroll
      for (int r = 0; r < 4; ++r) gv[r][jt] = grow[r][jc];
    }
    __syncthreads();
    f4v s[4];
    strip_dots_lds<4>(qa, Ks, col, g, s);
    f4v pv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x[4], mx = -INFINITY;
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        const int j = k0 + jt * 16 + col;
        float v = -INFINITY;
        if (j < a.Tk) v = kf[jt] == 0.f ? ATT_MASKED : s[jt][r] * 0.125f;
        x[jt] = v;
        mx = fmaxf(mx, v);
      }
      mx = row16_max(mx);
      const float mn = fmaxf(m[r], mx);  // finite: every tile holds a key < Tk
      const float alpha = expf(m[r] - mn);
      float zs = 0.f, ws = 0.f;
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        const int j = k0 + jt * 16 + col;
        const float e = j < a.Tk ? expf(x[jt] - mn) : 0.f;
        const float gg = j < a.Tk ? gv[r][jt] : 0.f;
        zs += e;
        ws += e * fabsf(gg);
        pv[jt][r] = e * gg;
      }
      zs = row16_sum(zs);
      ws = row16_sum(ws);
      Z[r] = Z[r] * alpha + zs;
      W[r] = W[r] * alpha + ws;
      m[r] = mn;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt][r] *= alpha;
    }
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
      *reinterpret_cast<f4v*>(&Pw[fl_img(jt * 16 + col, 4 * g)]) = pv[jt];
    __builtin_amdgcn_wave_barrier();
    fl_accum(Pw, Vs, col, g, o);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    if (i < a.Tq) {
      const float D = fmaxf(W[r], 1e-12f * Z[r]);
      const float sc = a.qflag[qb + i] / D;
      float* orow = a.o + (qb + i) * a.ldo + hd + col;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) orow[dt * 16] = o[dt][r] * sc;
      if (col == 0) {
        float* st = stats + (((int64_t)b * a.H + h) * a.Tq + i) * 4;
        st[0] = m[r];
        st[1] = Z[r];
        st[2] = W[r];
      }
    }
  }
}

// per-row backward coefficients from (m, Z, W, delta, qflag):
//   dS = e*g*rD*qf*dp - cd*e*|g| - pd*e ,  nq = e*g*rD*qf
struct RowCoef {
  float m, rD, qf, cd, pd, rZ;
  bool normal;
};
__device__ __forceinline__ RowCoef row_coef(const float* st, float qf, bool valid) {
  RowCoef c;
  if (!valid) {
    c.m = INFINITY;  // e = exp(s - inf) = 0
    c.rD = c.qf = c.cd = c.pd = c.rZ = 0.f;
    c.normal = true;
    return c;
  }
  const float mm = st[0], Z = st[1], W = st[2];
  c.normal = W >= 1e-12f * Z;
  const float D = c.normal ? W : 1e-12f * Z;
  c.m = mm;
  c.rD = 1.f / D;
  c.rZ = 1.f / Z;
  c.qf = qf;
  c.cd = c.pd = 0.f;
  return c;
}
__device__ __forceinline__ void coef_delta(RowCoef& c, float dl) {
  c.cd = c.normal ? dl * c.rD : 0.f;
  c.pd = c.normal ? 0.f : dl * c.rZ;
}

// ------------------------------------------------------------------------- dK / dV
// grid = B*H*nkt2 (key tiles of 16*nw keys; wave w owns keys j0 = tile*16nw + 16w)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void gattn_bwd_kv_flash_kernel(AttnArgs a,
                                                                const float* __restrict__ stats,
                                                                int nkt2) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nw = blockDim.x >> 6;
  // XCD-aware: the tiles of a (sample, head) and the heads of a sample share an XCD's L2
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kt = bid % nkt2, bh = bid / nkt2;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int j0 = kt * 16 * nw + w * 16;
  float* Qs = sm;                                  // [64][KLD]
  float* dOs = Qs + FL_KT * ATT_KLD;               // [64][KLD]
  float* cf = dOs + FL_KT * ATT_KLD;               // [64][8] per-query coefficients
  float* img = cf + FL_KT * 8 + w * FL_KT * FL_WLD;  // [64 queries][16] (keys 4g+r): N, then dS
  const int64_t qb = (int64_t)b * a.Tq, kb = (int64_t)b * a.Tk;
  const int hd = h * ATT_DK;
  const float* sth = stats + ((int64_t)b * a.H + h) * a.Tq * 4;

  f4v ka[4], va[4];
  fl_load_strip(a.k, a.ldk, kb + min(j0 + col, a.Tk - 1), hd, g, ka);
  fl_load_strip(a.v, a.ldv, kb + min(j0 + col, a.Tk - 1), hd, g, va);
  float kf[4];
  bool kval[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = j0 + 4 * g + r;
    kval[r] = j < a.Tk;
    kf[r] = a.kflag[kb + min(j, a.Tk - 1)];
  }
  f4v dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = f4v{0.f, 0.f, 0.f, 0.f};
  const int nqt = (a.Tq + FL_KT - 1) / FL_KT;
  for (int qt = 0; qt < nqt; ++qt) {
    const int iq0 = qt * FL_KT;
    __syncthreads();
    fl_stage2(a.q, a.ldq, a.dout, a.lddo, qb, iq0, a.Tq, hd, Qs, dOs);
    if (threadIdx.x < FL_KT) {
      const int i = iq0 + threadIdx.x;
      const bool valid = i < a.Tq;
      const int ic = min(i, a.Tq - 1);
      RowCoef c = row_coef(sth + (int64_t)ic * 4, a.qflag[qb + ic], valid);
      if (valid) coef_delta(c, sth[(int64_t)ic * 4 + 3]);
      float* cp = cf + threadIdx.x * 8;
      cp[0] = c.m;
      cp[1] = c.rD;
      cp[2] = c.qf;
      cp[3] = c.cd;
      cp[4] = c.pd;
    }
    float gv[4][4];  // [jt][r]: G[query iq0 + 16jt + col][key j0 + 4g + r]
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const float* gr = a.G + (qb + min(iq0 + jt * 16 + col, a.Tq - 1)) * a.Tk;
#pragma unroll
      for (int r = 0; r < 4; ++r) gv[jt][r] = gr[min(j0 + 4 * g + r, a.Tk - 1)];
    }
    __syncthreads();
    f4v s[4], dp[4];
    strip_dots_lds<4>(ka, Qs, col, g, s);   // [key 4g+r][query 16jt+col]
    strip_dots_lds<4>(va, dOs, col, g, dp);
    f4v nv[4], dsv[4];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const float* cp = cf + (jt * 16 + col) * 8;
      const f4v c0 = ld4(cp);
      const float pd = cp[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = kf[r] == 0.f ? ATT_MASKED : s[jt][r] * 0.125f;
        const float e = kval[r] ? expf(x - c0.x) : 0.f;
        const float gg = gv[jt][r];
        const float n = e * gg * c0.y;
        nv[jt][r] = n * c0.z;
        const float ds = n * c0.z * dp[jt][r] - c0.w * e * fabsf(gg) - pd * e;
        dsv[jt][r] = kf[r] == 0.f ? 0.f : ds;
      }
      *reinterpret_cast<f4v*>(&img[fl_img(jt * 16 + col, 4 * g)]) = nv[jt];
    }
    __builtin_amdgcn_wave_barrier();
    fl_accum(img, dOs, col, g, dv);  // dV_j += sum_i nq_ij dO_i
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
      *reinterpret_cast<f4v*>(&img[fl_img(jt * 16 + col, 4 * g)]) = dsv[jt];
    __builtin_amdgcn_wave_barrier();
    fl_accum(img, Qs, col, g, dk);   // dK_j += sum_i dS_ij Q_i   (x 1/8 at the end)
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = j0 + 4 * g + r;
    if (j < a.Tk) {
      const int64_t row = kb + j;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int c = hd + dt * 16 + col;
        a.dk[row * a.lddk + c] = a.k[row * a.ldk + c] > 0.f ? dk[dt][r] * 0.125f : 0.f;
        a.dv[row * a.lddv + c] = a.v[row * a.ldv + c] > 0.f ? dv[dt][r] : 0.f;
      }
    }
  }
}

// --------------------------------------------------------------------------- delta
// grid = B*H*nqt (query tiles of 16*nw rows), one sweep over the key tiles.
// dQ_i = sum_j dS_ij K_j / 8 with sum_j dS_ij = 0 analytically: the keys' common part
// cancels, so any residual of that sum comes back as (residual) x (mean key) -- with
// near-parallel V rows (dN_ij ~ delta_i) it is larger than dQ itself. The residual of
// the direct form n (dN - delta) is ~1 ulp of delta (its rounding, and sum_j |n_j| != 1
// by rounding), which measured 15x torch-fp32's dQ error at T = 1313
// (tools/dbg/flash_prec.py). So, per row, with a_j = e g qf dp and w_j = e |g| (normal)
// or e (clamped), both the exact fp32 values the dQ sweep recomputes:
//   delta sweep: A = sum_j a_j, W' = sum_j e|g|, Z' = sum_j e in fp64;  dx = A / sum_j w_j
//   dQ sweep:    dS_j = rD (a_j - dx w_j), the bracket in fp64 (sum_j dS_j = 0 to fp64 rounding)
// i.e. the softmax / L1-normalise adjoint with its common term removed exactly, as torch's
// softmax backward (x (g - sum x g)) removes it. (W', Z', delta) go to stats for dK / dV;
// dx travels to the dQ kernel as a float pair (hi, lo) in columns 0-1 of the row's own dQ
// head slice, which only that kernel's same wave overwrites, after reading it.
__global__ __launch_bounds__(256) void gattn_bwd_delta_flash_kernel(AttnArgs a,
                                                                   float* __restrict__ stats,
                                                                   int nqt) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nw = blockDim.x >> 6;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = bid % nqt, bh = bid / nqt;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int i0 = qt * 16 * nw + w * 16;
  float* Ks = sm;
  float* Vs = Ks + FL_KT * ATT_KLD;
  const int64_t qb = (int64_t)b * a.Tq, kb = (int64_t)b * a.Tk;
  const int hd = h * ATT_DK;
  const float* sth = stats + ((int64_t)b * a.H + h) * a.Tq * 4;

  f4v qa[4], oa[4];
  fl_load_strip(a.q, a.ldq, qb + min(i0 + col, a.Tq - 1), hd, g, qa);
  fl_load_strip(a.dout, a.lddo, qb + min(i0 + col, a.Tq - 1), hd, g, oa);
  float rm[4], rq[4];
  const float* grow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    const int ic = min(i, a.Tq - 1);
    const RowCoef c = row_coef(sth + (int64_t)ic * 4, a.qflag[qb + ic], i < a.Tq);
    rm[r] = c.m;
    rq[r] = c.qf;
    grow[r] = a.G + (qb + ic) * a.Tk;
  }
  double sa[4] = {0., 0., 0., 0.}, sw[4] = {0., 0., 0., 0.}, sz[4] = {0., 0., 0., 0.};
  const int nkt = (a.Tk + FL_KT - 1) / FL_KT;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * FL_KT;
    __syncthreads();
    fl_stage2(a.k, a.ldk, a.v, a.ldv, kb, k0, a.Tk, hd, Ks, Vs);
    float kf[4], gv[4][4];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const int jc = min(k0 + jt * 16 + col, a.Tk - 1);
      kf[jt] = a.kflag[kb + jc];
#pragma unroll
      for (int r = 0; r < 4; ++r) gv[r][jt] = grow[r][jc];
    }
    __syncthreads();
    f4v s[4], dp[4];
    strip_dots_lds<4>(qa, Ks, col, g, s);   // [query 4g+r][key 16jt+col]
    strip_dots_lds<4>(oa, Vs, col, g, dp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        const int j = k0 + jt * 16 + col;
        const float x = kf[jt] == 0.f ? ATT_MASKED : s[jt][r] * 0.125f;
        const float e = j < a.Tk ? expf(x - rm[r]) : 0.f;
        const float gg = gv[r][jt];
        sa[r] += (double)(e * gg * rq[r] * dp[jt][r]);
        sw[r] += (double)(e * fabsf(gg));
        sz[r] += (double)e;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    double A = sa[r], Wd = sw[r], Zd = sz[r];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      A += __shfl_xor(A, o, 16);
      Wd += __shfl_xor(Wd, o, 16);
      Zd += __shfl_xor(Zd, o, 16);
    }
    if (i < a.Tq && col == 0) {
      const float wf = (float)Wd, zf = (float)Zd;
      const bool normal = wf >= 1e-12f * zf;
      const float rD = 1.f / (normal ? wf : 1e-12f * zf);
      const double den = normal ? Wd : Zd;
      const double dx = den > 0. ? A / den : 0.;
      float* st = stats + (((int64_t)b * a.H + h) * a.Tq + i) * 4;
      st[1] = zf;
      st[2] = wf;
      st[3] = normal ? (float)dx : (float)(dx * (double)rD * Zd);
      const float hi = (float)dx;
      float* dxs = a.dq + (qb + i) * a.lddq + hd;
      dxs[0] = hi;
      dxs[1] = (float)(dx - (double)hi);
    }
  }
}

// ------------------------------------------------------------------------------ dQ
// grid = B*H*nqt (query tiles of 16*nw rows), loop over key tiles; reads (m, Z', W') from
// stats and dx from the delta kernel (see above)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void gattn_bwd_q_flash_kernel(AttnArgs a,
                                                               const float* __restrict__ stats,
                                                               int nqt) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nw = blockDim.x >> 6;
  // XCD-aware: the tiles of a (sample, head) and the heads of a sample share an XCD's L2
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = bid % nqt, bh = bid / nqt;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int i0 = qt * 16 * nw + w * 16;
  float* Ks = sm;
  float* Vs = Ks + FL_KT * ATT_KLD;
  float* Simg = Vs + FL_KT * ATT_KLD + w * FL_KT * FL_WLD;  // [64 keys][16] (queries 4g+r)
  const int64_t qb = (int64_t)b * a.Tq, kb = (int64_t)b * a.Tk;
  const int hd = h * ATT_DK;
  const float* sth = stats + ((int64_t)b * a.H + h) * a.Tq * 4;

  f4v qa[4], oa[4];
  fl_load_strip(a.q, a.ldq, qb + min(i0 + col, a.Tq - 1), hd, g, qa);
  fl_load_strip(a.dout, a.lddo, qb + min(i0 + col, a.Tq - 1), hd, g, oa);
  RowCoef rc[4];
  const float* grow[4];
  double dx[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    const int ic = min(i, a.Tq - 1);
    rc[r] = row_coef(sth + (int64_t)ic * 4, a.qflag[qb + ic], i < a.Tq);
    grow[r] = a.G + (qb + ic) * a.Tk;
    const float* dxs = a.dq + (qb + ic) * a.lddq + hd;
    dx[r] = i < a.Tq ? (double)dxs[0] + (double)dxs[1] : 0.;
  }
  f4v dq[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dq[dt] = f4v{0.f, 0.f, 0.f, 0.f};
  const int nkt = (a.Tk + FL_KT - 1) / FL_KT;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * FL_KT;
    __syncthreads();
    fl_stage2(a.k, a.ldk, a.v, a.ldv, kb, k0, a.Tk, hd, Ks, Vs);
    float kf[4], gv[4][4];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const int jc = min(k0 + jt * 16 + col, a.Tk - 1);
      kf[jt] = a.kflag[kb + jc];
#pragma unroll
      for (int r = 0; r < 4; ++r) gv[r][jt] = grow[r][jc];
    }
    __syncthreads();
    f4v s[4], dp[4];
    strip_dots_lds<4>(qa, Ks, col, g, s);   // [query 4g+r][key 16jt+col]
    strip_dots_lds<4>(oa, Vs, col, g, dp);
    f4v dsv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const RowCoef c = rc[r];
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        const int j = k0 + jt * 16 + col;
        const float x = kf[jt] == 0.f ? ATT_MASKED : s[jt][r] * 0.125f;
        const float e = j < a.Tk ? expf(x - c.m) : 0.f;
        const float gg = gv[r][jt];
        const float av = e * gg * c.qf * dp[jt][r];
        const float wv = c.normal ? e * fabsf(gg) : e;
        const float ds = (float)((double)av - dx[r] * (double)wv) * c.rD;
        dsv[jt][r] = (kf[jt] == 0.f || j >= a.Tk) ? 0.f : ds;
      }
    }
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
      *reinterpret_cast<f4v*>(&Simg[fl_img(jt * 16 + col, 4 * g)]) = dsv[jt];
    __builtin_amdgcn_wave_barrier();
    fl_accum(Simg, Ks, col, g, dq);  // dQ_i += sum_j dS_ij K_j   (x 1/8 at the end)
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    if (i < a.Tq) {
      const int64_t row = qb + i;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int c = hd + dt * 16 + col;
        a.dq[row * a.lddq + c] = a.q[row * a.ldq + c] > 0.f ? dq[dt][r] * 0.125f : 0.f;
      }
    }
  }
}

static int flash_validate(const AttnArgs& a, int64_t dk, const char* who) {
  if (dk != ATT_DK) return fail(SAVQA_EUNSUP, std::string(who) + ": head dim must be 64");
  if (a.Tk <= 0 || a.Tq <= 0 || a.B <= 0 || a.H <= 0)
    return fail(SAVQA_EINVAL, std::string(who) + ": empty");
  const uintptr_t al = (uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v;
  if ((al & 15) || (a.ldq & 3) || (a.ldk & 3) || (a.ldv & 3))
    return fail(SAVQA_EINVAL, std::string(who) + ": Q/K/V must be 16-B aligned with ld % 4 == 0");
  return 0;
}

static int waves_for(int rows) { return rows >= 64 ? 4 : (rows + 15) / 16; }

}  // namespace savqa

using namespace savqa;

extern "C" int savqa_gattn_fwd_flash(void* stream, const float* q, int64_t ldq, const float* k,
                                     int64_t ldk, const float* v, int64_t ldv, const float* G,
                                     const float* kflag, const float* qflag, int64_t B,
                                     int64_t Tq, int64_t Tk, int64_t H, int64_t dk, float* o,
                                     int64_t ldo, float* stats) {
  AttnArgs a{};
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv; a.G = G;
  a.kflag = kflag; a.qflag = qflag; a.B = (int)B; a.Tq = (int)Tq; a.Tk = (int)Tk; a.H = (int)H;
  a.o = o; a.ldo = ldo;
  if (int rc = flash_validate(a, dk, "savqa_gattn_fwd_flash")) return rc;
  if (!stats) return fail(SAVQA_EINVAL, "savqa_gattn_fwd_flash: stats buffer required");
  const int nw = waves_for((int)Tq);
  const int nqt = (int)((Tq + 16 * nw - 1) / (16 * nw));
  const size_t lds = sizeof(float) * ((size_t)2 * FL_KT * ATT_KLD + (size_t)nw * FL_KT * FL_WLD);
  hipLaunchKernelGGL(gattn_fwd_flash_kernel, dim3((unsigned)(B * H * nqt)), dim3(64 * nw), lds,
                     as_stream(stream), a, stats, nqt);
  return check_launch("savqa_gattn_fwd_flash");
}

extern "C" int savqa_gattn_bwd_flash(void* stream, const float* q, int64_t ldq, const float* k,
                                     int64_t ldk, const float* v, int64_t ldv, const float* G,
                                     const float* kflag, const float* qflag, int64_t B,
                                     int64_t Tq, int64_t Tk, int64_t H, int64_t dk,
                                     const float* dout, int64_t lddo, float* stats,
                                     float* dq, int64_t lddq, float* dk_, int64_t lddk, float* dv,
                                     int64_t lddv) {
  AttnArgs a{};
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv; a.G = G;
  a.kflag = kflag; a.qflag = qflag; a.B = (int)B; a.Tq = (int)Tq; a.Tk = (int)Tk; a.H = (int)H;
  a.dout = dout; a.lddo = lddo; a.dq = dq; a.lddq = lddq; a.dk = dk_; a.lddk = lddk;
  a.dv = dv; a.lddv = lddv;
  if (int rc = flash_validate(a, dk, "savqa_gattn_bwd_flash")) return rc;
  if (!stats) return fail(SAVQA_EINVAL, "savqa_gattn_bwd_flash: stats required");
  if ((((uintptr_t)dout) & 15) || (lddo & 3))
    return fail(SAVQA_EINVAL, "savqa_gattn_bwd_flash: dO must be 16-B aligned, ld % 4 == 0");
  hipStream_t s = as_stream(stream);
  {  // delta (stats[..][3]) for the dK/dV pass and dx for the dQ pass, then dQ
    const int nw = waves_for((int)Tq);
    const int nqt = (int)((Tq + 16 * nw - 1) / (16 * nw));
    hipLaunchKernelGGL(gattn_bwd_delta_flash_kernel, dim3((unsigned)(B * H * nqt)), dim3(64 * nw),
                       sizeof(float) * (size_t)2 * FL_KT * ATT_KLD, s, a, stats, nqt);
    if (int rc = check_launch("savqa_gattn_bwd_flash(delta)")) return rc;
    const size_t lds = sizeof(float) * ((size_t)2 * FL_KT * ATT_KLD + (size_t)nw * FL_KT * FL_WLD);
    hipLaunchKernelGGL(gattn_bwd_q_flash_kernel, dim3((unsigned)(B * H * nqt)), dim3(64 * nw), lds,
                       s, a, stats, nqt);
    if (int rc = check_launch("savqa_gattn_bwd_flash(dq)")) return rc;
  }
  {
    const int nw = waves_for((int)Tk);
    const int nkt2 = (int)((Tk + 16 * nw - 1) / (16 * nw));
    const size_t lds = sizeof(float) * ((size_t)2 * FL_KT * ATT_KLD + FL_KT * 8 +
                                        (size_t)nw * FL_KT * FL_WLD);
    hipLaunchKernelGGL(gattn_bwd_kv_flash_kernel, dim3((unsigned)(B * H * nkt2)), dim3(64 * nw),
                       lds, s, a, stats, nkt2);
  }
  return check_launch("savqa_gattn_bwd_flash(dkv)");
}
