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

#ifndef SAVQA_FL_DELTA_WPE
#define SAVQA_FL_DELTA_WPE 3  // delta kernel occupancy (4: 128 VGPRs with 20 dwords spilled, 3-4 % slower)
#endif

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

// Cooperative stage of rows [r0, r0 + 64) of X and Y ((sample, head) views) into LDS, zero
// past lim: thread t moves 16-B chunk t % 16 of rows t / 16 + 4 nw p, four passes' loads
// issued back to back before their stores (one memory latency per batch instead of one per
// guarded pass); one lane offset per view, the row block in soffset.
__device__ __forceinline__ void fl_stage2(const BView& X, const BView& Y, int r0, int lim,
                                          float* Xs, float* Ys) {
  const int t = threadIdx.x, rstep = blockDim.x >> 4;
  const uint32_t xvo = (uint32_t)(t >> 4) * X.ld + 16u * (t & 15);
  const uint32_t yvo = (uint32_t)(t >> 4) * Y.ld + 16u * (t & 15);
  for (int p0 = 0; p0 < FL_KT; p0 += 4 * rstep) {
    f4v xv[4], yv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t row = (uint32_t)(r0 + p0 + u * rstep);
      xv[u] = bld16b<f4v>(X, xvo, row * X.ld);
      yv[u] = bld16b<f4v>(Y, yvo, row * Y.ld);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = p0 + u * rstep + (t >> 4), c4 = (t & 15) * 4;
      if (j < FL_KT) {
        const bool ok = r0 + j < lim;
        const f4v z = {0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f4v*>(&Xs[j * ATT_KLD + c4]) = ok ? xv[u] : z;
        *reinterpret_cast<f4v*>(&Ys[j * ATT_KLD + c4]) = ok ? yv[u] : z;
      }
    }
  }
}

// strip operand of row `row` (relative to the view): 16 consecutive d per lane group
__device__ __forceinline__ void fl_load_strip(const BView& X, int row, int g, f4v (&x)[4]) {
  const uint32_t vo = (uint32_t)row * X.ld + 16u * g;
#pragma unroll
  for (int c = 0; c < 4; ++c) x[c] = bld16b<f4v>(X, vo, 64u * c);
}

// graph values G[i0 + 4g + r][k0 + 16 jt + col] and key flags of one key tile (rows / columns
// past T: neighbouring or zero values, masked by the callers)
__device__ __forceinline__ void fl_graph_tile(const BView& G, const BView& KF, int Tk, int i0,
                                              int k0, int g, int col, float (&kf)[4],
                                              float (&gv)[4][4]) {
  const uint32_t vo = (uint32_t)((i0 + 4 * g) * Tk + col) * 4u;
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    kf[jt] = bld1(KF, 4u * col, 4u * (k0 + 16 * jt));
#pragma unroll
    for (int r = 0; r < 4; ++r) gv[r][jt] = bld1(G, vo, (uint32_t)(r * Tk + k0 + 16 * jt) * 4u);
  }
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

// ------------------------------------------------------------- x6 products (SAVQA_FLASH_X6)
// The same kernels with every product on v_mfma_f32_16x16x32_bf16 over exact three-term bf16
// splits (the x6 GEMM's scheme, gemm_x6.hip: a = a0 + a1 + a2 truncated, six of the nine
// partial products, each exact in the fp32 accumulator): 96 bf16 MFMAs of 16 cycles where the
// fp32 16x16x4 form takes 128 of 32 per staged tile and wave. Every product is computed
// "swapped" -- the per-lane strip (the wave's 16 queries, or keys) is the B operand and the
// staged tile the A operand -- so the score tile comes out with the strip on the lanes and 16
// tile rows in registers: the online softmax reduces over registers and the 4 lane groups, and
// the following product (P V, dS K, ...) that sums over those rows takes the registers as its
// B operand with no LDS round trip. Its A operand (the staged tile, transposed) comes from
// ds_read_b64_tr_b16 reads of the same row-major bf16 planes the score product reads by rows.
#ifndef SAVQA_FLASH_X6
#define SAVQA_FLASH_X6 1
#endif
#ifndef SAVQA_FX_WPE_Q
#define SAVQA_FX_WPE_Q 3   // waves per SIMD the dQ / dK dV kernels are built for
#endif
#ifndef SAVQA_FX_WPE_KV
#define SAVQA_FX_WPE_KV 2
#endif
#ifndef SAVQA_FX_WPE_KVP
#define SAVQA_FX_WPE_KVP 2  // the pre-split (planes) dK / dV kernel (3: 39 VGPRs spilled)
#endif
typedef __bf16 fx_bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 fx_bf4 __attribute__((ext_vector_type(4)));
typedef short fx_s4 __attribute__((ext_vector_type(4)));
constexpr int FX_ROWB = 128;               // bytes per staged row and plane (64 bf16)
constexpr int FX_PLANE = FL_KT * FX_ROWB;  // 8 KB
constexpr int FX_TILE = 3 * FX_PLANE;      // one staged 64 x 64 tile: 24 KB

// Tile rows on the MFMA rows: row m = 4g + r of score block jt is tile row 16g + 4jt + r, so
// a lane group's registers cover 16 consecutive tile rows (16-B graph / flag loads) and the
// following product's k step s takes rows 16g + 8s .. +7.
__device__ __forceinline__ int fx_trow(int jt, int m) { return 16 * (m >> 2) + 4 * jt + (m & 3); }
// byte offset of (row, d) in a plane: 16-B chunk d / 8 XORed with row bits (5, 1, 4), so the
// ds_read_b128 row reads (16 lanes: rows fx_trow(jt, 0..15)) and the transposed reads (a
// 32-lane half: rows 16g + 8s + 4h + 0..3 for two g) hit distinct banks
__device__ __forceinline__ int fx_off(int row, int d) {
  const int f = ((row >> 5) & 1) | (((row >> 1) & 1) << 1) | (((row >> 4) & 1) << 2);
  return row * FX_ROWB + ((((d >> 3) ^ f) & 7) << 4) + ((d & 7) << 1);
}

// exact truncation split of 4 fp32 values into three bf16 terms (gemm_x6.hip split3)
__device__ __forceinline__ void fx_split4(f4v v, fx_bf4& p0, fx_bf4& p1, fx_bf4& p2) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  uint32_t t[3][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    f2 x = f2{v[2 * h], v[2 * h + 1]};
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const uint32_t ux = __float_as_uint(x[0]), uy = __float_as_uint(x[1]);
      t[p][h] = __builtin_amdgcn_perm(uy, ux, 0x07060302u);
      if (p < 2) x = x - f2{__uint_as_float(ux & 0xffff0000u), __uint_as_float(uy & 0xffff0000u)};
    }
  }
  p0 = __builtin_bit_cast(fx_bf4, u2{t[0][0], t[0][1]});
  p1 = __builtin_bit_cast(fx_bf4, u2{t[1][0], t[1][1]});
  p2 = __builtin_bit_cast(fx_bf4, u2{t[2][0], t[2][1]});
}
__device__ __forceinline__ fx_bf8 fx_cat(fx_bf4 lo, fx_bf4 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// 8 fp32 values -> three bf16x8 terms
__device__ __forceinline__ void fx_split8(f4v lo, f4v hi, fx_bf8 (&p)[3]) {
  fx_bf4 a[3], b[3];
  fx_split4(lo, a[0], a[1], a[2]);
  fx_split4(hi, b[0], b[1], b[2]);
#pragma unroll
  for (int t = 0; t < 3; ++t) p[t] = fx_cat(a[t], b[t]);
}
__device__ __forceinline__ f4v fx_mfma(fx_bf8 a, fx_bf8 b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// c += A B over one 32-wide k step from split operands, the small products first
__device__ __forceinline__ f4v fx_mfma6(const fx_bf8 (&a)[3], const fx_bf8 (&b)[3], f4v c) {
  c = fx_mfma(a[2], b[0], c);
  c = fx_mfma(a[1], b[1], c);
  c = fx_mfma(a[0], b[2], c);
  c = fx_mfma(a[1], b[0], c);
  c = fx_mfma(a[0], b[1], c);
  return fx_mfma(a[0], b[0], c);
}

// Cooperative stage of rows [r0, r0 + 64) of X and Y into LDS as three bf16 planes each
// (fx_off layout), zero past lim: thread t splits 16-B chunk t % 16 of rows t / 16 + 4 nw p.
__device__ __forceinline__ void fx_stage2(const BView& X, const BView& Y, int r0, int lim,
                                          char* Xs, char* Ys) {
  const int t = threadIdx.x, rstep = blockDim.x >> 4;
  const uint32_t xvo = (uint32_t)(t >> 4) * X.ld + 16u * (t & 15);
  const uint32_t yvo = (uint32_t)(t >> 4) * Y.ld + 16u * (t & 15);
  for (int p0 = 0; p0 < FL_KT; p0 += 4 * rstep) {
    f4v xv[4], yv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t row = (uint32_t)(r0 + p0 + u * rstep);
      xv[u] = bld16b<f4v>(X, xvo, row * X.ld);
      yv[u] = bld16b<f4v>(Y, yvo, row * Y.ld);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = p0 + u * rstep + (t >> 4);
      if (j < FL_KT) {
        const bool ok = r0 + j < lim;
        const f4v z = {0.f, 0.f, 0.f, 0.f};
        const int off = fx_off(j, 4 * (t & 15));
        fx_bf4 a0, a1, a2;
        fx_split4(ok ? xv[u] : z, a0, a1, a2);
        *reinterpret_cast<fx_bf4*>(Xs + off) = a0;
        *reinterpret_cast<fx_bf4*>(Xs + FX_PLANE + off) = a1;
        *reinterpret_cast<fx_bf4*>(Xs + 2 * FX_PLANE + off) = a2;
        fx_split4(ok ? yv[u] : z, a0, a1, a2);
        *reinterpret_cast<fx_bf4*>(Ys + off) = a0;
        *reinterpret_cast<fx_bf4*>(Ys + FX_PLANE + off) = a1;
        *reinterpret_cast<fx_bf4*>(Ys + 2 * FX_PLANE + off) = a2;
      }
    }
  }
}

// the lane's strip row as the B operand: X[row][32s + 8g .. +7], split (s = 0, 1)
__device__ __forceinline__ void fx_load_strip(const BView& X, int row, int g, fx_bf8 (&xp)[2][3]) {
  const uint32_t vo = (uint32_t)row * X.ld + 32u * g;
#pragma unroll
  for (int s = 0; s < 2; ++s)
    fx_split8(bld16b<f4v>(X, vo, 128u * s), bld16b<f4v>(X, vo, 128u * s + 16u), xp[s]);
}

// Pre-split operands (savqa_gattn_*_flash_ws): Q / K / V / dO of every (sample, head) split
// ONCE into bf16 plane tiles in global memory, in exactly the LDS image layout above -- tile t
// of (b, h) at ((b H + h) nt + t) FX_TILE bytes, rows past T zero -- so the kernels stage a tile
// with 16-B LDS-DMAs (no split VALU, no registers; every query tile's workgroup used to re-split
// the same K / V tiles) and read their strips' planes directly.
struct FxPlanes {
  const char* q;
  const char* k;
  const char* v;
  const char* dout;
  int ntq, ntk;  // tiles per (sample, head) of the query / key operands
};
typedef __attribute__((address_space(3))) void fx_lds_void;
__device__ __forceinline__ void fx_dma16(const void* src, char* dst) {
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(fx_lds_void*)dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(l) : "memory");
}
// DMA two pre-split tiles into LDS: wave w copies 1-KB chunks w, w + nw, ... of each; the
// caller's __syncthreads follows
__device__ __forceinline__ void fx_stage_dma(const char* x, const char* y, char* Xs, char* Ys,
                                             int w, int nw, int lane) {
  for (int c = w; c < FX_TILE / 1024; c += nw) {
    fx_dma16(x + c * 1024 + lane * 16, Xs + c * 1024);
    fx_dma16(y + c * 1024 + lane * 16, Ys + c * 1024);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// DMA one pre-split tile (no wait): wave w copies 1-KB chunks w, w + nw, ...
__device__ __forceinline__ void fx_dma_tile(const char* x, char* Xs, int w, int nw, int lane) {
  for (int c = w; c < FX_TILE / 1024; c += nw) fx_dma16(x + c * 1024 + lane * 16, Xs + c * 1024);
}
// vmcnt(0) through the builtin (expcnt / lgkmcnt left at their maxima), so that the
// compiler's waitcnt pass sees it too and drops its own later waits for loads it covers (an
// asm wait is invisible to it: it then waits again, and that wait also drains the DMAs issued
// after those loads)
__device__ __forceinline__ void fx_wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// the lane's strip row from pre-split tiles (tiles: the (sample, head)'s first tile)
__device__ __forceinline__ void fx_strip_planes(const char* tiles, int row, int g,
                                                fx_bf8 (&xp)[2][3]) {
  const char* tb = tiles + (int64_t)(row >> 6) * FX_TILE;
  const int r = row & 63;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int t = 0; t < 3; ++t)
      xp[s][t] = *reinterpret_cast<const fx_bf8*>(tb + t * FX_PLANE + fx_off(r, 32 * s + 8 * g));
}
__device__ __forceinline__ const char* fx_tiles(const char* base, int b, int H, int h, int nt) {
  return base + ((int64_t)b * H + h) * nt * (int64_t)FX_TILE;
}

// graph / key-flag values of the lane's query (row q of the sample) for the tile's keys
// k0 + 16g + 4jt + r (16-B loads; reads past T come back as neighbouring or zero values and are
// masked by the callers)
__device__ __forceinline__ void fx_graph_row(const BView& G, const BView& KF, uint32_t gvo,
                                             int k0, int g, f4v (&gv)[4], uint32_t& kmask) {
  kmask = 0;
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    const uint32_t so = (uint32_t)(k0 + 4 * jt) * 4u;
    const f4v kf = bld16b<f4v>(KF, 64u * g, so);
    gv[jt] = bld16b<f4v>(G, gvo, so);
#pragma unroll
    for (int r = 0; r < 4; ++r) kmask |= (kf[r] == 0.f ? 1u : 0u) << (4 * jt + r);
  }
}

// acc[jt][r] = sum_d T[16g + 4jt + r][d] * strip[col][d]: the staged tile's rows
// against the lane strip (A = tile rows by ds_read_b128, B = the strip's planes)
template <int NJT>
__device__ __forceinline__ void fx_dots(const char* Ts, const fx_bf8 (&xp)[2][3], int col, int g,
                                        f4v (&acc)[NJT]) {
#pragma unroll
  for (int jt = 0; jt < NJT; ++jt) {
    const int row = fx_trow(jt, col);
    f4v c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int off = fx_off(row, 32 * s + 8 * g);
      fx_bf8 a[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) a[t] = *reinterpret_cast<const fx_bf8*>(Ts + t * FX_PLANE + off);
      c = fx_mfma6(a, xp[s], c);
    }
    acc[jt] = c;
  }
}

// 4 bf16 of column (lane % 16) of 4 tile rows, by the transposed read (T10): the lane
// supplies row `row`, columns d .. d + 3
__device__ __forceinline__ fx_bf4 fx_tr(const char* base, int off) {
  typedef __attribute__((address_space(3))) fx_s4 lds_s4;
  const fx_s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(const_cast<char*>(base) + off));
  return __builtin_bit_cast(fx_bf4, v);
}

// o[dt][r] += sum over the tile's 64 rows j: T[j][16 dt + 4g + r] * w[j]  -- i.e. the
// transposed tile (A, by transposed reads) times the lane's per-row weights w (B: element j of
// k step s = w[2s + j / 4][j % 4], the registers of a preceding fx_dots tile (rows
// 16g + 8s + j), split here)
// one k step s of fx_accum: rows 16g + 8s .. +7, weights w0 (rows +0..3), w1 (+4..7)
__device__ __forceinline__ void fx_accum_s(const char* Ts, f4v w0, f4v w1, int s, int lane,
                                           f4v (&o)[4]) {
  const int g = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
  const int rl = 16 * g + 8 * s + qq;
  fx_bf8 b[3];
  fx_split8(w0, w1, b);
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int o0 = fx_off(rl, 16 * dt + 4 * p);
    const int o1 = fx_off(rl + 4, 16 * dt + 4 * p);
    fx_bf8 a[3];
#pragma unroll
    for (int t = 0; t < 3; ++t)
      a[t] = fx_cat(fx_tr(Ts + t * FX_PLANE, o0), fx_tr(Ts + t * FX_PLANE, o1));
    o[dt] = fx_mfma6(a, b, o[dt]);
  }
}
__device__ __forceinline__ void fx_accum(const char* Ts, const f4v (&w)[4], int lane, f4v (&o)[4]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) fx_accum_s(Ts, w[2 * s], w[2 * s + 1], s, lane, o);
}

// ---------------------------------------------------------------------------------- fwd
// grid = B*H*nqt, block = 64*nw (wave w: query strip qt*16nw + 16w). Scores run in base 2
// (attn_common.h ATT_SCALE2): m and every exponent below are log2-scaled, in all four kernels.
__global__ __launch_bounds__(256) void gattn_fwd_flash_kernel(AttnArgs a, float* __restrict__ stats,
                                                             int nqt) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nw = blockDim.x >> 6;
  // XCD-aware: the tiles of a (sample, head) and the heads of a sample share an XCD's L2
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = bid % nqt, bh = bid / nqt;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int i0 = qt * 16 * nw + w * 16;
  float* Ks = sm;
  float* Vs = Ks + FL_KT * ATT_KLD;
  float* Pw = Vs + FL_KT * ATT_KLD + w * FL_KT * FL_WLD;
  const StripViews<AttnArgs> sv(a, b, h);

  f4v qa[4];
  fl_load_strip(sv.q, i0 + col, g, qa);
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
    float kf[4], gv[4][4];
    fl_graph_tile(sv.g, sv.kf, a.Tk, i0, k0, g, col, kf, gv);
    fl_stage2(sv.k, sv.v, k0, a.Tk, Ks, Vs);
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
        if (j < a.Tk) v = kf[jt] == 0.f ? ATT_MASKED : s[jt][r] * ATT_SCALE2;
        x[jt] = v;
        mx = fmaxf(mx, v);
      }
      mx = row16_max(mx);
      const float mn = fmaxf(m[r], mx);  // finite: every tile holds a key < Tk
      const float alpha = att_exp2(m[r] - mn);
      float zs = 0.f, ws = 0.f;
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        const int j = k0 + jt * 16 + col;
        const float e = j < a.Tk ? att_exp2(x[jt] - mn) : 0.f;
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
  const int64_t qb = (int64_t)b * a.Tq;
  const BView O = head_view(a.o, a.ldo, (int64_t)a.B * a.Tq, qb, h * ATT_DK);
  const uint32_t ovo = (uint32_t)(i0 + 4 * g) * O.ld + 4u * col;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    if (i < a.Tq) {
      const float D = fmaxf(W[r], 1e-12f * Z[r]);
      const float sc = bld1(sv.qf, 4u * (i0 + 4 * g), 4u * r) / D;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) bst32(O, o[dt][r] * sc, ovo, r * O.ld + 64u * dt);
      if (col == 0) {
        float* st = stats + (((int64_t)b * a.H + h) * a.Tq + i) * 4;
        st[0] = m[r];
        st[1] = Z[r];
        st[2] = W[r];
      }
    }
  }
}

// x6 form of the forward (see "x6 products" above): lane (col, g) of wave w owns query
// i0 + col; its registers hold the tile's keys 16g + 4jt + r, so the row statistics
// reduce over 16 registers and the 4 lane groups, and O^T[d][q] accumulates in o[dt][r]
// (d = 16 dt + 4g + r).
template <bool PL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void gattn_fwd_flash_x6_kernel(
    AttnArgs a, float* __restrict__ stats, int nqt, FxPlanes pl) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nw = blockDim.x >> 6;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = bid % nqt, bh = bid / nqt;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int i0 = qt * 16 * nw + w * 16;
  char* Ks = reinterpret_cast<char*>(sm);
  char* Vs = Ks + FX_TILE;
  const StripViews<AttnArgs> sv(a, b, h);

  fx_bf8 qp[2][3];
  if constexpr (PL) fx_strip_planes(fx_tiles(pl.q, b, a.H, h, pl.ntq), i0 + col, g, qp);
  else fx_load_strip(sv.q, i0 + col, g, qp);
  float m = -INFINITY, Z = 0.f, W = 0.f;
  f4v o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f4v{0.f, 0.f, 0.f, 0.f};
  const uint32_t gvo = (uint32_t)((i0 + col) * a.Tk + 16 * g) * 4u;
  const int nkt = (a.Tk + FL_KT - 1) / FL_KT;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * FL_KT;
    __syncthreads();  // every wave is done with the previous tile
    f4v gv[4];
    uint32_t kmask = 0;  // bit 4 jt + r: key masked (kflag 0)
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const uint32_t so = (uint32_t)(k0 + 4 * jt) * 4u;
      const f4v kf = bld16b<f4v>(sv.kf, 64u * g, so);
      gv[jt] = bld16b<f4v>(sv.g, gvo, so);
#pragma unroll
      for (int r = 0; r < 4; ++r) kmask |= (kf[r] == 0.f ? 1u : 0u) << (4 * jt + r);
    }
    if constexpr (PL)
      fx_stage_dma(fx_tiles(pl.k, b, a.H, h, pl.ntk) + (int64_t)kt * FX_TILE,
                   fx_tiles(pl.v, b, a.H, h, pl.ntk) + (int64_t)kt * FX_TILE, Ks, Vs, w, nw, lane);
    else
      fx_stage2(sv.k, sv.v, k0, a.Tk, Ks, Vs);
    __syncthreads();
    f4v s[4];
    fx_dots<4>(Ks, qp, col, g, s);
    float mx = -INFINITY;
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = k0 + 16 * g + 4 * jt + r;
        float v = -INFINITY;
        if (j < a.Tk) v = (kmask >> (4 * jt + r)) & 1u ? ATT_MASKED : s[jt][r] * ATT_SCALE2;
        s[jt][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mn = fmaxf(m, mx);  // finite: every tile holds a key < Tk
    const float alpha = att_exp2(m - mn);
    float zs = 0.f, ws = 0.f;
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = k0 + 16 * g + 4 * jt + r;
        const float e = j < a.Tk ? att_exp2(s[jt][r] - mn) : 0.f;
        const float gg = j < a.Tk ? gv[jt][r] : 0.f;
        zs += e;
        ws += e * fabsf(gg);
        s[jt][r] = e * gg;
      }
    zs += __shfl_xor(zs, 16);
    zs += __shfl_xor(zs, 32);
    ws += __shfl_xor(ws, 16);
    ws += __shfl_xor(ws, 32);
    Z = Z * alpha + zs;
    W = W * alpha + ws;
    m = mn;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
    fx_accum(Vs, s, lane, o);
  }
  const int i = i0 + col;
  if (i < a.Tq) {
    const int64_t qb = (int64_t)b * a.Tq;
    const BView O = head_view(a.o, a.ldo, (int64_t)a.B * a.Tq, qb, h * ATT_DK);
    const float D = fmaxf(W, 1e-12f * Z);
    const float sc = bld1(sv.qf, 4u * i, 0u) / D;
    const uint32_t ovo = (uint32_t)i * O.ld + 16u * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) bst16b(O, o[dt] * sc, ovo, 64u * dt);
    if (g == 0) {
      float* st = stats + (((int64_t)b * a.H + h) * a.Tq + i) * 4;
      st[0] = m;
      st[1] = Z;
      st[2] = W;
    }
  }
}

// The forward over pre-split tiles with the K / V DMAs pipelined behind compute: K(t+1) is
// fetched while P V reads V(t), V(t+1) while the next tile's scores read K(t+1) and its
// softmax runs (two barriers per tile, as the unpipelined form, and the same 48 KB of LDS).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void gattn_fwd_flash_x6pp_kernel(
    AttnArgs a, float* __restrict__ stats, int nqt, FxPlanes pl) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nw = blockDim.x >> 6;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = bid % nqt, bh = bid / nqt;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int i0 = qt * 16 * nw + w * 16;
  char* Ks = reinterpret_cast<char*>(sm);
  char* Vs = Ks + FX_TILE;
  const StripViews<AttnArgs> sv(a, b, h);
  const char* ktl = fx_tiles(pl.k, b, a.H, h, pl.ntk);
  const char* vtl = fx_tiles(pl.v, b, a.H, h, pl.ntk);

  fx_dma_tile(ktl, Ks, w, nw, lane);
  fx_dma_tile(vtl, Vs, w, nw, lane);
  fx_bf8 qp[2][3];
  fx_strip_planes(fx_tiles(pl.q, b, a.H, h, pl.ntq), i0 + col, g, qp);
  float m = -INFINITY, Z = 0.f, W = 0.f;
  f4v o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f4v{0.f, 0.f, 0.f, 0.f};
  const uint32_t gvo = (uint32_t)((i0 + col) * a.Tk + 16 * g) * 4u;
  const int nkt = (a.Tk + FL_KT - 1) / FL_KT;
  fx_wait_vm0();
  __syncthreads();  // K(0), V(0) staged
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * FL_KT;
    f4v gv[4], kf[4];  // consumed only after the scores: their wait (which also covers
                       // the V DMAs issued before them) sits behind the score MFMAs
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const uint32_t so = (uint32_t)(k0 + 4 * jt) * 4u;
      kf[jt] = bld16b<f4v>(sv.kf, 64u * g, so);
      gv[jt] = bld16b<f4v>(sv.g, gvo, so);
    }
    __builtin_amdgcn_sched_barrier(0);  // ... issued ahead of the score MFMAs
    f4v s[4];
    fx_dots<4>(Ks, qp, col, g, s);
    __builtin_amdgcn_sched_barrier(0);  // the flags' first use (and its wait) stays behind
    uint32_t kmask = 0;
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) kmask |= (kf[jt][r] == 0.f ? 1u : 0u) << (4 * jt + r);
    float mx = -INFINITY;
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = k0 + 16 * g + 4 * jt + r;
        float v = -INFINITY;
        if (j < a.Tk) v = (kmask >> (4 * jt + r)) & 1u ? ATT_MASKED : s[jt][r] * ATT_SCALE2;
        s[jt][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mn = fmaxf(m, mx);
    const float alpha = att_exp2(m - mn);
    float zs = 0.f, ws = 0.f;
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = k0 + 16 * g + 4 * jt + r;
        const float e = j < a.Tk ? att_exp2(s[jt][r] - mn) : 0.f;
        const float gg = j < a.Tk ? gv[jt][r] : 0.f;
        zs += e;
        ws += e * fabsf(gg);
        s[jt][r] = e * gg;
      }
    zs += __shfl_xor(zs, 16);
    zs += __shfl_xor(zs, 32);
    ws += __shfl_xor(ws, 16);
    ws += __shfl_xor(ws, 32);
    Z = Z * alpha + zs;
    W = W * alpha + ws;
    m = mn;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
    fx_wait_vm0();    // this wave's V(kt) DMAs (issued last tile) have landed
    __syncthreads();  // every wave: done with K(kt), V(kt) staged
    if (kt + 1 < nkt) fx_dma_tile(ktl + (int64_t)(kt + 1) * FX_TILE, Ks, w, nw, lane);
    fx_accum(Vs, s, lane, o);
    fx_wait_vm0();    // this wave's K(kt + 1) DMAs have landed
    __syncthreads();  // every wave: done with V(kt), K(kt + 1) staged
    if (kt + 1 < nkt) fx_dma_tile(vtl + (int64_t)(kt + 1) * FX_TILE, Vs, w, nw, lane);
  }
  const int i = i0 + col;
  if (i < a.Tq) {
    const int64_t qb = (int64_t)b * a.Tq;
    const BView O = head_view(a.o, a.ldo, (int64_t)a.B * a.Tq, qb, h * ATT_DK);
    const float D = fmaxf(W, 1e-12f * Z);
    const float sc = bld1(sv.qf, 4u * i, 0u) / D;
    const uint32_t ovo = (uint32_t)i * O.ld + 16u * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) bst16b(O, o[dt] * sc, ovo, 64u * dt);
    if (g == 0) {
      float* st = stats + (((int64_t)b * a.H + h) * a.Tq + i) * 4;
      st[0] = m;
      st[1] = Z;
      st[2] = W;
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
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int j0 = kt * 16 * nw + w * 16;
  float* Qs = sm;                                  // [64][KLD]
  float* dOs = Qs + FL_KT * ATT_KLD;               // [64][KLD]
  float* cf = dOs + FL_KT * ATT_KLD;               // [64][8] per-query coefficients
  float* img = cf + FL_KT * 8 + w * FL_KT * FL_WLD;  // [64 queries][16] (keys 4g+r): N, then dS
  const int64_t qb = (int64_t)b * a.Tq, kb = (int64_t)b * a.Tk;
  const float* sth = stats + ((int64_t)b * a.H + h) * a.Tq * 4;
  const StripViews<AttnArgs> sv(a, b, h);
  const BView DO = head_view(a.dout, a.lddo, (int64_t)a.B * a.Tq, qb, h * ATT_DK);

  f4v ka[4], va[4];
  fl_load_strip(sv.k, j0 + col, g, ka);
  fl_load_strip(sv.v, j0 + col, g, va);
  float kf[4];
  bool kval[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    kval[r] = j0 + 4 * g + r < a.Tk;
    kf[r] = bld1(sv.kf, 4u * (j0 + 4 * g), 4u * r);
  }
  f4v dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = f4v{0.f, 0.f, 0.f, 0.f};
  const uint32_t gvo = (uint32_t)(col * a.Tk + j0 + 4 * g) * 4u;
  const int nqt = (a.Tq + FL_KT - 1) / FL_KT;
  for (int qt = 0; qt < nqt; ++qt) {
    const int iq0 = qt * FL_KT;
    __syncthreads();
    float gv[4][4];  // [jt][r]: G[query iq0 + 16jt + col][key j0 + 4g + r]
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) gv[jt][r] = bld1(sv.g, gvo, (uint32_t)((iq0 + 16 * jt) * a.Tk + r) * 4u);
    fl_stage2(sv.q, DO, iq0, a.Tq, Qs, dOs);
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
        const float x = kf[r] == 0.f ? ATT_MASKED : s[jt][r] * ATT_SCALE2;
        const float e = kval[r] ? att_exp2(x - c0.x) : 0.f;
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
  const int64_t nk = (int64_t)a.B * a.Tk;
  const BView DK = head_view(a.dk, a.lddk, nk, kb, h * ATT_DK);
  const BView DV = head_view(a.dv, a.lddv, nk, kb, h * ATT_DK);
  const uint32_t kvo = (uint32_t)(j0 + 4 * g) * sv.k.ld + 4u * col;
  const uint32_t vvo = (uint32_t)(j0 + 4 * g) * sv.v.ld + 4u * col;
  const uint32_t dkvo = (uint32_t)(j0 + 4 * g) * DK.ld + 4u * col;
  const uint32_t dvvo = (uint32_t)(j0 + 4 * g) * DV.ld + 4u * col;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (j0 + 4 * g + r < a.Tk) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const float kx = bld1(sv.k, kvo, r * sv.k.ld + 64u * dt);
        const float vx = bld1(sv.v, vvo, r * sv.v.ld + 64u * dt);
        bst32(DK, kx > 0.f ? dk[dt][r] * 0.125f : 0.f, dkvo, r * DK.ld + 64u * dt);
        bst32(DV, vx > 0.f ? dv[dt][r] : 0.f, dvvo, r * DV.ld + 64u * dt);
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
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SAVQA_FL_DELTA_WPE))) void gattn_bwd_delta_flash_kernel(AttnArgs a,
                                                                   float* __restrict__ stats,
                                                                   int nqt) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nw = blockDim.x >> 6;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = bid % nqt, bh = bid / nqt;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int i0 = qt * 16 * nw + w * 16;
  float* Ks = sm;
  float* Vs = Ks + FL_KT * ATT_KLD;
  const int64_t qb = (int64_t)b * a.Tq;
  const int hd = h * ATT_DK;
  const float* sth = stats + ((int64_t)b * a.H + h) * a.Tq * 4;
  const StripViews<AttnArgs> sv(a, b, h);
  const BView DO = head_view(a.dout, a.lddo, (int64_t)a.B * a.Tq, qb, h * ATT_DK);

  f4v qa[4], oa[4];
  fl_load_strip(sv.q, i0 + col, g, qa);
  fl_load_strip(DO, i0 + col, g, oa);
  float rm[4], rq[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    const int ic = min(i, a.Tq - 1);
    const RowCoef c = row_coef(sth + (int64_t)ic * 4, a.qflag[qb + ic], i < a.Tq);
    rm[r] = c.m;
    rq[r] = c.qf;
  }
  double sa[4] = {0., 0., 0., 0.}, sw[4] = {0., 0., 0., 0.}, sz[4] = {0., 0., 0., 0.};
  const int nkt = (a.Tk + FL_KT - 1) / FL_KT;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * FL_KT;
    __syncthreads();
    float kf[4], gv[4][4];
    fl_graph_tile(sv.g, sv.kf, a.Tk, i0, k0, g, col, kf, gv);
    fl_stage2(sv.k, sv.v, k0, a.Tk, Ks, Vs);
    __syncthreads();
    f4v s[4], dp[4];
    strip_dots_lds<4>(qa, Ks, col, g, s);   // [query 4g+r][key 16jt+col]
    strip_dots_lds<4>(oa, Vs, col, g, dp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        const int j = k0 + jt * 16 + col;
        const float x = kf[jt] == 0.f ? ATT_MASKED : s[jt][r] * ATT_SCALE2;
        const float e = j < a.Tk ? att_exp2(x - rm[r]) : 0.f;
        const float gg = j < a.Tk ? gv[r][jt] : 0.f;
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
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int i0 = qt * 16 * nw + w * 16;
  float* Ks = sm;
  float* Vs = Ks + FL_KT * ATT_KLD;
  float* Simg = Vs + FL_KT * ATT_KLD + w * FL_KT * FL_WLD;  // [64 keys][16] (queries 4g+r)
  const int64_t qb = (int64_t)b * a.Tq;
  const int hd = h * ATT_DK;
  const float* sth = stats + ((int64_t)b * a.H + h) * a.Tq * 4;
  const StripViews<AttnArgs> sv(a, b, h);
  const BView DO = head_view(a.dout, a.lddo, (int64_t)a.B * a.Tq, qb, h * ATT_DK);

  f4v qa[4], oa[4];
  fl_load_strip(sv.q, i0 + col, g, qa);
  fl_load_strip(DO, i0 + col, g, oa);
  RowCoef rc[4];
  double dx[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + 4 * g + r;
    const int ic = min(i, a.Tq - 1);
    rc[r] = row_coef(sth + (int64_t)ic * 4, a.qflag[qb + ic], i < a.Tq);
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
    float kf[4], gv[4][4];
    fl_graph_tile(sv.g, sv.kf, a.Tk, i0, k0, g, col, kf, gv);
    fl_stage2(sv.k, sv.v, k0, a.Tk, Ks, Vs);
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
        const float x = kf[jt] == 0.f ? ATT_MASKED : s[jt][r] * ATT_SCALE2;
        const float e = j < a.Tk ? att_exp2(x - c.m) : 0.f;
        const float gg = j < a.Tk ? gv[r][jt] : 0.f;
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

// ---------------------------------------------------------------- x6 backward kernels
// The three backward kernels above with x6 products (see "x6 products"): identical math per
// (query, key) pair; the strips on the lanes (queries for delta / dQ, keys for dK / dV), the
// staged tile's rows in registers.

template <bool PL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void gattn_bwd_delta_flash_x6_kernel(
    AttnArgs a, float* __restrict__ stats, int nqt, FxPlanes pl) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nw = blockDim.x >> 6;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = bid % nqt, bh = bid / nqt;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int i0 = qt * 16 * nw + w * 16;
  char* Ks = reinterpret_cast<char*>(sm);
  char* Vs = Ks + FX_TILE;
  const int64_t qb = (int64_t)b * a.Tq;
  const int hd = h * ATT_DK;
  const float* sth = stats + ((int64_t)b * a.H + h) * a.Tq * 4;
  const StripViews<AttnArgs> sv(a, b, h);
  const BView DO = head_view(a.dout, a.lddo, (int64_t)a.B * a.Tq, qb, h * ATT_DK);

  fx_bf8 qp[2][3], op[2][3];
  if constexpr (PL) {
    fx_strip_planes(fx_tiles(pl.q, b, a.H, h, pl.ntq), i0 + col, g, qp);
    fx_strip_planes(fx_tiles(pl.dout, b, a.H, h, pl.ntq), i0 + col, g, op);
  } else {
    fx_load_strip(sv.q, i0 + col, g, qp);
    fx_load_strip(DO, i0 + col, g, op);
  }
  const int i = i0 + col;
  const int ic = min(i, a.Tq - 1);
  const RowCoef rc = row_coef(sth + (int64_t)ic * 4, a.qflag[qb + ic], i < a.Tq);
  const uint32_t gvo = (uint32_t)(i * a.Tk + 16 * g) * 4u;
  double sa = 0., sw = 0., sz = 0.;
  const int nkt = (a.Tk + FL_KT - 1) / FL_KT;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * FL_KT;
    __syncthreads();
    f4v gv[4];
    uint32_t kmask;
    fx_graph_row(sv.g, sv.kf, gvo, k0, g, gv, kmask);
    if constexpr (PL)
      fx_stage_dma(fx_tiles(pl.k, b, a.H, h, pl.ntk) + (int64_t)kt * FX_TILE,
                   fx_tiles(pl.v, b, a.H, h, pl.ntk) + (int64_t)kt * FX_TILE, Ks, Vs, w, nw, lane);
    else
      fx_stage2(sv.k, sv.v, k0, a.Tk, Ks, Vs);
    __syncthreads();
    f4v s[4], dp[4];
    fx_dots<4>(Ks, qp, col, g, s);   // [key 16g + 4jt + r][query col]
    fx_dots<4>(Vs, op, col, g, dp);
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = k0 + 16 * g + 4 * jt + r;
        const float x = (kmask >> (4 * jt + r)) & 1u ? ATT_MASKED : s[jt][r] * ATT_SCALE2;
        const float e = j < a.Tk ? att_exp2(x - rc.m) : 0.f;
        const float gg = j < a.Tk ? gv[jt][r] : 0.f;
        sa += (double)(e * gg * rc.qf * dp[jt][r]);
        sw += (double)(e * fabsf(gg));
        sz += (double)e;
      }
  }
  double A = sa, Wd = sw, Zd = sz;
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) {
    A += __shfl_xor(A, o);
    Wd += __shfl_xor(Wd, o);
    Zd += __shfl_xor(Zd, o);
  }
  if (i < a.Tq && g == 0) {
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

template <bool PL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SAVQA_FX_WPE_Q))) void gattn_bwd_q_flash_x6_kernel(
    AttnArgs a, const float* __restrict__ stats, int nqt, FxPlanes pl) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nw = blockDim.x >> 6;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = bid % nqt, bh = bid / nqt;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int i0 = qt * 16 * nw + w * 16;
  char* Ks = reinterpret_cast<char*>(sm);
  char* Vs = Ks + FX_TILE;
  const int64_t qb = (int64_t)b * a.Tq;
  const int hd = h * ATT_DK;
  const float* sth = stats + ((int64_t)b * a.H + h) * a.Tq * 4;
  const StripViews<AttnArgs> sv(a, b, h);
  const BView DO = head_view(a.dout, a.lddo, (int64_t)a.B * a.Tq, qb, h * ATT_DK);

  fx_bf8 qp[2][3], op[2][3];
  if constexpr (PL) {
    fx_strip_planes(fx_tiles(pl.q, b, a.H, h, pl.ntq), i0 + col, g, qp);
    fx_strip_planes(fx_tiles(pl.dout, b, a.H, h, pl.ntq), i0 + col, g, op);
  } else {
    fx_load_strip(sv.q, i0 + col, g, qp);
    fx_load_strip(DO, i0 + col, g, op);
  }
  const int i = i0 + col;
  const int ic = min(i, a.Tq - 1);
  const RowCoef c = row_coef(sth + (int64_t)ic * 4, a.qflag[qb + ic], i < a.Tq);
  const float* dxs = a.dq + (qb + ic) * a.lddq + hd;
  const double dx = i < a.Tq ? (double)dxs[0] + (double)dxs[1] : 0.;
  const uint32_t gvo = (uint32_t)(i * a.Tk + 16 * g) * 4u;
  f4v dq[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dq[dt] = f4v{0.f, 0.f, 0.f, 0.f};
  const int nkt = (a.Tk + FL_KT - 1) / FL_KT;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * FL_KT;
    __syncthreads();
    f4v gv[4];
    uint32_t kmask;
    fx_graph_row(sv.g, sv.kf, gvo, k0, g, gv, kmask);
    if constexpr (PL)
      fx_stage_dma(fx_tiles(pl.k, b, a.H, h, pl.ntk) + (int64_t)kt * FX_TILE,
                   fx_tiles(pl.v, b, a.H, h, pl.ntk) + (int64_t)kt * FX_TILE, Ks, Vs, w, nw, lane);
    else
      fx_stage2(sv.k, sv.v, k0, a.Tk, Ks, Vs);
    __syncthreads();
    f4v s[4], dp[4];
    fx_dots<4>(Ks, qp, col, g, s);
    fx_dots<4>(Vs, op, col, g, dp);
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = k0 + 16 * g + 4 * jt + r;
        const bool masked = (kmask >> (4 * jt + r)) & 1u;
        const float x = masked ? ATT_MASKED : s[jt][r] * ATT_SCALE2;
        const float e = j < a.Tk ? att_exp2(x - c.m) : 0.f;
        const float gg = j < a.Tk ? gv[jt][r] : 0.f;
        const float av = e * gg * c.qf * dp[jt][r];
        const float wv = c.normal ? e * fabsf(gg) : e;
        const float ds = (float)((double)av - dx * (double)wv) * c.rD;
        s[jt][r] = (masked || j >= a.Tk) ? 0.f : ds;
      }
    fx_accum(Ks, s, lane, dq);  // dQ_i += sum_j dS_ij K_j   (x 1/8 at the end)
  }
  if (i < a.Tq) {
    const int64_t row = qb + i;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cc = hd + dt * 16 + 4 * g + r;
        a.dq[row * a.lddq + cc] = a.q[row * a.ldq + cc] > 0.f ? dq[dt][r] * 0.125f : 0.f;
      }
  }
}

template <bool PL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PL ? SAVQA_FX_WPE_KVP : SAVQA_FX_WPE_KV))) void gattn_bwd_kv_flash_x6_kernel(
    AttnArgs a, const float* __restrict__ stats, int nkt2, FxPlanes pl) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nw = blockDim.x >> 6;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kt = bid % nkt2, bh = bid / nkt2;
  const int b = bh / a.H, h = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15, g = lane >> 4;
  const int j0 = kt * 16 * nw + w * 16;
  char* Qs = reinterpret_cast<char*>(sm);
  char* dOs = Qs + FX_TILE;
  float* cf = reinterpret_cast<float*>(dOs + FX_TILE);  // [64][8] per-query coefficients
  const int64_t qb = (int64_t)b * a.Tq, kb = (int64_t)b * a.Tk;
  const float* sth = stats + ((int64_t)b * a.H + h) * a.Tq * 4;
  const StripViews<AttnArgs> sv(a, b, h);
  const BView DO = head_view(a.dout, a.lddo, (int64_t)a.B * a.Tq, qb, h * ATT_DK);

  const int j = j0 + col;  // the lane's key
  fx_bf8 kp[2][3], vp[2][3];
  if constexpr (PL) {
    fx_strip_planes(fx_tiles(pl.k, b, a.H, h, pl.ntk), j, g, kp);
    fx_strip_planes(fx_tiles(pl.v, b, a.H, h, pl.ntk), j, g, vp);
  } else {
    fx_load_strip(sv.k, j, g, kp);
    fx_load_strip(sv.v, j, g, vp);
  }
  const bool kval = j < a.Tk;
  const bool kmasked = bld1(sv.kf, 4u * j, 0u) == 0.f;
  f4v dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = f4v{0.f, 0.f, 0.f, 0.f};
  const uint32_t gvo = (uint32_t)(16 * g * a.Tk + j) * 4u;
  const int nqt = (a.Tq + FL_KT - 1) / FL_KT;
  for (int qt = 0; qt < nqt; ++qt) {
    const int iq0 = qt * FL_KT;
    __syncthreads();
    float gv[4][4];  // G[query iq0 + 16g + 4jt + r][key j]
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        gv[jt][r] = bld1(sv.g, gvo, (uint32_t)((iq0 + 4 * jt + r) * a.Tk) * 4u);
    if constexpr (PL)
      fx_stage_dma(fx_tiles(pl.q, b, a.H, h, pl.ntq) + (int64_t)qt * FX_TILE,
                   fx_tiles(pl.dout, b, a.H, h, pl.ntq) + (int64_t)qt * FX_TILE, Qs, dOs, w, nw,
                   lane);
    else
      fx_stage2(sv.q, DO, iq0, a.Tq, Qs, dOs);
    if (threadIdx.x < FL_KT) {
      const int iq = iq0 + threadIdx.x;
      const bool valid = iq < a.Tq;
      const int icl = min(iq, a.Tq - 1);
      RowCoef c = row_coef(sth + (int64_t)icl * 4, a.qflag[qb + icl], valid);
      if (valid) coef_delta(c, sth[(int64_t)icl * 4 + 3]);
      float* cp = cf + threadIdx.x * 8;
      cp[0] = c.m;
      cp[1] = c.rD;
      cp[2] = c.qf;
      cp[3] = c.cd;
      cp[4] = c.pd;
    }
    __syncthreads();
    f4v s[4], dp[4];
    fx_dots<4>(Qs, kp, col, g, s);    // [query 16g + 4jt + r][key col]
    fx_dots<4>(dOs, vp, col, g, dp);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {  // queries 16g + 8 s2 .. +7: one k step of both products
      f4v nv[2], dsv[2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int jt = 2 * s2 + jj;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float* cp = cf + (16 * g + 4 * jt + r) * 8;
          const f4v c0 = ld4(cp);
          const float pd = cp[4];
          const float x = kmasked ? ATT_MASKED : s[jt][r] * ATT_SCALE2;
          const float e = kval ? att_exp2(x - c0.x) : 0.f;
          const float gg = gv[jt][r];
          const float n = e * gg * c0.y;
          nv[jj][r] = n * c0.z;
          const float ds = n * c0.z * dp[jt][r] - c0.w * e * fabsf(gg) - pd * e;
          dsv[jj][r] = kmasked ? 0.f : ds;
        }
      }
      fx_accum_s(dOs, nv[0], nv[1], s2, lane, dv);  // dV_j += sum_i nq_ij dO_i
      fx_accum_s(Qs, dsv[0], dsv[1], s2, lane, dk);  // dK_j += sum_i dS_ij Q_i   (x 1/8 at the end)
    }
  }
  if (kval) {
    const int64_t nk = (int64_t)a.B * a.Tk;
    const BView DK = head_view(a.dk, a.lddk, nk, kb, h * ATT_DK);
    const BView DV = head_view(a.dv, a.lddv, nk, kb, h * ATT_DK);
    const uint32_t kvo = (uint32_t)j * sv.k.ld + 16u * g;
    const uint32_t vvo = (uint32_t)j * sv.v.ld + 16u * g;
    const uint32_t dkvo = (uint32_t)j * DK.ld + 16u * g;
    const uint32_t dvvo = (uint32_t)j * DV.ld + 16u * g;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f4v kx = bld16b<f4v>(sv.k, kvo, 64u * dt);
      const f4v vx = bld16b<f4v>(sv.v, vvo, 64u * dt);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bst32(DK, kx[r] > 0.f ? dk[dt][r] * 0.125f : 0.f, dkvo, 64u * dt + 4u * r);
        bst32(DV, vx[r] > 0.f ? dv[dt][r] : 0.f, dvvo, 64u * dt + 4u * r);
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

// the x6 kernels (SAVQA_FLASH_X6 at build time; SAVQA_FLASH_X6=0 in the environment selects
// the fp32-MFMA kernels at run time, for A/B runs)
static bool flash_x6() {
  if (!SAVQA_FLASH_X6) return false;
  const char* e = getenv("SAVQA_FLASH_X6");
  return !(e && e[0] == '0');
}

}  // namespace savqa

using namespace savqa;

namespace savqa {
// One (sample, head, 64-row tile) of X per workgroup, split into FX_TILE bytes of bf16 planes
// (fx_stage2's image, rows past T zero).
__global__ __launch_bounds__(256) void attn_planes_kernel(const float* __restrict__ X, int64_t ldx,
                                                          int T, int H, int nt, char* __restrict__ out) {
  const int blk = blockIdx.x, t = blk % nt, bh = blk / nt;
  const int b = bh / H, h = bh % H;
  char* img = out + (int64_t)blk * FX_TILE;
  const float* base = X + ((int64_t)b * T + (int64_t)t * FL_KT) * ldx + h * ATT_DK;
  const int d4 = 4 * (threadIdx.x & 15);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int row = (threadIdx.x >> 4) + 16 * u;
    f4v v = {0.f, 0.f, 0.f, 0.f};
    if (t * FL_KT + row < T) v = *reinterpret_cast<const f4v*>(base + (int64_t)row * ldx + d4);
    fx_bf4 a0, a1, a2;
    fx_split4(v, a0, a1, a2);
    const int off = fx_off(row, d4);
    *reinterpret_cast<fx_bf4*>(img + off) = a0;
    *reinterpret_cast<fx_bf4*>(img + FX_PLANE + off) = a1;
    *reinterpret_cast<fx_bf4*>(img + 2 * FX_PLANE + off) = a2;
  }
}

static int64_t planes_bytes(int64_t B, int64_t T, int64_t H) {
  return B * H * ((T + FL_KT - 1) / FL_KT) * (int64_t)FX_TILE;
}

static int make_planes(hipStream_t s, const float* X, int64_t ldx, int64_t B, int64_t T,
                       int64_t H, char* out) {
  const int nt = (int)((T + FL_KT - 1) / FL_KT);
  hipLaunchKernelGGL(attn_planes_kernel, dim3((unsigned)(B * H * nt)), dim3(256), 0, s, X, ldx,
                     (int)T, (int)H, nt, out);
  return check_launch("savqa_gattn_flash(planes)");
}

// Carve the workspace into Q / K / V (/ dO) plane tiles and fill them; false: no workspace
static int flash_planes(hipStream_t s, const AttnArgs& a, bool bwd, void* ws, int64_t ws_bytes,
                        FxPlanes& pl, bool& on, const char* who) {
  on = false;
  if (!ws) return 0;
  const int64_t nq = planes_bytes(a.B, a.Tq, a.H), nk = planes_bytes(a.B, a.Tk, a.H);
  if (((uintptr_t)ws & 15) || ws_bytes < nq + 2 * nk + (bwd ? nq : 0))
    return fail(SAVQA_EINVAL, std::string(who) + ": workspace smaller than "
                              "savqa_gattn_flash_ws_bytes or not 16-B aligned");
  char* w = static_cast<char*>(ws);
  pl.q = w;
  pl.k = w + nq;
  pl.v = w + nq + nk;
  pl.dout = bwd ? w + nq + 2 * nk : nullptr;
  pl.ntq = (a.Tq + FL_KT - 1) / FL_KT;
  pl.ntk = (a.Tk + FL_KT - 1) / FL_KT;
  if (int rc = make_planes(s, a.q, a.ldq, a.B, a.Tq, a.H, w)) return rc;
  if (int rc = make_planes(s, a.k, a.ldk, a.B, a.Tk, a.H, w + nq)) return rc;
  if (int rc = make_planes(s, a.v, a.ldv, a.B, a.Tk, a.H, w + nq + nk)) return rc;
  if (bwd)
    if (int rc = make_planes(s, a.dout, a.lddo, a.B, a.Tq, a.H, w + nq + 2 * nk)) return rc;
  on = true;
  return 0;
}

static int flash_fwd(hipStream_t s, AttnArgs& a, int64_t dk, float* stats, void* ws,
                     int64_t ws_bytes) {
  if (int rc = flash_validate(a, dk, "savqa_gattn_fwd_flash")) return rc;
  if (!stats) return fail(SAVQA_EINVAL, "savqa_gattn_fwd_flash: stats buffer required");
  const int nw = waves_for(a.Tq);
  const int nqt = (a.Tq + 16 * nw - 1) / (16 * nw);
  const dim3 grid((unsigned)((int64_t)a.B * a.H * nqt)), block(64 * nw);
  if (flash_x6()) {
    FxPlanes pl{};
    bool on;
    if (int rc = flash_planes(s, a, false, ws, ws_bytes, pl, on, "savqa_gattn_fwd_flash"))
      return rc;
    const char* pe = getenv("SAVQA_FX_PIPE");
    if (on && !(pe && pe[0] == '0'))
      hipLaunchKernelGGL(gattn_fwd_flash_x6pp_kernel, grid, block, (size_t)2 * FX_TILE, s, a,
                         stats, nqt, pl);
    else if (on)
      hipLaunchKernelGGL(gattn_fwd_flash_x6_kernel<true>, grid, block, (size_t)2 * FX_TILE, s, a,
                         stats, nqt, pl);
    else
      hipLaunchKernelGGL(gattn_fwd_flash_x6_kernel<false>, grid, block, (size_t)2 * FX_TILE, s, a,
                         stats, nqt, pl);
    return check_launch("savqa_gattn_fwd_flash");
  }
  const size_t lds = sizeof(float) * ((size_t)2 * FL_KT * ATT_KLD + (size_t)nw * FL_KT * FL_WLD);
  hipLaunchKernelGGL(gattn_fwd_flash_kernel, grid, block, lds, s, a, stats, nqt);
  return check_launch("savqa_gattn_fwd_flash");
}

static int flash_bwd(hipStream_t s, AttnArgs& a, int64_t dk, float* stats, void* ws,
                     int64_t ws_bytes) {
  if (int rc = flash_validate(a, dk, "savqa_gattn_bwd_flash")) return rc;
  if (!stats) return fail(SAVQA_EINVAL, "savqa_gattn_bwd_flash: stats required");
  if ((((uintptr_t)a.dout) & 15) || (a.lddo & 3))
    return fail(SAVQA_EINVAL, "savqa_gattn_bwd_flash: dO must be 16-B aligned, ld % 4 == 0");
  const int nw = waves_for(a.Tq);
  const int nqt = (a.Tq + 16 * nw - 1) / (16 * nw);
  const int nwk = waves_for(a.Tk);
  const int nkt2 = (a.Tk + 16 * nwk - 1) / (16 * nwk);
  const dim3 gq((unsigned)((int64_t)a.B * a.H * nqt)), bq(64 * nw);
  const dim3 gk((unsigned)((int64_t)a.B * a.H * nkt2)), bk(64 * nwk);
  if (flash_x6()) {
    FxPlanes pl{};
    bool on;
    if (int rc = flash_planes(s, a, true, ws, ws_bytes, pl, on, "savqa_gattn_bwd_flash"))
      return rc;
    const size_t lq = (size_t)2 * FX_TILE, lk = lq + sizeof(float) * FL_KT * 8;
    // delta (stats[..][3]) for the dK/dV pass and dx for the dQ pass, then dQ, then dK / dV
    if (on) {
      hipLaunchKernelGGL(gattn_bwd_delta_flash_x6_kernel<true>, gq, bq, lq, s, a, stats, nqt, pl);
      if (int rc = check_launch("savqa_gattn_bwd_flash(delta)")) return rc;
      hipLaunchKernelGGL(gattn_bwd_q_flash_x6_kernel<true>, gq, bq, lq, s, a, stats, nqt, pl);
      if (int rc = check_launch("savqa_gattn_bwd_flash(dq)")) return rc;
      hipLaunchKernelGGL(gattn_bwd_kv_flash_x6_kernel<true>, gk, bk, lk, s, a, stats, nkt2, pl);
    } else {
      hipLaunchKernelGGL(gattn_bwd_delta_flash_x6_kernel<false>, gq, bq, lq, s, a, stats, nqt, pl);
      if (int rc = check_launch("savqa_gattn_bwd_flash(delta)")) return rc;
      hipLaunchKernelGGL(gattn_bwd_q_flash_x6_kernel<false>, gq, bq, lq, s, a, stats, nqt, pl);
      if (int rc = check_launch("savqa_gattn_bwd_flash(dq)")) return rc;
      hipLaunchKernelGGL(gattn_bwd_kv_flash_x6_kernel<false>, gk, bk, lk, s, a, stats, nkt2, pl);
    }
    return check_launch("savqa_gattn_bwd_flash(dkv)");
  }
  hipLaunchKernelGGL(gattn_bwd_delta_flash_kernel, gq, bq,
                     sizeof(float) * (size_t)2 * FL_KT * ATT_KLD, s, a, stats, nqt);
  if (int rc = check_launch("savqa_gattn_bwd_flash(delta)")) return rc;
  const size_t lds = sizeof(float) * ((size_t)2 * FL_KT * ATT_KLD + (size_t)nw * FL_KT * FL_WLD);
  hipLaunchKernelGGL(gattn_bwd_q_flash_kernel, gq, bq, lds, s, a, stats, nqt);
  if (int rc = check_launch("savqa_gattn_bwd_flash(dq)")) return rc;
  const size_t ldk = sizeof(float) * ((size_t)2 * FL_KT * ATT_KLD + FL_KT * 8 +
                                      (size_t)nwk * FL_KT * FL_WLD);
  hipLaunchKernelGGL(gattn_bwd_kv_flash_kernel, gk, bk, ldk, s, a, stats, nkt2);
  return check_launch("savqa_gattn_bwd_flash(dkv)");
}
}  // namespace savqa

static AttnArgs flash_args(const float* q, int64_t ldq, const float* k, int64_t ldk,
                           const float* v, int64_t ldv, const float* G, const float* kflag,
                           const float* qflag, int64_t B, int64_t Tq, int64_t Tk, int64_t H) {
  AttnArgs a{};
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv; a.G = G;
  a.kflag = kflag; a.qflag = qflag; a.B = (int)B; a.Tq = (int)Tq; a.Tk = (int)Tk; a.H = (int)H;
  return a;
}

extern "C" int64_t savqa_gattn_flash_ws_bytes(int64_t B, int64_t Tq, int64_t Tk, int64_t H,
                                              int32_t backward) {
  if (B <= 0 || Tq <= 0 || Tk <= 0 || H <= 0) return 0;
  return (backward ? 2 : 1) * planes_bytes(B, Tq, H) + 2 * planes_bytes(B, Tk, H);
}

extern "C" int savqa_gattn_fwd_flash_ws(void* stream, const float* q, int64_t ldq, const float* k,
                                        int64_t ldk, const float* v, int64_t ldv, const float* G,
                                        const float* kflag, const float* qflag, int64_t B,
                                        int64_t Tq, int64_t Tk, int64_t H, int64_t dk, float* o,
                                        int64_t ldo, float* stats, void* ws, int64_t ws_bytes) {
  AttnArgs a = flash_args(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H);
  a.o = o; a.ldo = ldo;
  return flash_fwd(as_stream(stream), a, dk, stats, ws, ws_bytes);
}

extern "C" int savqa_gattn_fwd_flash(void* stream, const float* q, int64_t ldq, const float* k,
                                     int64_t ldk, const float* v, int64_t ldv, const float* G,
                                     const float* kflag, const float* qflag, int64_t B,
                                     int64_t Tq, int64_t Tk, int64_t H, int64_t dk, float* o,
                                     int64_t ldo, float* stats) {
  return savqa_gattn_fwd_flash_ws(stream, q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H,
                                  dk, o, ldo, stats, nullptr, 0);
}

extern "C" int savqa_gattn_bwd_flash_ws(void* stream, const float* q, int64_t ldq, const float* k,
                                        int64_t ldk, const float* v, int64_t ldv, const float* G,
                                        const float* kflag, const float* qflag, int64_t B,
                                        int64_t Tq, int64_t Tk, int64_t H, int64_t dk,
                                        const float* dout, int64_t lddo, float* stats, float* dq,
                                        int64_t lddq, float* dk_, int64_t lddk, float* dv,
                                        int64_t lddv, void* ws, int64_t ws_bytes) {
  AttnArgs a = flash_args(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H);
  a.dout = dout; a.lddo = lddo; a.dq = dq; a.lddq = lddq; a.dk = dk_; a.lddk = lddk;
  a.dv = dv; a.lddv = lddv;
  return flash_bwd(as_stream(stream), a, dk, stats, ws, ws_bytes);
}

extern "C" int savqa_gattn_bwd_flash(void* stream, const float* q, int64_t ldq, const float* k,
                                     int64_t ldk, const float* v, int64_t ldv, const float* G,
                                     const float* kflag, const float* qflag, int64_t B,
                                     int64_t Tq, int64_t Tk, int64_t H, int64_t dk,
                                     const float* dout, int64_t lddo, float* stats,
                                     float* dq, int64_t lddq, float* dk_, int64_t lddk, float* dv,
                                     int64_t lddv) {
  return savqa_gattn_bwd_flash_ws(stream, q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H,
                                  dk, dout, lddo, stats, dq, lddq, dk_, lddk, dv, lddv, nullptr, 0);
}
