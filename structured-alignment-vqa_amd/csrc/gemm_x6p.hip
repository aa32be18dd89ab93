// fp32 GEMM on the bf16 matrix cores from PRE-SPLIT operands (savqa_gemm_desc.prec = 6 with
// plane operands: desc.ap / desc.bp). Same operator, epilogue, launch plan (split-K, tail split,
// slabs) and accuracy as gemm_x6_kernel (gemm_x6.hip): each fp32 operand value is the exact sum
// of three bf16 terms, a = a0 + a1 + a2, and a*b is the sum of the six products of order <= 2,
// summed per k-tile into a zero-started partial that is added to the accumulator once per
// k-tile (two-level accumulation). The difference is where the split happens: savqa_split3
// writes the three bf16 PLANES of an operand to memory once (or a producer's epilogue does),
// and this kernel streams the planes into LDS by LDS-DMA -- no register staging, no split VALU
// in the k-loop, so the loop is MFMAs, fragment reads and one DMA batch per k-tile.
//
// Tile: 256 threads = 4 waves (2x2, one per SIMD), 128x128 outputs, k-tile 32; each wave
// 64x64 = 4x4 fragments of 16x16 (v_mfma_f32_16x16x32_bf16). One workgroup per CU (a 144 KB
// three-slot LDS ring: each slot holds 3 A planes + 3 B planes of one k-tile, 8 KB each), so
// the DMAs of k-tiles t+1 and t+2 are in flight while t is computed, with one counted
// `s_waitcnt vmcnt` + barrier per k-tile. Plane images keep the operand's global orientation:
//   R image (k contiguous: A of NT / NN, B of NT): [128 rows][32 k] bf16, 64-B rows, 16-B chunk
//     c of row r at c ^ ((r ^ (r >> 1)) & 3) -- fragments are conflict-free ds_read_b128;
//   T image (m / n contiguous: B of NN, A and B of TN): [32 k rows][128 cols] bf16, 256-B rows,
//     byte b of row r at b ^ 32 h(r) -- fragments are two ds_read_b64_tr_b16.
// LDS-DMA writes lane-linear 16-B granules, so the swizzle is applied to each lane's source.
#include "gemm_common.h"

#include <type_traits>

namespace savqa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int XP_TILE = 128;
constexpr int XP_BK = 32;                   // k per k-tile (one 16x16x32 MFMA per product)
constexpr int XP_PLANE = XP_TILE * XP_BK * 2;  // bytes of one plane image (8 KB)
constexpr int XP_STAGE = 6 * XP_PLANE;      // A planes 0-2, B planes 0-2 (48 KB)
constexpr int XP_NS = 3;                    // ring slots (144 KB)
#ifndef SAVQA_X6P_WAVES
#define SAVQA_X6P_WAVES 8
#endif
constexpr int XP_W = SAVQA_X6P_WAVES;       // waves per workgroup (4: 2x2 of 64x64, 8: 2x4 of 64x32)
constexpr int XP_NT = 64 * XP_W;
constexpr int XP_U = 8 / XP_W;              // DMA instructions per wave per plane
constexpr int XP_PER = 6 * XP_U;            // LDS-DMA instructions per wave per k-tile
constexpr int XP_WN = XP_W / 2;             // waves along n
constexpr int XP_TN = 128 / XP_WN;          // wave tile columns
constexpr int XP_FN = XP_TN / 16;           // fragments along n

__device__ __attribute__((aligned(16))) uint4 g_xp_zero[1];

__device__ __forceinline__ int xp_rswz(int r) { return (r ^ (r >> 1)) & 3; }
__device__ __forceinline__ int xp_th(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

// LDS-DMA sources of one operand's three planes: wave w issues instructions 2w, 2w+1 of each
// plane image (8 x 1 KB).
//   R: instruction s covers rows 16s .. 16s+15; lane L -> row 16s + L/4, physical chunk L%4,
//      logical chunk (L%4) ^ rswz(row). Rows past lim re-read row lim-1 (never stored).
//   T: instruction s covers k rows 4s .. 4s+3; lane L -> k row 4s + L/16, physical chunk L%16,
//      logical chunk (L%16) ^ 2h(row). Columns past lim8 re-read the last 8 (never stored).
template <bool T>
struct XpStage {
  const char* p[XP_U];
  int koff[XP_U];       // k of this lane's granule within a k-tile
  int64_t step;      // bytes per k-tile
  int64_t pstride;   // bytes between planes

  __device__ __forceinline__ void setup(const void* base, int64_t ld, int64_t ps,
                                        const int64_t* __restrict__ rows, int64_t r0, int64_t lim,
                                        int64_t kbeg, int wave, int lane) {
    const char* b = static_cast<const char*>(base);
#pragma unroll
    for (int u = 0; u < XP_U; ++u) {
      const int s = XP_U * wave + u;
      if constexpr (!T) {
        const int r = 16 * s + (lane >> 2);
        const int lc = (lane & 3) ^ xp_rswz(r);
        int64_t m = r0 + r;
        m = m < lim ? m : lim - 1;
        const int64_t rr = rows ? rows[m] : m;
        p[u] = b + (rr * ld + kbeg + lc * 8) * 2;
        koff[u] = lc * 8;
      } else {
        const int r = 4 * s + (lane >> 4);
        const int lc = (lane & 15) ^ (2 * xp_th(r));
        const int64_t lim8 = (lim + 7) & ~(int64_t)7;
        int64_t c = r0 + lc * 8;
        c = c + 8 <= lim8 ? c : lim8 - 8;
        p[u] = b + ((kbeg + r) * ld + c) * 2;
        koff[u] = r;
      }
    }
    step = T ? (int64_t)XP_BK * ld * 2 : XP_BK * 2;
    pstride = ps * 2;
  }

  // k-tile t into the three plane images at img (branch-free: every full k-tile)
  __device__ __forceinline__ void issue(char* img, int wave, int64_t t) const {
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int u = 0; u < XP_U; ++u)
        __builtin_amdgcn_global_load_lds(
            p[u] + q * pstride + t * step,
            (lds_void*)(img + q * XP_PLANE + (XP_U * wave + u) * 1024), 16, 0, 0);
  }

  // the partial last k-tile: granules at k >= krem load zeros
  __device__ __forceinline__ void issue_tail(char* img, int wave, int64_t t, int krem) const {
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int u = 0; u < XP_U; ++u)
        __builtin_amdgcn_global_load_lds(
            koff[u] < krem ? (const void*)(p[u] + q * pstride + t * step) : (const void*)g_xp_zero,
            (lds_void*)(img + q * XP_PLANE + (XP_U * wave + u) * 1024), 16, 0, 0);
  }
};

// fragment: 16 rows (R image) / 16 columns (T image) from base, k 8g .. 8g+7 (g = lane / 16)
template <bool T>
__device__ __forceinline__ bf16x8 xp_frag(const char* img, int base, int lane) {
  const int g = lane >> 4;
  if constexpr (!T) {
    const int r = base + (lane & 15);
    return *reinterpret_cast<const bf16x8*>(img + r * 64 + ((g ^ xp_rswz(r)) << 4));
  } else {
    const int q = (lane & 15) >> 2, pp = lane & 3;
    const int r1 = 8 * g + q, r2 = r1 + 4;
    const int cb = (base + 4 * pp) * 2;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(img + r1 * 256 + (cb ^ (32 * xp_th(r1)))));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(img + r2 * 256 + (cb ^ (32 * xp_th(r2)))));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

__device__ __forceinline__ f4 xp_mma(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void xp_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// A(m, k): AT = false -> R image of the A planes (rows m), AT = true -> T image (rows k).
// B(k, n): BT = true -> R image (rows n), BT = false -> T image (rows k).
template <bool AT, bool BT>
__global__ __launch_bounds__(XP_NT, 1) void gemm_x6p_kernel(savqa_gemm_desc d, GemmGrid gg) {
  __shared__ __attribute__((aligned(1024))) char smem[XP_NS * XP_STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave / XP_WN, wn = wave % XP_WN;
  const int bid = blockIdx.x;
  int t, slice;
  int64_t kbeg, kend;
  bool first_split, atomic;
  float* slab = nullptr;
  if (bid < gg.full) {
    split_remap(gg.full, t, slice);
    kbeg = (int64_t)slice * gg.kchunk;
    kend = min(d.K, kbeg + gg.kchunk);
    first_split = slice == 0;
    atomic = d.atomic || gridDim.y > 1;
    if (gg.slab && gridDim.y > 1) slab = gg.slab + slice * gg.slab_stride;
  } else {
    const int u = bid - gg.full;
    slice = u % gg.tail_f;
    t = gg.tail_t0 + u / gg.tail_f;
    kbeg = (int64_t)slice * gg.tail_kchunk;
    kend = min(d.K, kbeg + gg.tail_kchunk);
    first_split = slice == 0;
    atomic = true;
    if (gg.slab) slab = gg.slab + slice * gg.slab_stride;
  }
  const int tn = t % gg.tiles_n, tm = t / gg.tiles_n;
  const int64_t m0 = (int64_t)tm * XP_TILE, n0 = (int64_t)tn * XP_TILE;
  const int nt = kend > kbeg ? (int)((kend - kbeg + XP_BK - 1) / XP_BK) : 0;
  const int krem = nt > 0 ? (int)(kend - kbeg - (int64_t)(nt - 1) * XP_BK) : 0;

  XpStage<AT> sa;
  XpStage<!BT> sb;
  sa.setup(d.ap, d.ldap, d.psa, AT ? nullptr : d.a_rows, m0, d.M, kbeg, wave, lane);
  sb.setup(d.bp, d.ldbp, d.psb, BT ? d.b_rows : nullptr, n0, d.N, kbeg, wave, lane);

  f4 acc[4][XP_FN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < XP_FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const bool do_cs = AT && d.colsum_a != nullptr && tn == 0;
  float cs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = 0.f;

  auto stage = [&](int s, int kt) {
    char* img = smem + s * XP_STAGE;
    if (kt + 1 == nt && krem < XP_BK) {
      sa.issue_tail(img, wave, kt, krem);
      sb.issue_tail(img + 3 * XP_PLANE, wave, kt, krem);
    } else {
      sa.issue(img, wave, kt);
      sb.issue(img + 3 * XP_PLANE, wave, kt);
    }
  };
  if (nt > 0) {
    stage(0, 0);
    if (nt > 1) {
      stage(1, 1);
      xp_wait_vm<XP_PER>();
    } else {
      xp_wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    int cur = 0;
    for (int kt = 0; kt < nt; ++kt) {
      const char* ia = smem + cur * XP_STAGE;
      const char* ib = ia + 3 * XP_PLANE;
      if (kt + 2 < nt) stage(cur == 0 ? 2 : cur - 1, kt + 2);  // slot read in iteration kt-1
      bf16x8 b[XP_FN][3];
#pragma unroll
      for (int j = 0; j < XP_FN; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q)
          b[j][q] = xp_frag<!BT>(ib + q * XP_PLANE, wn * XP_TN + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bf16x8 a[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) a[q] = xp_frag<AT>(ia + q * XP_PLANE, wm * 64 + 16 * i, lane);
        f4 tt[XP_FN];
#pragma unroll
        for (int j = 0; j < XP_FN; ++j) tt[j] = xp_mma(a[2], b[j][0], f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int j = 0; j < XP_FN; ++j) tt[j] = xp_mma(a[1], b[j][1], tt[j]);
#pragma unroll
        for (int j = 0; j < XP_FN; ++j) tt[j] = xp_mma(a[0], b[j][2], tt[j]);
#pragma unroll
        for (int j = 0; j < XP_FN; ++j) tt[j] = xp_mma(a[1], b[j][0], tt[j]);
#pragma unroll
        for (int j = 0; j < XP_FN; ++j) tt[j] = xp_mma(a[0], b[j][1], tt[j]);
#pragma unroll
        for (int j = 0; j < XP_FN; ++j) tt[j] = xp_mma(a[0], b[j][0], tt[j]);
#pragma unroll
        for (int j = 0; j < XP_FN; ++j) acc[i][j] += tt[j];
      }
      if constexpr (AT) {
        if (do_cs) {  // block-uniform: bias gradient, the A^T image's k rows summed in fp32
          // thread (rg, cg): k rows 2rg, 2rg+1 (rg < 16 per wave-pair... all 256 threads: 16 row
          // groups x 16 column groups of 8), the three planes added back to the fp32 value
          const int cg = threadIdx.x & 15, rg = threadIdx.x >> 4;  // rg < XP_W * 4
#pragma unroll
          for (int h = 0; h < 32 / (XP_W * 4); ++h) {
            const int r = (32 / (XP_W * 4)) * rg + h;
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
            for (int q = 2; q >= 0; --q) {
              const bf16x8 x = *reinterpret_cast<const bf16x8*>(
                  ia + q * XP_PLANE + r * 256 + ((16 * cg) ^ (32 * xp_th(r))));
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] += (float)x[e];
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) cs[e] += v[e];
          }
        }
      }
      if (kt + 1 < nt) {  // k-tile kt+1 landed (kt+2 stays in flight); slot kt free after this
        if (kt + 2 < nt) xp_wait_vm<XP_PER>();
        else xp_wait_vm<0>();
        __builtin_amdgcn_s_barrier();
      }
      cur = cur == XP_NS - 1 ? 0 : cur + 1;
    }
  }
  __syncthreads();  // every wave's last reads are done: LDS is free
  if constexpr (AT) {
    if (do_cs) {  // fold the 16 row groups, one value per column (slab or atomic)
      float* red = reinterpret_cast<float*>(smem);  // [row groups][128 columns]
      const int cg = threadIdx.x & 15, rg = threadIdx.x >> 4;
      *reinterpret_cast<f4*>(&red[rg * 128 + 8 * cg]) = f4{cs[0], cs[1], cs[2], cs[3]};
      *reinterpret_cast<f4*>(&red[rg * 128 + 8 * cg + 4]) = f4{cs[4], cs[5], cs[6], cs[7]};
      __syncthreads();
      if (threadIdx.x < 128 && m0 + threadIdx.x < d.M) {
        float v = 0.f;
#pragma unroll
        for (int g = 0; g < XP_W * 4; ++g) v += red[g * 128 + threadIdx.x];
        if (gg.slab_cs) gg.slab_cs[slice * d.M + m0 + threadIdx.x] = v;
        else atomicAdd(&d.colsum_a[m0 + threadIdx.x], v);
      }
    }
  }
  gemm_epilogue16<4, XP_FN, 64, XP_TN>(d, acc, m0, n0, wm, wn, lane, first_split, atomic, slab,
                                       gg.slab_r0);
}

// Exact three-term split of fp32 rows into bf16 planes (savqa_split3): out plane q at
// P + q * ps, row r at r * ldp; columns [cols, ldp) are written as zeros. 8 columns per
// thread: two 16-B loads, three 16-B stores.
__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ X, int64_t rows,
                                                     int64_t cols, int64_t ldx,
                                                     const int64_t* __restrict__ rmap,
                                                     __bf16* __restrict__ P, int64_t ldp,
                                                     int64_t ps) {
  const int64_t per = ldp >> 3;
  const int64_t total = rows * per;
  const bool vec = (cols & 7) == 0 && (ldx & 3) == 0 && ((uintptr_t)X & 15) == 0;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total;
       u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = u / per, c = (u - r * per) * 8;
    const float* xr = X + (rmap ? rmap[r] : r) * ldx;
    float v[8];
    if (vec && c + 8 <= cols) {
      const f4 x0 = *reinterpret_cast<const f4*>(xr + c);
      const f4 x1 = *reinterpret_cast<const f4*>(xr + c + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = x0[e]; v[4 + e] = x1[e]; }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = c + e < cols ? xr[c + e] : 0.f;
    }
    bf16x8 p0, p1, p2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const __bf16 h0 = (__bf16)v[e];
      const float r1 = v[e] - (float)h0;
      const __bf16 h1 = (__bf16)r1;
      const float r2 = r1 - (float)h1;
      p0[e] = h0;
      p1[e] = h1;
      p2[e] = (__bf16)r2;
    }
    __bf16* o = P + r * ldp + c;
    *reinterpret_cast<bf16x8*>(o) = p0;
    *reinterpret_cast<bf16x8*>(o + ps) = p1;
    *reinterpret_cast<bf16x8*>(o + 2 * ps) = p2;
  }
}

}  // namespace savqa

int savqa_launch_gemm_x6p(const savqa_gemm_desc& d, const savqa::GemmGrid& gg, int grid_x,
                          int nsplit, hipStream_t s) {
  using namespace savqa;
  const dim3 g(grid_x, nsplit), b(XP_NT);
  if (!d.a_trans && d.b_trans) hipLaunchKernelGGL((gemm_x6p_kernel<false, true>), g, b, 0, s, d, gg);
  else if (!d.a_trans && !d.b_trans) hipLaunchKernelGGL((gemm_x6p_kernel<false, false>), g, b, 0, s, d, gg);
  else if (d.a_trans && !d.b_trans) hipLaunchKernelGGL((gemm_x6p_kernel<true, false>), g, b, 0, s, d, gg);
  else hipLaunchKernelGGL((gemm_x6p_kernel<true, true>), g, b, 0, s, d, gg);
  return 0;
}

extern "C" int savqa_split3(void* stream, const float* X, int64_t rows, int64_t cols, int64_t ldx,
                            const int64_t* row_map, void* planes, int64_t ldp, int64_t ps) {
  using namespace savqa;
  if (rows <= 0) return 0;
  if (!X || !planes) return fail(SAVQA_EINVAL, "savqa_split3: null argument");
  if (ldp < cols || (ldp & 7) || ((uintptr_t)planes & 15) || (ps & 7) || ps < rows * ldp)
    return fail(SAVQA_EINVAL, "savqa_split3: planes need ldp >= cols, ldp % 8 == 0, 16-B "
                              "alignment and a plane stride >= rows * ldp (multiple of 8)");
  const int64_t work = rows * (ldp >> 3);
  const int blocks = (int)std::min<int64_t>((work + 255) / 256, 8192);
  hipLaunchKernelGGL(split3_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), X, rows, cols,
                     ldx, row_map, static_cast<__bf16*>(planes), ldp, ps);
  return check_launch("savqa_split3");
}
