// fp32 GEMM on the bf16 matrix cores of gfx950 (savqa_gemm_desc.prec = 6).
//
// Same operator, operand layouts, epilogues and launch plan as gemm_f32_kernel (gemm.hip);
// only the products move from v_mfma_f32_16x16x4_f32 (64 FLOP/clk/SIMD) to
// v_mfma_f32_16x16x32_bf16 (1024 FLOP/clk/SIMD). Every fp32 operand value is split EXACTLY
// into three bf16 terms while its tile is staged (truncation split, SAVQA_X6_TRUNC):
//   a0 = a with its low 16 mantissa bits cleared, a1 = (a - a0) likewise, a2 = a - a0 - a1
// (both differences are exact fp32 values of a's sign, and the last remainder has at most 8
// significant bits, so a2 is a bf16 value: the split loses nothing), and each product is the
// sum of the six terms of order <= 2:
//   a*b = a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0)      [+ a1 b2 + a2 b1 + a2 b2]
// The dropped bracket is below 2^-21 |a b| in the worst case (|a1| < 2^-7 |a|, |a2| < 2^-15
// |a|; about 2^-25 on average, of ab's sign -- a rounded split would bound it by 2^-23 with
// either sign), bf16 x bf16 products are exact in the fp32 accumulator, and the
// accumulation is fp32 -- the accuracy of an fp32 GEMM (tests/test_kernels_gpu.py holds it to
// the native fp32 kernel's error against fp64 on every cfg-2 step shape) at 6/16 of the fp32
// MFMA's cycles per product.
// Range: every finite fp32 operand splits (truncation never rounds a term up to a bf16
// infinity). An infinite operand gives a0 = +-inf and a - a0 = NaN, and the other operand's
// terms would meet it as inf * b1 with b1 = 0 or of the opposite sign (NaN, where fp32 gives
// +-inf): x6 cannot reproduce fp32's infinities, so it does not try (a guard would cost 8 VALU
// per float4 of the split). What it does keep: an output is non-finite exactly where the fp32
// GEMM's is (NaN in place of +-inf), so overflow still surfaces
// (tests/test_kernels_gpu.py::test_gemm_x6_infinite_operands). At the small end a1 / a2 of
// |x| < 2^-110 fall below the fp32 normal range and stay exact as fp32 / bf16 subnormals (the
// 'tiny' range test holds such operands to the native kernel's error).
//
// Tiling: 256 threads = 4 waves (2x2), 128x128 outputs, k-tile 32; each wave owns 64x64 =
// 4x4 fragments of 16x16. Operand tiles are register-staged (float4 global loads issued one
// k-tile ahead, a whole k-tile of MFMAs -- 96 per wave -- to land), split in registers and
// written as three bf16 planes per operand into ONE LDS stage (48 KB: two workgroups per
// CU), two barriers per k-tile. Plane images are k-major for both operands: [128 rows][32 k]
// bf16 (64-B rows), 16-B chunk c of row r at chunk c ^ S[(r >> 2) & 3], S = {0, 2, 3, 1}, so
// a fragment (16 rows x 8 k per lane group) is one conflict-free ds_read_b128 over every
// lane group of gfx950. k-contiguous operands (X, W of the forward; dY of dX) store their
// float4s as they are; m-contiguous ones (W of dX; dY^T and X of dW) are loaded as 4k x 4m
// blocks and transposed in registers before their ds_write_b64s.
#include "gemm_common.h"

#include <type_traits>

namespace savqa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int X6_TILE = 128;
constexpr int X6_BK = 32;
constexpr int X6_ROWB = X6_BK * 2;           // bytes per plane row
constexpr int X6_PLANE = X6_TILE * X6_ROWB;  // bytes per plane (8 KB)
constexpr int X6_OCC = 2;                    // workgroups per CU (VGPR-limited)
#ifndef SAVQA_X6_DEPTH
#define SAVQA_X6_DEPTH 1
#endif
constexpr int X6_DEPTH = SAVQA_X6_DEPTH;     // k-tiles of operand loads in flight (1 or 2)

// chunk XOR of plane row r: S[(r >> 2) & 3], S = {0, 2, 3, 1}
__device__ __forceinline__ int x6_swz(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }

__device__ __forceinline__ int x6_off(int r, int k) {  // byte offset of (row, k) in a plane
  return r * X6_ROWB + ((((k >> 3) ^ x6_swz(r))) << 4) + (k & 7) * 2;
}

// exact three-term split of four fp32 values, packed as bf16 pairs: per pair one
// v_cvt_pk_bf16_f32 per term, the rounded term read back by a shift / mask of the packed word
// (22 VALU per float4; letting the compiler widen bf16x4 back to float cost 30)
__device__ __forceinline__ uint32_t pk_bf16(float x, float y) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{x, y}, bf16x2));
}
__device__ __forceinline__ float pk_lo(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float pk_hi(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

#ifndef SAVQA_X6_TRUNC
#define SAVQA_X6_TRUNC 1
#endif
#if SAVQA_X6_TRUNC
// truncation split: a0 = a with its low 16 bits cleared (the upper halves of a pair packed by
// one v_perm_b32), a - a0 exact and of the same sign, and so on. Per pair: 2 masks + 1 perm +
// 1 packed subtract per term (v_pk_add_f32), 9 VALU against 11 for the rounded split, and no
// term can round up to a bf16 infinity, so every finite fp32 operand splits.
__device__ __forceinline__ void split3(f4 v, bf16x4& p0, bf16x4& p1, bf16x4& p2) {
  typedef float f2 __attribute__((ext_vector_type(2)));
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
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  p0 = __builtin_bit_cast(bf16x4, u2{t[0][0], t[0][1]});
  p1 = __builtin_bit_cast(bf16x4, u2{t[1][0], t[1][1]});
  p2 = __builtin_bit_cast(bf16x4, u2{t[2][0], t[2][1]});
}
#else
__device__ __forceinline__ void split3(f4 v, bf16x4& p0, bf16x4& p1, bf16x4& p2) {
  uint32_t t0[2], t1[2], t2[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float x = v[2 * h], y = v[2 * h + 1];
    t0[h] = pk_bf16(x, y);
    const float rx = x - pk_lo(t0[h]), ry = y - pk_hi(t0[h]);
    t1[h] = pk_bf16(rx, ry);
    const float sx = rx - pk_lo(t1[h]), sy = ry - pk_hi(t1[h]);
    t2[h] = pk_bf16(sx, sy);
  }
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  p0 = __builtin_bit_cast(bf16x4, u2{t0[0], t0[1]});
  p1 = __builtin_bit_cast(bf16x4, u2{t1[0], t1[1]});
  p2 = __builtin_bit_cast(bf16x4, u2{t2[0], t2[1]});
}
#endif

__device__ __forceinline__ void put3(char* img, int off, f4 v) {
  bf16x4 p0, p1, p2;
  split3(v, p0, p1, p2);
  *reinterpret_cast<bf16x4*>(img + off) = p0;
  *reinterpret_cast<bf16x4*>(img + X6_PLANE + off) = p1;
  *reinterpret_cast<bf16x4*>(img + 2 * X6_PLANE + off) = p2;
}

// One operand's share of a 128 x 32 tile: 4 float4 per thread.
//   ROW (k contiguous in memory): float4 u = tid + 256 it covers tile row u / 8, k 4 (u % 8).
//   COL (m contiguous): thread (g = tid / 8, kg = tid % 8) owns tile rows 4g .. 4g+3 and
//        k 4kg .. 4kg+3; float4 it = k row 4kg + it (16 B at column 4g), transposed at store
//        time. (Each 16-lane store group covers two rows of one parity: a 2-way conflict that
//        costs a ds_write_b64 2 of its 6 cycles; staggering the rows per lane took 62 VALU.)
template <bool ROW>
struct X6Operand {
  f4 r[X6_DEPTH][4];  // X6_DEPTH register sets: k-tiles in flight
  const float* rp[4];
  // COL operands under a k-row gather (rows of the operand are k: dW's X through the GloVe
  // row map, say): the row of each float4 comes from kr per k-tile, cb = base + column
  const int64_t* kr = nullptr;
  const float* cb = nullptr;

  // FAST path pointers, resolved once per block. Edge tiles clamp: a ROW operand's rows past
  // mlim re-read row mlim-1, a COL operand's float4 groups past mlim re-read the last group
  // (mlim % 4 == 0); those plane rows only reach outputs the epilogue never stores.
  __device__ __forceinline__ void setup_fast(const float* __restrict__ base, int64_t ld,
                                             const int64_t* __restrict__ rows, int64_t m0,
                                             int64_t mlim, int tid) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      if constexpr (ROW) {
        const int u = tid + 256 * it;
        const int64_t m = min(m0 + (u >> 3), mlim - 1);
        const int64_t rr = rows ? rows[m] : m;
        rp[it] = base + rr * ld + 4 * (u & 7);
      } else {
        rp[it] = base + (int64_t)(4 * (tid & 7) + it) * ld + min(m0 + 4 * (tid >> 3), mlim - 4);
      }
    }
    if constexpr (!ROW) cb = base + min(m0 + 4 * (tid >> 3), mlim - 4);
  }

  template <int S>
  __device__ __forceinline__ void load_fast(int64_t ld, int64_t k0, int tid) {
    if constexpr (!ROW) {
      if (kr) {  // block-uniform
        const int64_t* kp = kr + k0 + 4 * (tid & 7);
        int64_t rr[4];
#pragma unroll
        for (int it = 0; it < 4; ++it) rr[it] = kp[it];
#pragma unroll
        for (int it = 0; it < 4; ++it) r[S][it] = *reinterpret_cast<const f4*>(cb + rr[it] * ld);
        return;
      }
    }
#pragma unroll
    for (int it = 0; it < 4; ++it)
      r[S][it] = *reinterpret_cast<const f4*>(ROW ? rp[it] + k0 : rp[it] + k0 * ld);
  }

  // guarded: clamped addresses, out-of-range elements selected to 0 (branch-free); rows
  // gathers the m index (ROW) or the k index (COL)
  template <int S>
  __device__ __forceinline__ void load_slow(const float* __restrict__ base, int64_t ld,
                                            const int64_t* __restrict__ rows, int64_t mlim,
                                            int64_t m0, int64_t k0, int64_t kend, int tid) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      int64_t row, col, rlim, clim;
      if constexpr (ROW) {
        const int u = tid + 256 * it;
        row = m0 + (u >> 3);
        col = k0 + 4 * (u & 7);
        rlim = mlim;
        clim = kend;
      } else {
        row = k0 + 4 * (tid & 7) + it;
        col = m0 + 4 * (tid >> 3);
        rlim = kend;
        clim = mlim;
      }
      const bool rok = row < rlim;
      const int64_t rc = rok ? row : 0;
      const int64_t rr = rows ? rows[rc] : rc;
      const float* p = base + rr * ld;
      float e[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = rok && (col + q < clim);
        const float val = p[ok ? col + q : 0];
        e[q] = ok ? val : 0.f;
      }
      r[S][it] = f4{e[0], e[1], e[2], e[3]};
    }
  }

  // colsum_a (dW bias gradient, COL operand): cs[q] += sum over this thread's 4 k of
  // A(m = 4g + q, k)
  template <int S>
  __device__ __forceinline__ void accum(f4& cs) const {
    cs += (r[S][0] + r[S][1]) + (r[S][2] + r[S][3]);
  }

  // split and store the staged values of set S into the three planes at img
  template <int S>
  __device__ __forceinline__ void store(char* img, int tid) const {
    if constexpr (ROW) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int u = tid + 256 * it;
        put3(img, x6_off(u >> 3, 4 * (u & 7)), r[S][it]);
      }
    } else {
      const int g = tid >> 3, kg = tid & 7;
#pragma unroll
      for (int s = 0; s < 4; ++s)  // k = 4kg .. 4kg+3 of tile row 4g + s
        put3(img, x6_off(4 * g + s, 4 * kg),
             f4{r[S][0][s], r[S][1][s], r[S][2][s], r[S][3][s]});
    }
  }
};

// fragment of plane img: 16 rows from base, lane (i = lane % 16, c = lane / 16) holds row
// base + i, k 8c .. 8c+7
__device__ __forceinline__ bf16x8 x6_frag(const char* img, int base, int lane) {
  const int r = base + (lane & 15);
  return *reinterpret_cast<const bf16x8*>(img + r * X6_ROWB + (((lane >> 4) ^ x6_swz(r)) << 4));
}

// 16-B LDS-DMA from an asm statement (hipcc does not track it, so it neither drains it at the
// next LDS read nor at __syncthreads(); the x6 loop counts it itself): the pre-split B planes
// (savqa_gemm_desc.b_planes). M0 is saved and restored (cdna_hip_programming.md 5.7).
typedef __attribute__((address_space(3))) void x6_lds_void;
__device__ __forceinline__ void x6_dma16(const void* src, char* dst) {
  const uint32_t l =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(x6_lds_void*)dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(l) : "memory");
}
template <int N>
__device__ __forceinline__ void x6_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ f4 mma(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// one k-tile: acc[i][j] += A_i B_j^T over 32 k, six products per term pair, smallest first.
// Two-level accumulation (X6_TWO_LEVEL): the six products of a k-tile are summed into a
// zero-started partial t and t is added to acc once per k-tile, so the running sum takes one
// rounding per 32 k instead of one per MFMA (six per 32 k; the native kernel: eight). Where one
// product dominates an output (operands spanning many decades, as real activations do) the
// single-level form rounded that product's six slices at the big accumulator's ulp: up to
// 1.5x the native kernel's error (tests/test_kernels_gpu.py::test_gemm_x6_wide_dynamic_range).
#ifndef SAVQA_X6_TWO_LEVEL
#define SAVQA_X6_TWO_LEVEL 1
#endif
__device__ __forceinline__ void x6_compute(const char* As, const char* Bs, int wm, int wn,
                                           int lane, f4 (&acc)[4][4]) {
  bf16x8 b[4][3];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int p = 0; p < 3; ++p) b[j][p] = x6_frag(Bs + p * X6_PLANE, wn * 64 + 16 * j, lane);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    bf16x8 a[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = x6_frag(As + p * X6_PLANE, wm * 64 + 16 * i, lane);
    f4 t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      t[j] = mma(a[2], b[j][0], SAVQA_X6_TWO_LEVEL ? f4{0.f, 0.f, 0.f, 0.f} : acc[i][j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = mma(a[1], b[j][1], t[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = mma(a[0], b[j][2], t[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = mma(a[1], b[j][0], t[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = mma(a[0], b[j][1], t[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) t[j] = mma(a[0], b[j][0], t[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = SAVQA_X6_TWO_LEVEL ? acc[i][j] + t[j] : t[j];
  }
}

// k-loop load mode (block-uniform): 0 = guarded loads everywhere (edge widths that are not
// whole float4 groups), 1 = branch-free loads on every k-tile, 2 = branch-free except a
// guarded last k-tile (K not a multiple of 32); k-row gathers take the same modes
template <bool AT, bool BT>
__device__ __forceinline__ int x6_mode(const savqa_gemm_desc& d, int64_t m0, int64_t n0,
                                       int64_t kbeg, int64_t kend) {
  if (m0 + X6_TILE > d.M && AT && (d.M & 3)) return 0;
  if (n0 + X6_TILE > d.N && !BT && (d.N & 3)) return 0;
  return ((kend - kbeg) % X6_BK == 0) ? 1 : 2;
}

// Split accumulators (SAVQA_X6_HILO): the dominant product a0 b0 accumulates in acc (hi), the
// five smaller ones (a2 b0, a1 b0, a1 b1, a0 b1, a0 b2: each below 2^-7 |ab|) in a second set
// lo, and hi + lo is formed once after the k-loop. hi takes one rounding per 32 k at the
// output's scale (the native fp32 kernel: eight), the small products round at lo's ulp, at
// least 2^7 finer -- more accurate than two-level, and no per-k-tile adds (whose latency behind
// the last MFMA of each partial cost cfg 2 3.5 %). Loop order is B-plane-major: b0's fragments
// meet a0 / a1 / a2, b1's a0 / a1, b2's a0 -- 28 fragment registers instead of 60, paid for by
// re-reading A fragments (36 ds_read_b128 per wave per k-tile instead of 24).
#ifndef SAVQA_X6_HILO
#define SAVQA_X6_HILO 1
#endif
#ifndef SAVQA_X6_TL_MASK
#define SAVQA_X6_TL_MASK 0  // layouts on the two-level form instead: 1 NT, 2 NN, 4 TN / TT
#endif
template <bool AT, bool BT, bool HL>
constexpr bool x6_hilo() {
  return HL && SAVQA_X6_HILO && !((SAVQA_X6_TL_MASK & (AT ? 4 : (BT ? 1 : 2))) != 0);
}
#ifndef SAVQA_X6_REREAD
#define SAVQA_X6_REREAD 0
#endif
// (hipcc keeps the A fragments of the first section live for the later ones unless a compiler
// barrier forces the re-reads: SAVQA_X6_REREAD)
__device__ __forceinline__ void x6_reread_fence() {
  if constexpr (SAVQA_X6_REREAD) asm volatile("" ::: "memory");
}
__device__ __forceinline__ void x6_compute_hilo(const char* As, const char* Bs, int wm, int wn,
                                                int lane, f4 (&hi)[4][4], f4 (&lo)[4][4]) {
  bf16x8 b[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = x6_frag(Bs, wn * 64 + 16 * j, lane);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bf16x8 a2 = x6_frag(As + 2 * X6_PLANE, wm * 64 + 16 * i, lane);
    const bf16x8 a1 = x6_frag(As + X6_PLANE, wm * 64 + 16 * i, lane);
    const bf16x8 a0 = x6_frag(As, wm * 64 + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) lo[i][j] = mma(a2, b[j], lo[i][j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) lo[i][j] = mma(a1, b[j], lo[i][j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) hi[i][j] = mma(a0, b[j], hi[i][j]);
  }
  x6_reread_fence();
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = x6_frag(Bs + X6_PLANE, wn * 64 + 16 * j, lane);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bf16x8 a1 = x6_frag(As + X6_PLANE, wm * 64 + 16 * i, lane);
    const bf16x8 a0 = x6_frag(As, wm * 64 + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) lo[i][j] = mma(a1, b[j], lo[i][j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) lo[i][j] = mma(a0, b[j], lo[i][j]);
  }
  x6_reread_fence();
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = x6_frag(Bs + 2 * X6_PLANE, wn * 64 + 16 * j, lane);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bf16x8 a0 = x6_frag(As, wm * 64 + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) lo[i][j] = mma(a0, b[j], lo[i][j]);
  }
}

template <bool AT, bool BT, int MODE, bool HL, bool BP>
__device__ __forceinline__ void x6_mainloop(const savqa_gemm_desc& d, char* smem, int64_t m0,
                                            int64_t n0, int64_t kbeg, int64_t kend, int ntiles,
                                            f4 (&acc)[4][4], bool do_cs, f4& cs) {
  X6Operand<!AT> la;
  X6Operand<BT> lb;
  f4 lo[4][4];  // SAVQA_X6_HILO: the small products' accumulators
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) lo[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  if constexpr (MODE != 0) {
    la.setup_fast(d.A, d.lda, AT ? nullptr : d.a_rows, m0, d.M, tid);
    lb.setup_fast(d.B, d.ldb, BT ? d.b_rows : nullptr, n0, d.N, tid);
    if constexpr (AT) la.kr = d.a_rows;
    if constexpr (!BT) lb.kr = d.b_rows;
  }
  auto load = [&](auto set, int64_t k0) {
    constexpr int S = decltype(set)::value;
    if (MODE == 1 || (MODE == 2 && k0 + X6_BK <= kend)) {
      la.template load_fast<S>(d.lda, k0, tid);
      lb.template load_fast<S>(d.ldb, k0, tid);
    } else {
      la.template load_slow<S>(d.A, d.lda, d.a_rows, d.M, m0, k0, kend, tid);
      lb.template load_slow<S>(d.B, d.ldb, d.b_rows, d.N, n0, k0, kend, tid);
    }
  };
  // k-tile tt from register set S: split into the planes, refill S with k-tile tt + DEPTH
  // (DEPTH k-tiles of loads in flight), then the MFMAs
  auto step = [&](auto set, int tt) {
    constexpr int S = decltype(set)::value;
    if (do_cs) la.template accum<S>(cs);
    if (tt > 0) __syncthreads();  // every wave has read k-tile tt-1's planes
    la.template store<S>(smem, tid);
    lb.template store<S>(smem + 3 * X6_PLANE, tid);
    if (tt + X6_DEPTH < ntiles) load(set, kbeg + (int64_t)(tt + X6_DEPTH) * X6_BK);
    __syncthreads();
    if constexpr (x6_hilo<AT, BT, HL>())
      x6_compute_hilo(smem, smem + 3 * X6_PLANE, wm, wn, lane, acc, lo);
    else
      x6_compute(smem, smem + 3 * X6_PLANE, wm, wn, lane, acc);
  };
  if constexpr (BP) {
    // B from its pre-split planes (savqa_x6_weight_planes): 24 KB per k-tile, DMA'd one k-tile
    // ahead into the other half of a double buffer (6 x 1 KB per wave); A as usual. Before the
    // barrier that precedes k-tile tt's MFMAs, tt's DMA must have landed: the wave issued at
    // least 4 A loads and 6 DMAs after it (k-tile tt+1), so vmcnt(10) retires it.
    static_assert(!AT, "planes: the A operand must be the k-contiguous one");
    const int64_t KT = (d.K + X6_BK - 1) / X6_BK;
    const char* bsrc = static_cast<const char*>(d.b_planes) +
                       ((n0 / X6_TILE) * KT + kbeg / X6_BK) * (3 * X6_PLANE) + wave * 6 * 1024 +
                       lane * 16;
    auto dma_b = [&](int buf, int tt) {
      char* dst = smem + 3 * X6_PLANE + buf * 3 * X6_PLANE + wave * 6 * 1024;
      const char* src = bsrc + (int64_t)tt * (3 * X6_PLANE);
#pragma unroll
      for (int u = 0; u < 6; ++u) x6_dma16(src + u * 1024, dst + u * 1024);
    };
    auto load_a = [&](int64_t k0) {
      if (MODE == 1 || (MODE == 2 && k0 + X6_BK <= kend))
        la.template load_fast<0>(d.lda, k0, tid);
      else
        la.template load_slow<0>(d.A, d.lda, d.a_rows, d.M, m0, k0, kend, tid);
    };
    load_a(kbeg);
    dma_b(0, 0);
    for (int tt = 0; tt < ntiles; ++tt) {
      if (tt > 0) __syncthreads();  // every wave has read k-tile tt-1's planes
      la.template store<0>(smem, tid);
      const bool nx = tt + 1 < ntiles;  // (uniform)
      if (nx) {
        load_a(kbeg + (int64_t)(tt + 1) * X6_BK);
        dma_b((tt + 1) & 1, tt + 1);
        x6_wait_vm<10>();
      } else {
        x6_wait_vm<0>();
      }
      __syncthreads();
      const char* Bs = smem + 3 * X6_PLANE + (tt & 1) * 3 * X6_PLANE;
      if constexpr (x6_hilo<AT, BT, HL>())
        x6_compute_hilo(smem, Bs, wm, wn, lane, acc, lo);
      else
        x6_compute(smem, Bs, wm, wn, lane, acc);
    }
    if constexpr (x6_hilo<AT, BT, HL>()) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += lo[i][j];
    }
    __syncthreads();
    return;
  }
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, X6_DEPTH - 1>;
  load(S0{}, kbeg);
  if (X6_DEPTH > 1 && ntiles > 1) load(S1{}, kbeg + X6_BK);
  for (int tt = 0; tt < ntiles; tt += X6_DEPTH) {
    step(S0{}, tt);
    if (X6_DEPTH > 1 && tt + 1 < ntiles) step(S1{}, tt + 1);
  }
  if constexpr (x6_hilo<AT, BT, HL>()) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] += lo[i][j];
  }
  __syncthreads();  // LDS is reused by the colsum fold
}

// HL: the hi / lo accumulators (x6_compute_hilo); false: the two-level form (x6_compute),
// which adds each k-tile's partial into the accumulator with a VALU (RNE) add instead of
// inside the MFMA -- savqa_gemm_desc.prec = 5, for launches whose outputs feed a rounding-
// sensitive chain (the engine's decoder K / V projection: a softmax over T keys in all 6
// decoder layers)
template <bool AT, bool BT, bool HL, bool BP>
__global__ __launch_bounds__(GEMM_NT, X6_OCC) void gemm_x6_kernel(savqa_gemm_desc d, GemmGrid gg) {
  // A planes 0-2, B planes 0-2 (BP: B planes double-buffered, 72 KB: still two per CU)
  __shared__ __attribute__((aligned(16))) char smem[(BP ? 9 : 6) * X6_PLANE];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int bid = blockIdx.x;
  int t, slice;
  int64_t kbeg, kend;
  bool first_split, atomic;
  float* slab = nullptr;  // slab mode: this block's partial-tile slab
  if (bid < gg.full) {    // (split launches have no tail: grid.x == gg.full)
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
  const int64_t m0 = (int64_t)tm * X6_TILE, n0 = (int64_t)tn * X6_TILE;
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int ntiles = kend > kbeg ? (int)((kend - kbeg + X6_BK - 1) / X6_BK) : 0;
  // colsum_a (a_trans only): column tile 0 also sums its A tiles over k (bias gradient)
  const bool do_cs = AT && d.colsum_a != nullptr && tn == 0;
  f4 cs = {0.f, 0.f, 0.f, 0.f};
  if (ntiles > 0) {
    const int mode = x6_mode<AT, BT>(d, m0, n0, kbeg, kend);
    if (mode == 1)
      x6_mainloop<AT, BT, 1, HL, BP>(d, smem, m0, n0, kbeg, kend, ntiles, acc, do_cs, cs);
    else if (mode == 2)
      x6_mainloop<AT, BT, 2, HL, BP>(d, smem, m0, n0, kbeg, kend, ntiles, acc, do_cs, cs);
    else
      x6_mainloop<AT, BT, 0, HL, BP>(d, smem, m0, n0, kbeg, kend, ntiles, acc, do_cs, cs);
  }
  if constexpr (AT) {
    if (do_cs) {  // block-uniform; LDS is free after the main loop's last barrier
      // thread (g, kg) holds partials of columns 4g .. 4g+3: plain LDS rows per kg, then one
      // thread per column (no LDS float atomics)
      float* red = reinterpret_cast<float*>(smem);
      *reinterpret_cast<f4*>(&red[(threadIdx.x & 7) * X6_TILE + 4 * (threadIdx.x >> 3)]) = cs;
      __syncthreads();
      for (int i = threadIdx.x; i < X6_TILE; i += GEMM_NT) {
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) v += red[r * X6_TILE + i];
        if (m0 + i < d.M) {
          if (gg.slab_cs) gg.slab_cs[slice * d.M + m0 + i] = v;
          else atomicAdd(&d.colsum_a[m0 + i], v);
        }
      }
    }
  }
  gemm_epilogue16<4, 4, 64, 64>(d, acc, m0, n0, wm, wn, lane, first_split, atomic, slab,
                                gg.slab_r0);
}

}  // namespace savqa

// Launch of the x6 kernels on a plan made by savqa_gemm (gemm.hip): grid (grid_x, nsplit).
int savqa_launch_gemm_x6(const savqa_gemm_desc& d, const savqa::GemmGrid& gg, int grid_x,
                         int nsplit, hipStream_t s, bool two_level) {
  using namespace savqa;
  const dim3 g(grid_x, nsplit), b(GEMM_NT);
#define SAVQA_X6_GO(AT_, BT_, HL_, BP_) \
  hipLaunchKernelGGL((gemm_x6_kernel<AT_, BT_, HL_, BP_>), g, b, 0, s, d, gg)
  if (d.b_planes && !d.a_trans) {  // (the caller checked the planes' fit: savqa_gemm)
    if (two_level) {
      if (d.b_trans) SAVQA_X6_GO(false, true, false, true);
      else SAVQA_X6_GO(false, false, false, true);
    } else {
      if (d.b_trans) SAVQA_X6_GO(false, true, true, true);
      else SAVQA_X6_GO(false, false, true, true);
    }
    return 0;
  }
  if (two_level) {
    if (!d.a_trans && d.b_trans) SAVQA_X6_GO(false, true, false, false);
    else if (!d.a_trans && !d.b_trans) SAVQA_X6_GO(false, false, false, false);
    else if (d.a_trans && !d.b_trans) SAVQA_X6_GO(true, false, false, false);
    else SAVQA_X6_GO(true, true, false, false);
    return 0;
  }
  if (!d.a_trans && d.b_trans) SAVQA_X6_GO(false, true, true, false);
  else if (!d.a_trans && !d.b_trans) SAVQA_X6_GO(false, false, true, false);
  else if (d.a_trans && !d.b_trans) SAVQA_X6_GO(true, false, true, false);
  else SAVQA_X6_GO(true, true, true, false);
#undef SAVQA_X6_GO
  return 0;
}

// ------------------------------------------------------------------ pre-split B planes
namespace savqa {
// Up to X6_PJOBS operands per launch (an optimizer step's weights in one or a few launches:
// one launch per weight ran ~6 us each, latency-bound at one workgroup per CU).
constexpr int X6_PJOBS = 32;
struct X6PlanesJob {
  const float* B;
  int64_t ldb, N, K;
  char* out;
  int32_t b_trans, KT;
};
struct X6PlanesBatch {
  X6PlanesJob j[X6_PJOBS];
  int32_t start[X6_PJOBS + 1];  // first workgroup of each job; start[n] = grid size
  int32_t n;
};

// one workgroup per (n tile, k tile) of one job: the 128 x 32 B tile split like the kernel's
// own staging (X6Operand<ROW / COL>::store), zeros past N / K. k-contiguous B (b_trans):
// thread u -> row u / 8, k 4 (u % 8), 16-B loads along k; n-contiguous B: thread (g, kg) ->
// rows 4g .. 4g+3, k 4kg .. 4kg+3, 16-B loads along n, transposed in registers.
__global__ __launch_bounds__(256) void x6_planes_kernel(const X6PlanesBatch bt) {
  int j = 0;
  while (j + 1 < bt.n && (int)blockIdx.x >= bt.start[j + 1]) ++j;  // uniform: scalar loop
  const X6PlanesJob& J = bt.j[j];
  const int tile = (int)blockIdx.x - bt.start[j];
  const int nt = tile / J.KT, kt = tile - nt * J.KT;
  const float* __restrict__ Bp = J.B;
  const int64_t n0 = (int64_t)nt * X6_TILE, k0 = (int64_t)kt * X6_BK, ldb = J.ldb;
  char* img = J.out + (int64_t)tile * (3 * X6_PLANE);
  const bool full = n0 + X6_TILE <= J.N && k0 + X6_BK <= J.K && (ldb & 3) == 0 &&
                    ((uintptr_t)Bp & 15) == 0;
  const int t = threadIdx.x;
  if (J.b_trans) {
    f4 v[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int u = t + 256 * it, r = u >> 3, k4 = 4 * (u & 7);
      const float* src = Bp + (n0 + r) * ldb + k0 + k4;
      if (full) {
        v[it] = *reinterpret_cast<const f4*>(src);
      } else {
        v[it] = f4{0.f, 0.f, 0.f, 0.f};
        if (n0 + r < J.N)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (k0 + k4 + e < J.K) v[it][e] = src[e];
      }
    }
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int u = t + 256 * it;
      put3(img, x6_off(u >> 3, 4 * (u & 7)), v[it]);
    }
  } else {
    const int g = t >> 3, kg = t & 7;
    f4 v[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int64_t k = k0 + 4 * kg + it;
      const float* src = Bp + k * ldb + n0 + 4 * g;
      if (full) {
        v[it] = *reinterpret_cast<const f4*>(src);
      } else {
        v[it] = f4{0.f, 0.f, 0.f, 0.f};
        if (k < J.K)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n0 + 4 * g + e < J.N) v[it][e] = src[e];
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
      put3(img, x6_off(4 * g + s, 4 * kg), f4{v[0][s], v[1][s], v[2][s], v[3][s]});
  }
}
}  // namespace savqa

extern "C" int64_t savqa_x6_weight_planes_bytes(int64_t N, int64_t K) {
  if (N <= 0 || K <= 0) return 0;
  return ((N + 127) / 128) * ((K + 31) / 32) * 3 * (int64_t)savqa::X6_PLANE;
}

extern "C" int savqa_x6_weight_planes_batch(void* stream, const savqa_x6_planes_job* jobs,
                                            int32_t n) {
  using namespace savqa;
  if (n < 0 || (n > 0 && !jobs))
    return fail(SAVQA_EINVAL, "savqa_x6_weight_planes_batch: null job list");
  for (int i = 0; i < n; ++i) {
    const savqa_x6_planes_job& q = jobs[i];
    if (q.N <= 0 || q.K <= 0) continue;
    if (!q.B || !q.out || ((uintptr_t)q.out & 15) || q.ldb < (q.b_trans ? q.K : q.N))
      return fail(SAVQA_EINVAL, "savqa_x6_weight_planes: null operand, unaligned output or "
                                "leading dimension below the operand's extent");
  }
  X6PlanesBatch bt;
  int i = 0;
  while (i < n) {
    bt.n = 0;
    int64_t blocks = 0;
    for (; i < n && bt.n < X6_PJOBS; ++i) {
      const savqa_x6_planes_job& q = jobs[i];
      if (q.N <= 0 || q.K <= 0) continue;
      const int64_t KT = (q.K + X6_BK - 1) / X6_BK, NT = (q.N + X6_TILE - 1) / X6_TILE;
      if (blocks + NT * KT > (int64_t)INT32_MAX) break;
      X6PlanesJob& J = bt.j[bt.n];
      J.B = q.B;
      J.ldb = q.ldb;
      J.N = q.N;
      J.K = q.K;
      J.out = static_cast<char*>(q.out);
      J.b_trans = q.b_trans ? 1 : 0;
      J.KT = (int32_t)KT;
      bt.start[bt.n++] = (int32_t)blocks;
      blocks += NT * KT;
    }
    if (bt.n == 0) {
      if (i < n && blocks == 0) return fail(SAVQA_EINVAL, "savqa_x6_weight_planes: operand too large");
      break;
    }
    bt.start[bt.n] = (int32_t)blocks;
    hipLaunchKernelGGL(x6_planes_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), bt);
    const int rc = check_launch("savqa_x6_weight_planes");
    if (rc) return rc;
  }
  return 0;
}

extern "C" int savqa_x6_weight_planes(void* stream, const float* Bp, int64_t ldb, int32_t b_trans,
                                      int64_t N, int64_t K, void* out) {
  savqa_x6_planes_job q = {Bp, ldb, b_trans, 0, N, K, out};
  return savqa_x6_weight_planes_batch(stream, &q, 1);
}
