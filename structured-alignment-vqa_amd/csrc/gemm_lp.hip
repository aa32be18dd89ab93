// Low-precision-operand GEMM for gfx950 (savqa_gemm_lp, include/savqa.h): bf16-resident
// operands on v_mfma_f32_16x16x32_bf16, or fp8-e4m3 operands with e8m0 block scales on
// v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 rate per clock), fp32 accumulation,
// fused epilogue with fp32 and/or bf16 outputs. It carries the big Linears of the bf16 /
// fp8 training modes (BASELINE cfg 3 / cfg 5): forward C = X W^T (NT), dX = dY W (NN) and
// dW += dY^T X (TN) on the same 128x128 tile machinery.
//
// Tile: 256 threads = 4 waves (2x2), 128x128 outputs, k-tile = 128 bytes of every operand
// row (64 bf16 / 128 fp8). Both operand tiles are staged by LDS-DMA (global_load_lds
// dwordx4, 16 per wave per k-tile), double-buffered (64 KB: two workgroups per CU), one
// barrier per k-tile. Each operand keeps its GLOBAL orientation in LDS and the transpose,
// where the MFMA needs one, happens in the read:
//   R image (k contiguous: X / W of the forward, dY of dX): [128 rows][128 B], 16-B chunk
//     c of row r stored at chunk c ^ swz(r) -- fragments are ds_read_b128 (conflict-free);
//   T image (m / n contiguous: W of dX, dY and X of dW): [64 k rows][128 cols] bf16,
//     256-B rows, byte b of row r stored at b ^ 32*h(r) -- fragments are two
//     ds_read_b64_tr_b16 (hardware transpose; conflict-free with this swizzle).
// LDS-DMA writes lane-linear 16-B granules, so the swizzle is applied to each lane's
// SOURCE address (cdna_hip_programming.md rule 21) and undone by the reads.
// The MFMA is issued with the operands swapped (C^T tile = B^T A^T), so each lane holds
// 4 consecutive output COLUMNS of one row: 16-B fp32 / 8-B bf16 epilogue stores.
#include "gemm_common.h"

#include <type_traits>

#include <algorithm>

namespace savqa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int LP_NT = 256;        // threads per workgroup
constexpr int LP_TILE = 128;      // output rows / columns per workgroup
constexpr int LP_KB = 128;        // k bytes per operand row per k-tile
constexpr int LP_IMG = 128 * 128; // bytes of one operand image (16 KB)
constexpr int LP_OCC = 2;         // workgroups per CU (64 KB LDS each)

// R-image swizzle: 16-B chunk c of tile row r lives at chunk c ^ (r & 7). bf16 fragments read
// chunk (4*kk + g) of 16 rows, fp8 fragments chunks (g, g+4): both ds_read_b128 patterns
// are conflict-free with it (checked against the gfx950 lane groups).
template <bool FP8>
__device__ __forceinline__ int rswz(int r) {
  return r & 7;
}
// T-image swizzle: byte b of k-row r at b ^ (32 * h(r)); a 32-lane half of a transposed read
// touches rows {8G+q, 8G+8+q}, which h maps to 8 distinct 32-B columns.
__device__ __forceinline__ int th(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

__device__ __forceinline__ void glds16(const void* src, lds_void* dst) {
  __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
}

// The same LDS-DMA as an asm statement hipcc does not see (cdna_hip_programming.md 5.7,
// the M0 save / restore recipe). hipcc treats a pending __builtin_amdgcn_global_load_lds as a
// write to LDS it cannot tell apart from the k-tile being read, and waits vmcnt(0) before the
// first ds_read after it: in the 128 x 128 kernel that drained the NEXT k-tile's DMAs before
// every k-tile's MFMAs (the .s showed s_waitcnt vmcnt(0) at the loop head) -- no overlap of
// staging and compute at all. Hidden in asm, the DMAs stay in flight; the kernel counts them
// itself (lp_wait_vm before each barrier).
#ifndef SAVQA_LP_ASM_DMA
#define SAVQA_LP_ASM_DMA 1
#endif
template <int BYTES>
__device__ __forceinline__ void glds_asm(const void* src, lds_void* dst) {
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
  unsigned keep;
  if constexpr (BYTES == 16)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(l) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(l) : "memory");
}
template <int BYTES>
__device__ __forceinline__ void glds_k(const void* src, lds_void* dst) {  // the k-loop's DMAs
  if constexpr (SAVQA_LP_ASM_DMA) glds_asm<BYTES>(src, dst);
  else if constexpr (BYTES == 16) __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
  else __builtin_amdgcn_global_load_lds(src, dst, 4, 0, 0);
}

// 16 zero bytes: the LDS-DMA source of every operand granule past the end of K (the last,
// partial k-tile of a K that is not a multiple of the k-tile)
__device__ __attribute__((aligned(16))) uint4 g_lp_zero[1];

struct LpArgs {
  savqa_gemm_lp_desc d;
  int tiles_n, ntiles_k;  // k-tiles per split slice
  int64_t kchunk;         // elements of k per split slice
  int nblk;               // tiles (grid.x)
  // tail split (gemm_lp_kernel, unsplit launches): blocks >= full take the last tiles, from
  // tail_t0 on, in tail_f k-slices of tail_kchunk each, accumulated atomically into C
  int full, tail_t0, tail_f;
  int64_t tail_kchunk;
  float* slab;            // split-K partial slabs [slice][M][N] (savqa_gemm_lp_desc.ws), or null
  float* tail_slab;       // tail-split partial slabs [slice][M - tail_r0][N] (same workspace),
  int64_t tail_r0;        // or null: the tail tiles' slices then add into C atomically
  float* cs_slab;         // split-K launches with slabs: the fused column sum's per-slice
                          // partials [slice][M] (after the C slabs), else null (atomics)
  int dbg;                // diagnostic builds only (SAVQA_LP_DIAG=1, tools/lp_bench.py --dbg):
                          // 1 = skip the MFMAs, 2 = skip the k-loop DMAs, 4 = skip the
                          // epilogue; production builds compile every test of it away
};

#ifndef SAVQA_LP_DIAG
#define SAVQA_LP_DIAG 0
#endif
__device__ __forceinline__ int lp_dbg(const LpArgs& a) { return SAVQA_LP_DIAG ? a.dbg : 0; }

// Per-lane LDS-DMA sources of one operand, resolved once per workgroup.
//   R image: instruction u of wave w covers tile rows 8(4w+u) .. +7; lane L -> row
//     8(4w+u) + L/8, physical chunk L%8, logical chunk (L%8) ^ swz(row).
//   T image: instruction u covers k rows 4(4w+u) .. +3; lane L -> row 4(4w+u) + L/16,
//     physical chunk L%16, logical chunk (L%16) ^ 2h(row); advances by whole rows.
template <bool T, bool FP8>
struct LpStage {
  const char* p[4];
  int koff[4];   // k of this lane's granule within a k-tile
  int64_t step;  // bytes per k-tile

  __device__ __forceinline__ void setup(const void* base, int64_t ld, int esz,
                                        const int64_t* __restrict__ rows, int64_t r0, int64_t lim,
                                        int64_t kbeg, int wave, int lane) {
    const char* b = static_cast<const char*>(base);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ins = 4 * wave + u;
      if constexpr (!T) {
        const int r = 8 * ins + (lane >> 3);
        const int lc = (lane & 7) ^ rswz<FP8>(r);
        int64_t m = r0 + r;
        m = m < lim ? m : lim - 1;
        const int64_t rr = rows ? rows[m] : m;
        p[u] = b + (rr * ld + kbeg) * esz + lc * 16;
        koff[u] = lc * 16 / esz;
      } else {
        const int r = 4 * ins + (lane >> 4);
        const int lc = (lane & 15) ^ (2 * th(r));
        int64_t c = r0 + lc * 8;
        c = c + 8 <= lim ? c : lim - 8;
        p[u] = b + ((kbeg + r) * ld + c) * esz;
        koff[u] = r;
      }
    }
    step = T ? (int64_t)64 * ld * esz : LP_KB;
  }

  __device__ __forceinline__ void issue(char* img, int wave, int64_t t) const {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      glds_k<16>(p[u] + t * step, (lds_void*)(img + (4 * wave + u) * 1024));
  }

  // partial last k-tile: granules at k >= krem (within the tile) load zeros
  __device__ __forceinline__ void issue_tail(char* img, int wave, int64_t t, int krem) const {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      glds_k<16>(koff[u] < krem ? (const void*)(p[u] + t * step) : (const void*)g_lp_zero,
                 (lds_void*)(img + (4 * wave + u) * 1024));
  }
};

// L2 prefetch of a future k-tile (SAVQA_LP_PF k-tiles beyond the one being staged; bf16
// 128 x 128 kernel): every lane touches one 128-B line of its workgroup's operand tiles -- waves
// 0-1 the A tile's 128 lines, waves 2-3 the B tile's -- by a 4-byte LDS-DMA into a dummy slot
// (no VGPR destination, nothing reads it). A k-loop launch whose operands come cold from HBM
// (the split-K weight gradients of a training step read activations written long before: in-step
// they ran 1.2x their back-to-back time, profiles/r06_cfg3_gemm_replay.txt) otherwise waits a
// full HBM latency per k-tile, since only the next k-tile is in flight; with the prefetch the
// stage DMAs hit L2. The wait at the end of a k-tile becomes vmcnt(1) (the newest prefetch may
// stay in flight; LDS-DMAs complete in issue order) with a raw barrier.
// Measured (tools/gemm_replay.py, cfg-3 in-step launches, interleaved builds on one box):
// with the DMAs in asm, the split-K dW 140 -> 106 us in-step; prefetching 2 or 4 k-tiles ahead
// on top made it slower again (126-142 us: a line request per lane per k-tile through the
// TA), so the prefetch is built but off.
#ifndef SAVQA_LP_PF
#define SAVQA_LP_PF 0
#endif
constexpr int LP_PF = SAVQA_LP_PF;
constexpr int LP_PF_BYTES = LP_PF > 0 ? 1024 : 0;  // dummy LDS-DMA slots, 256 B per wave

struct LpPf {
  const char* base;  // this lane's line at k-tile 0 (k-row 0 of the tile for T images)
  int64_t step;      // bytes per k-tile
  int64_t krow, kmax;  // T image: this lane's k row within the launch; last valid row (K - 1)
  int64_t ld_b;        // T image: bytes per k row
  bool t;

  template <bool T>
  __device__ __forceinline__ void setup(const void* b0, int64_t ld, int esz,
                                        const int64_t* __restrict__ rows, int64_t r0, int64_t lim,
                                        int64_t kbeg, int64_t K, int q) {
    const char* b = static_cast<const char*>(b0);
    t = T;
    if constexpr (!T) {  // tile row q (one 128-B line: 64 bf16 of k)
      int64_t m = r0 + q;
      m = m < lim ? m : lim - 1;
      const int64_t rr = rows ? rows[m] : m;
      base = b + (rr * ld + kbeg) * esz;
      step = LP_KB;
      krow = kmax = 0;
      ld_b = 0;
    } else {             // k row q / 2, columns 64 (q & 1) .. +63 of the tile
      int64_t c = r0 + 64 * (q & 1);
      c = c + 8 <= lim ? c : lim - 8;
      base = b + c * esz;
      krow = kbeg + (q >> 1);
      kmax = K - 1;
      ld_b = ld * esz;
      step = 64;
    }
  }

  __device__ __forceinline__ void issue(int64_t kt, lds_void* dummy) const {
    const char* src;
    if (t) {
      int64_t k = krow + kt * step;
      k = k < kmax ? k : kmax;
      src = base + k * ld_b;
    } else {
      src = base + kt * step;
    }
    glds_k<4>(src, dummy);
  }
};

template <int N>
__device__ __forceinline__ void lp_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// bf16 fragment of 16 rows (R image) / 16 columns (T image), k 32kk + 8g .. +7 per lane
template <bool T>
__device__ __forceinline__ bf16x8 frag_bf16(const char* img, int base, int kk, int lane) {
  const int g = lane >> 4;
  if constexpr (!T) {
    const int r = base + (lane & 15);
    const int pc = (4 * kk + g) ^ rswz<false>(r);
    return *reinterpret_cast<const bf16x8*>(img + r * 128 + pc * 16);
  } else {
    const int q = (lane & 15) >> 2, p = lane & 3;
    const int r1 = 32 * kk + 8 * g + q, r2 = r1 + 4;
    const int cb = (base + 4 * p) * 2;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(img + r1 * 256 + (cb ^ (32 * th(r1)))));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(img + r2 * 256 + (cb ^ (32 * th(r2)))));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

// fp8 fragment (R image only): 16 rows x 128 k. Measured lane map of the scaled MFMA
// (tools/probe_mfma_fp8.hip): lane (row l&15, g = l>>4) holds two 16-k halves, k 16g..16g+15
// (bytes 0-15) and 64+16g..64+16g+15 (bytes 16-31); the e8m0 scale of 32-k block b of row
// r comes from lane r + 16b. Both operands use the same map, so each lane's scale register
// carries block g of its row.
__device__ __forceinline__ i32x8 frag_fp8(const char* img, int base, int lane) {
  const int g = lane >> 4;
  const int r = base + (lane & 15);
  const int s = rswz<true>(r);
  const i32x4 a = *reinterpret_cast<const i32x4*>(img + r * 128 + (g ^ s) * 16);
  const i32x4 b = *reinterpret_cast<const i32x4*>(img + r * 128 + ((g + 4) ^ s) * 16);
  return i32x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

__device__ __forceinline__ float bf2f(__bf16 v) { return (float)v; }

// Row-major store of G rows of one wave's staged [64][64] image (rows 4(Gh + q) + lane/16,
// q < G; 4 columns per lane), with every epilogue operand of the G rows loaded BEFORE the
// first store: a load issued after a store waits for it (vmcnt counts both), so loading
// per row serialised the whole epilogue on store latency. Requires the vector layout
// (N % 4 == 0, 16-B / 8-B aligned rows: lp_vec_epilogue). Rows past M and columns past N
// load a clamped (valid) address and are not stored. MK: 0 none, 1 bf16 mask, 2 fp32 mask.
template <int G, bool RES, int MK, bool RV>
__device__ __forceinline__ void lp_rows(const savqa_gemm_lp_desc& d, const char* reg,
                                         int64_t rbase, int h, int64_t n, bool nok, int64_t nc,
                                         f4 bv, bool ident, int lane) {
  const int c = lane & 15;
  f4 rs[G], rv[G], mk[G];
#pragma unroll
  for (int q = 0; q < G; ++q) {
    const int lr = 4 * (G * h + q) + (lane >> 4);
    int64_t m = rbase + lr;
    m = m < d.M ? m : d.M - 1;
    if constexpr (RES) rs[q] = *reinterpret_cast<const f4*>(d.resid + m * d.ldr + nc);
    if constexpr (RV)
      rv[q] = *reinterpret_cast<const f4*>(d.rowvec + (m % d.rowvec_period) * d.ldrv + nc);
    if constexpr (MK != 0) {
      const int64_t mr = d.mask_arows ? d.a_rows[m] : m;
      if constexpr (MK == 1)
        mk[q] = __builtin_convertvector(
            *reinterpret_cast<const bf16x4*>(static_cast<const __bf16*>(d.mask) + mr * d.ldmask + nc), f4);
      else
        mk[q] = *reinterpret_cast<const f4*>(static_cast<const float*>(d.mask) + mr * d.ldmask + nc);
    }
  }
#pragma unroll
  for (int q = 0; q < G; ++q) {
    const int lr = 4 * (G * h + q) + (lane >> 4);
    const int64_t m = rbase + lr;
    f4 v = *reinterpret_cast<const f4*>(reg + (lr & 63) * 256 + ((c ^ (lr & 15)) * 16));
    v = v * d.alpha + bv;
    if constexpr (RV) v += rv[q];
    if (d.relu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
    }
    if constexpr (MK != 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (!(mk[q][r] > 0.f)) v[r] = 0.f;
    }
    if constexpr (RES) v += rs[q];
    if (m < d.M && nok) {
      int64_t cr = m;
      if (!ident) {
        const uint32_t mu = (uint32_t)m, cg = (uint32_t)d.c_group;
        cr = (int64_t)(mu / cg) * d.c_stride + (int64_t)(mu % cg) + d.c_offset;
      }
      if (d.C) *reinterpret_cast<f4*>(d.C + cr * d.ldc + n) = v;
      if (d.Cb)
        *reinterpret_cast<bf16x4*>(static_cast<__bf16*>(d.Cb) + cr * d.ldcb + n) =
            __builtin_convertvector(v, bf16x4);
    }
  }
}

// whether every epilogue operand and output allows the vector rows of lp_rows
__host__ __device__ __forceinline__ bool lp_vec_epilogue(const savqa_gemm_lp_desc& d) {
  auto al = [](const void* p, int b) { return (((uintptr_t)p) & (b - 1)) == 0; };
  if (d.N % 4) return false;
  if (d.rowvec && (d.resid || d.mask)) return false;  // not instantiated: per-row path
  if (d.C && ((d.ldc & 3) || !al(d.C, 16))) return false;
  if (d.Cb && ((d.ldcb & 3) || !al(d.Cb, 8))) return false;
  if (d.resid && ((d.ldr & 3) || !al(d.resid, 16))) return false;
  if (d.rowvec && ((d.ldrv & 3) || !al(d.rowvec, 16))) return false;
  if (d.mask && ((d.ldmask & 3) || !al(d.mask, d.mask_type == SAVQA_DT_BF16 ? 8 : 16))) return false;
  return true;
}

// Output column of staged-image column c (0..63) of a wave tile whose two 32-column halves
// start at col0 and col_hi (col_hi = col0 + 32 for a contiguous 64-column wave tile).
__device__ __forceinline__ int64_t ecol(int64_t col0, int64_t col_hi, int c) {
  return c < 32 ? col0 + c : col_hi + (c - 32);
}

// Wide row stores for bf16-only outputs: a wave64 store of bf16x4 per lane (8 B) makes the
// epilogue store-issue-bound (cdna_hip_programming.md T21), so each lane takes 8 consecutive
// columns (two 16-B chunks of the staged fp32 row) and stores them as one 16-B bf16x8: 8 lanes
// per 128-B row segment, 8 rows per instruction, 8 instructions per 64-row pass. Optional
// bf16 ReLU-backward mask (16-B loads in the same map), loaded here or prefetched (PRE).
__host__ __device__ __forceinline__ bool lp_wide_epilogue(const savqa_gemm_lp_desc& d) {
  auto al = [](const void* p, int b) { return (((uintptr_t)p) & (b - 1)) == 0; };
  if (!d.Cb || d.C || d.resid || d.rowvec || d.atomic || d.N % 8) return false;
  if ((d.ldcb & 7) || !al(d.Cb, 16)) return false;
  if (d.mask && d.mask_type != SAVQA_DT_BITS &&
      (d.mask_type != SAVQA_DT_BF16 || (d.ldmask & 7) || !al(d.mask, 16)))
    return false;
  return true;
}

// the gate bytes of one lane in the wide map (SAVQA_DT_BITS mask: bits 0-7 = its 8 columns of
// rows rb + 8q + lane/8), one zero-extended byte per register so a prefetch holds no wait
__device__ __forceinline__ void lp_wide_bits(const savqa_gemm_lp_desc& d, uint32_t (&mb)[8],
                                             int64_t rb, int64_t col0, int lane,
                                             int64_t col_hi = -1) {
  const int64_t n = ecol(col0, col_hi < 0 ? col0 + 32 : col_hi, 8 * (lane & 7));
  const int64_t nc = n < d.N ? n : d.N - 8;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    int64_t m = rb + 8 * q + (lane >> 3);
    m = m < d.M ? m : d.M - 1;
    const int64_t mr = d.mask_arows ? d.a_rows[m] : m;
    mb[q] = static_cast<const uint8_t*>(d.mask)[mr * d.ldmask + (nc >> 3)];
  }
}

// the mask rows of one lane in the wide map (rows rb + 8q + lane/8, columns col0 + 8(lane%8))
__device__ __forceinline__ void lp_wide_mask(const savqa_gemm_lp_desc& d, bf16x8 (&mk)[8],
                                             int64_t rb, int64_t col0, int lane,
                                             int64_t col_hi = -1) {
  const int64_t n = ecol(col0, col_hi < 0 ? col0 + 32 : col_hi, 8 * (lane & 7));
  const int64_t nc = n < d.N ? n : d.N - 8;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    int64_t m = rb + 8 * q + (lane >> 3);
    m = m < d.M ? m : d.M - 1;
    const int64_t mr = d.mask_arows ? d.a_rows[m] : m;
    mk[q] = *reinterpret_cast<const bf16x8*>(static_cast<const __bf16*>(d.mask) + mr * d.ldmask + nc);
  }
}

// MK: 0 no mask, 1 bf16 mask values (mk), 2 gate bits (mb); d.bits_out: this output's gate
// bits, one byte per lane and row (computed from the stored bf16 values)
template <int MK>
__device__ __forceinline__ void lp_pass_wide(const savqa_gemm_lp_desc& d, const char* reg,
                                             int64_t rb, int64_t col0, bool first_split,
                                             const bf16x8 (&mk)[8], const uint32_t (&mb)[8],
                                             int lane, int64_t col_hi = -1) {
  const int c8 = lane & 7, r8 = lane >> 3;
  const bool ident = d.c_group <= 0;
  const int64_t n = ecol(col0, col_hi < 0 ? col0 + 32 : col_hi, 8 * c8);
  const bool nok = n < d.N;  // N % 8 == 0: a lane's 8 columns are all in or all out
  const int64_t nc = nok ? n : d.N - 8;
  f4 b0 = {0.f, 0.f, 0.f, 0.f}, b1 = b0;
  if (first_split && d.bias) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      b0[r] = d.bias[nc + r];
      b1[r] = d.bias[nc + 4 + r];
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int lr = 8 * q + r8;
    const int64_t m = rb + lr;
    f4 lo = *reinterpret_cast<const f4*>(reg + lr * 256 + (((2 * c8) ^ (lr & 15)) * 16));
    f4 hi = *reinterpret_cast<const f4*>(reg + lr * 256 + (((2 * c8 + 1) ^ (lr & 15)) * 16));
    lo = lo * d.alpha + b0;
    hi = hi * d.alpha + b1;
    if (d.relu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        lo[r] = fmaxf(lo[r], 0.f);
        hi[r] = fmaxf(hi[r], 0.f);
      }
    }
    if constexpr (MK == 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (!((float)mk[q][r] > 0.f)) lo[r] = 0.f;
        if (!((float)mk[q][4 + r] > 0.f)) hi[r] = 0.f;
      }
    } else if constexpr (MK == 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (!((mb[q] >> r) & 1u)) lo[r] = 0.f;
        if (!((mb[q] >> (4 + r)) & 1u)) hi[r] = 0.f;
      }
    }
    if (m < d.M && nok) {
      int64_t cr = m;
      if (!ident) {
        const uint32_t mu = (uint32_t)m, cg = (uint32_t)d.c_group;
        cr = (int64_t)(mu / cg) * d.c_stride + (int64_t)(mu % cg) + d.c_offset;
      }
      const bf16x4 l = __builtin_convertvector(lo, bf16x4), h = __builtin_convertvector(hi, bf16x4);
      *reinterpret_cast<bf16x8*>(static_cast<__bf16*>(d.Cb) + cr * d.ldcb + n) =
          bf16x8{l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
      if (d.bits_out) {
        uint32_t bits = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          bits |= (uint32_t)((float)l[r] > 0.f) << r;
          bits |= (uint32_t)((float)h[r] > 0.f) << (4 + r);
        }
        d.bits_out[cr * d.ldbits + (n >> 3)] = (uint8_t)bits;
      }
    }
  }
}

// Epilogue of one wave's TM x 64 output tile (savqa_gemm_lp formula), staged through the
// wave's own 16 KB of LDS in passes of 64 rows so that the global traffic is whole rows:
// the swapped-MFMA accumulators (lane: 4 consecutive columns of one row) are written as
// f4s into a [64][64] fp32 image (16-B chunk c of row r at c ^ (r & 15): conflict-free
// for both the writes and the read-back), then read back row-major -- 16 lanes cover one
// row's 256 B, so every epilogue operand load and every store is a 16-B access in full
// lines; atomic outputs read one float per lane so a wave instruction adds 256 contiguous
// bytes (the full-rate shape of global float atomics). The caller has barriered the
// workgroup after its last k-tile read.
template <int I, int N, class F>
__device__ __forceinline__ void lp_static_for(F& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    lp_static_for<I + 1, N>(f);
  }
}

template <int FM, int FN>
__device__ __forceinline__ void lp_epilogue(const savqa_gemm_lp_desc& d, f4 (&acc)[FM][FN],
                                            char* reg, int64_t row0, int64_t col0,
                                            bool first_split, int lane, int64_t rstep = 64,
                                            int64_t col_hi = -1, bool tail_atomic = false) {
  if (col_hi < 0) col_hi = col0 + 32;
  static_assert(FN == 4, "wave tiles are 64 columns wide");
  const int g = lane >> 4;
  const bool ident = d.c_group <= 0;
  const bool vec_c = (d.ldc & 3) == 0 && (((uintptr_t)d.C) & 15) == 0;
  const bool vec_cb = (d.ldcb & 3) == 0 && (((uintptr_t)d.Cb) & 7) == 0;
  // gate bits of every pass, loaded before the first image write (8 registers per pass)
  const bool bits = d.mask && d.mask_type == SAVQA_DT_BITS && !d.atomic && !tail_atomic;
  uint32_t mbits[FM / 4][8];
  if (bits) {
#pragma unroll
    for (int pass = 0; pass < FM / 4; ++pass)
      lp_wide_bits(d, mbits[pass], row0 + rstep * pass, col0, lane, col_hi);
  }
  // passes of 64 rows as a compile-time loop: a runtime pass index would put the
  // accumulators in scratch when the body is too large for the unroller
  auto pass_body = [&](auto pc) {
    constexpr int pass = decltype(pc)::value;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int lr = 16 * i + (lane & 15);
        *reinterpret_cast<f4*>(reg + lr * 256 + (((4 * j + g) ^ (lr & 15)) * 16)) = acc[4 * pass + i][j];
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's image is complete
    __builtin_amdgcn_wave_barrier();
    if (d.atomic || tail_atomic) {
      // one float per lane: row q, column lane (256 contiguous bytes per atomic instruction)
      const int64_t n = ecol(col0, col_hi, lane);
      const float bv = (first_split && d.bias && n < d.N) ? d.bias[n] : 0.f;
      // the pass's output rows (c_rows scatter) and mask rows, lane q holding row q, loaded
      // before the first atomic and broadcast per row: loaded inside the loop, each row's
      // load waited for every atomic before it (vmcnt counts both) -- the GloVe-table
      // scatter paid one atomic round trip per row
      int64_t rowv = 0, mrv = 0;
      {
        int64_t m = row0 + rstep * pass + lane;
        m = m < d.M ? m : d.M - 1;
        if (d.c_rows) rowv = d.c_rows[m];
        if (d.mask && d.mask_arows) mrv = d.a_rows[m];
      }
      auto bcast = [](int64_t v, int q) {
        const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, q);
        const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), q);
        return (int64_t)(((uint64_t)hi << 32) | lo);
      };
      for (int q = 0; q < 64; ++q) {
        const int64_t m = row0 + rstep * pass + q;
        if (m >= d.M) break;
        float v = *reinterpret_cast<const float*>(reg + q * 256 + ((((lane >> 2) ^ (q & 15)) * 16)) +
                                                  (lane & 3) * 4);
        if (n >= d.N || (d.n_store > 0 && n >= d.n_store)) continue;
        v = v * d.alpha + bv;
        if (first_split && d.rowvec) v += d.rowvec[(m % d.rowvec_period) * d.ldrv + n];
        if (d.relu) v = fmaxf(v, 0.f);
        if (d.mask) {
          const int64_t mr = d.mask_arows ? bcast(mrv, q) : m;
          const float mv = d.mask_type == SAVQA_DT_BF16
                               ? bf2f(static_cast<const __bf16*>(d.mask)[mr * d.ldmask + n])
                               : static_cast<const float*>(d.mask)[mr * d.ldmask + n];
          if (!(mv > 0.f)) v = 0.f;
        }
        if (first_split && d.resid) v += d.resid[m * d.ldr + n];
        int64_t cr = m;
        if (d.c_rows) {
          cr = bcast(rowv, q);
        } else if (!ident) {
          const uint32_t mu = (uint32_t)m, cg = (uint32_t)d.c_group;
          cr = (int64_t)(mu / cg) * d.c_stride + (int64_t)(mu % cg) + d.c_offset;
        }
        atomicAdd(d.C + cr * d.ldc + n, v);
      }
    } else if (lp_wide_epilogue(d)) {
      const int64_t rb = row0 + rstep * pass;
      bf16x8 mk[8];
      if (bits) {
        lp_pass_wide<2>(d, reg, rb, col0, first_split, mk, mbits[pass], lane, col_hi);
      } else if (d.mask) {
        lp_wide_mask(d, mk, rb, col0, lane, col_hi);
        lp_pass_wide<1>(d, reg, rb, col0, first_split, mk, mbits[0], lane, col_hi);
      } else {
        lp_pass_wide<0>(d, reg, rb, col0, first_split, mk, mbits[0], lane, col_hi);
      }
    } else if (lp_vec_epilogue(d)) {
      // 16 lanes per row, 4 rows per instruction, groups of G instructions per pass, each
      // group's operand loads issued before its stores
      const int64_t n = ecol(col0, col_hi, 4 * (lane & 15));
      const bool nok = n < d.N;  // N % 4 == 0: a lane's 4 columns are all in or all out
      const int64_t nc = nok ? n : d.N - 4;
      f4 bv = {0.f, 0.f, 0.f, 0.f};
      if (first_split && d.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = d.bias[nc + r];
      }
      const bool res = first_split && d.resid, rv = first_split && d.rowvec;
      const int mk = !d.mask ? 0 : (d.mask_type == SAVQA_DT_BF16 ? 1 : 2);
      const int64_t rb = row0 + rstep * pass;
      // (groups of 4 rows when the wave still holds a second pass of accumulators)
      constexpr int G = FM > 4 ? 4 : 8;
#define SAVQA_ROWS(R_, M_, V_)                                                  \
  for (int h = 0; h < 16 / G; ++h) lp_rows<G, R_, M_, V_>(d, reg, rb, h, n, nok, nc, bv, ident, lane)
      if (rv) {
        SAVQA_ROWS(false, 0, true);   // the input projection: + position table, no mask / resid
      } else if (res) {
        if (mk == 1) SAVQA_ROWS(true, 1, false);
        else if (mk == 2) SAVQA_ROWS(true, 2, false);
        else SAVQA_ROWS(true, 0, false);
      } else {
        if (mk == 1) SAVQA_ROWS(false, 1, false);
        else if (mk == 2) SAVQA_ROWS(false, 2, false);
        else SAVQA_ROWS(false, 0, false);
      }
#undef SAVQA_ROWS
    } else {
      // 16 lanes per row, 4 rows per instruction, 16 instructions per pass
      const int c = lane & 15;
      const int64_t n = ecol(col0, col_hi, 4 * c);
      const bool full = n + 4 <= d.N;
      f4 bv = {0.f, 0.f, 0.f, 0.f};
      if (first_split && d.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = n + r < d.N ? d.bias[n + r] : 0.f;
      }
#pragma unroll 4
      for (int q = 0; q < 16; ++q) {
        const int lr = 4 * q + (lane >> 4);
        const int64_t m = row0 + rstep * pass + lr;
        if (m >= d.M || n >= d.N) continue;
        f4 v = *reinterpret_cast<const f4*>(reg + lr * 256 + ((c ^ (lr & 15)) * 16));
        v = v * d.alpha + bv;
        if (first_split && d.rowvec) {
          const float* rp = d.rowvec + (m % d.rowvec_period) * d.ldrv + n;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += n + r < d.N ? rp[r] : 0.f;
        }
        if (d.relu) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if (d.mask) {
          const int64_t mr = d.mask_arows ? d.a_rows[m] : m;
          f4 mv;
          if (d.mask_type == SAVQA_DT_BF16) {
            const __bf16* mp = static_cast<const __bf16*>(d.mask) + mr * d.ldmask + n;
            if (full && (d.ldmask & 3) == 0 && (((uintptr_t)d.mask) & 7) == 0) {
              mv = __builtin_convertvector(*reinterpret_cast<const bf16x4*>(mp), f4);
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) mv[r] = n + r < d.N ? bf2f(mp[r]) : 0.f;
            }
          } else {
            const float* mp = static_cast<const float*>(d.mask) + mr * d.ldmask + n;
#pragma unroll
            for (int r = 0; r < 4; ++r) mv[r] = n + r < d.N ? mp[r] : 0.f;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (!(mv[r] > 0.f)) v[r] = 0.f;
        }
        if (first_split && d.resid) {
          const float* rp = d.resid + m * d.ldr + n;
          if (full && (d.ldr & 3) == 0 && (((uintptr_t)d.resid) & 15) == 0) {
            v += *reinterpret_cast<const f4*>(rp);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += n + r < d.N ? rp[r] : 0.f;
          }
        }
        int64_t cr = m;
        if (!ident) {
          const uint32_t mu = (uint32_t)m, cg = (uint32_t)d.c_group;
          cr = (int64_t)(mu / cg) * d.c_stride + (int64_t)(mu % cg) + d.c_offset;
        }
        if (d.C) {
          float* cp = d.C + cr * d.ldc + n;
          if (full && vec_c) {
            *reinterpret_cast<f4*>(cp) = v;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < d.N) cp[r] = v[r];
          }
        }
        if (d.Cb) {
          __bf16* cp = static_cast<__bf16*>(d.Cb) + cr * d.ldcb + n;
          const bf16x4 h = __builtin_convertvector(v, bf16x4);
          if (full && vec_cb) {
            *reinterpret_cast<bf16x4*>(cp) = h;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < d.N) cp[r] = h[r];
          }
        }
      }
    }
    if (pass + 1 < FM / 4) {
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
  };
  lp_static_for<0, FM / 4>(pass_body);
}

// Split-K slab epilogue (128 x 128 kernel): the slice's partial tile goes to its own slab
// [slice][M][N] with plain 16-B stores straight from the swapped-MFMA accumulators (lane:
// row 16i + lane % 16, columns 16j + 4 (lane / 16) .. +3); lp_slab_reduce_kernel then adds the
// slices into C. Replaces the fp32 atomics (~1.3 TB/s chip-wide: ~30 % of a cfg-3 dW launch,
// all of it after the last k-tile) with full-rate stores and one pass over the slabs, and
// makes the sum deterministic. Linear epilogue only (host-checked): alpha, and bias / row
// vector / residual on slice 0; N % 4 == 0.
__device__ __forceinline__ void lp_epilogue_slab(const savqa_gemm_lp_desc& d, const f4 (&acc)[4][4],
                                                 int64_t row0, int64_t col0, bool first_split,
                                                 int lane, float* __restrict__ slab,
                                                 int64_t r0 = 0) {
  const int ri = lane & 15, g = lane >> 4;
  f4 bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t n = col0 + 16 * j + 4 * g;
    bv[j] = f4{0.f, 0.f, 0.f, 0.f};
    if (first_split && d.bias && n < d.N) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[j][r] = d.bias[n + r];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = row0 + 16 * i + ri;
    if (m >= d.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = col0 + 16 * j + 4 * g;
      if (n >= d.N) continue;
      f4 v = acc[i][j] * d.alpha + bv[j];
      if (first_split && (d.rowvec || d.resid)) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (d.rowvec) v[r] += d.rowvec[(m % d.rowvec_period) * d.ldrv + n + r];
          if (d.resid) v[r] += d.resid[m * d.ldr + n + r];
        }
      }
      *reinterpret_cast<f4*>(slab + (m - r0) * d.N + n) = v;
    }
  }
}

// C[r0 + m][n] (+)= sum over the ns slabs [ns][rows][N] (fixed order), four columns per thread,
// columns < nst stored (n_store; a multiple of 4); assign: the split-off tail tiles' rows
// (C = sum), else split-K accumulation (C += sum). Blocks from cs_blk0 on add the fused column
// sum's ns partials [ns][cs_n] (cs_slab) into colsum in the same slice order.
__global__ __launch_bounds__(256) void lp_slab_reduce_kernel(const float* __restrict__ slab, int ns,
                                                             int64_t rows, int64_t N, int64_t nst,
                                                             float* __restrict__ C, int64_t ldc,
                                                             int vec, int64_t r0, int assign,
                                                             int64_t cs_blk0,
                                                             const float* __restrict__ cs_slab,
                                                             int64_t cs_n, float* __restrict__ colsum) {
  if ((int64_t)blockIdx.x >= cs_blk0) {
    const int64_t m = ((int64_t)blockIdx.x - cs_blk0) * 256 + threadIdx.x;
    if (m >= cs_n) return;
    float v = cs_slab[m];
    for (int k = 1; k < ns; ++k) v += cs_slab[k * cs_n + m];
    colsum[m] += v;
    return;
  }
  const int64_t n4 = N / 4;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= rows * n4) return;
  const int64_t m = t / n4, n = 4 * (t - m * n4);
  if (n >= nst) return;
  const int64_t plane = rows * N;
  f4 acc = *reinterpret_cast<const f4*>(slab + m * N + n);
  for (int k = 1; k < ns; ++k) acc += *reinterpret_cast<const f4*>(slab + k * plane + m * N + n);
  float* cp = C + (r0 + m) * ldc + n;
  if (vec) {
    f4* c4 = reinterpret_cast<f4*>(cp);
    *c4 = assign ? acc : *c4 + acc;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) cp[r] = assign ? acc[r] : cp[r] + acc[r];
  }
}

// Epilogue operands prefetched under the last k-tile's MFMAs (128 x 128 kernel, one 64-row
// pass per wave): PRE = 1 the fp32 residual (the 16 rows x 4 columns each lane stores,
// lp_rows' map), PRE = 2 the bf16 ReLU-backward mask of a bf16-only output (optionally through
// the A-row gather; lp_pass_wide's map).
// Chosen by the host for non-atomic, unsplit launches in the vector layout with exactly
// that one operand; their loads then overlap the k-loop instead of following it.
// (the residual's second 8 rows are loaded at the start of the epilogue, before any store:
// 16 prefetched f4s beside the accumulators spill)
template <int PRE>
struct LpPre {
  f4 r[PRE == 1 ? 8 : 1];
  bf16x8 m[PRE == 2 ? 8 : 1];
  uint32_t mb[8];  // PRE == 3: the gate bytes (SAVQA_DT_BITS mask), loaded before the k-loop

  __device__ __forceinline__ void load(const savqa_gemm_lp_desc& d, int64_t row0, int64_t col0,
                                       int lane) {
    const int64_t n = col0 + 4 * (lane & 15);
    const int64_t nc = n < d.N ? n : d.N - 4;
    if constexpr (PRE == 1) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        int64_t m = row0 + 4 * q + (lane >> 4);
        m = m < d.M ? m : d.M - 1;
        r[q] = *reinterpret_cast<const f4*>(d.resid + m * d.ldr + nc);
      }
    }
    if constexpr (PRE == 2) lp_wide_mask(d, this->m, row0, col0, lane);
    if constexpr (PRE == 3) lp_wide_bits(d, this->mb, row0, col0, lane);
  }
};

template <int PRE>
__device__ __forceinline__ void lp_epilogue_pre(const savqa_gemm_lp_desc& d, f4 (&acc)[4][4],
                                                char* reg, int64_t row0, int64_t col0,
                                                const LpPre<PRE>& pre, int lane) {
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int lr = 16 * i + (lane & 15);
      *reinterpret_cast<f4*>(reg + lr * 256 + (((4 * j + g) ^ (lr & 15)) * 16)) = acc[i][j];
    }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's image is complete
  __builtin_amdgcn_wave_barrier();
  if constexpr (PRE == 2) {
    lp_pass_wide<1>(d, reg, row0, col0, true, pre.m, pre.mb, lane);
    return;
  }
  if constexpr (PRE == 3) {
    bf16x8 unused[8];
    lp_pass_wide<2>(d, reg, row0, col0, true, unused, pre.mb, lane);
    return;
  }
  const bool ident = d.c_group <= 0;
  const int64_t n = col0 + 4 * c;
  const bool nok = n < d.N;
  const int64_t nc = nok ? n : d.N - 4;
  f4 bv = {0.f, 0.f, 0.f, 0.f};
  if (d.bias) {
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = d.bias[nc + r];
  }
  f4 r2[PRE == 1 ? 8 : 1];
  if constexpr (PRE == 1) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      int64_t m = row0 + 4 * (q + 8) + (lane >> 4);
      m = m < d.M ? m : d.M - 1;
      r2[q] = *reinterpret_cast<const f4*>(d.resid + m * d.ldr + nc);
    }
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int lr = 4 * q + (lane >> 4);
    const int64_t m = row0 + lr;
    f4 v = *reinterpret_cast<const f4*>(reg + lr * 256 + ((c ^ (lr & 15)) * 16));
    v = v * d.alpha + bv;
    if (d.relu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
    }
    if constexpr (PRE == 1) v += q < 8 ? pre.r[q & 7] : r2[q & 7];
    if (m < d.M && nok) {
      int64_t cr = m;
      if (!ident) {
        const uint32_t mu = (uint32_t)m, cg = (uint32_t)d.c_group;
        cr = (int64_t)(mu / cg) * d.c_stride + (int64_t)(mu % cg) + d.c_offset;
      }
      if (d.C) *reinterpret_cast<f4*>(d.C + cr * d.ldc + n) = v;
      if (d.Cb)
        *reinterpret_cast<bf16x4*>(static_cast<__bf16*>(d.Cb) + cr * d.ldcb + n) =
            __builtin_convertvector(v, bf16x4);
    }
  }
}

template <bool AT, bool BT, bool FP8, int PRE>
__global__ __launch_bounds__(LP_NT, LP_OCC) void gemm_lp_kernel(LpArgs args) {
  const savqa_gemm_lp_desc& d = args.d;
  // fp8: + two 1-KB e8m0 scale images [A rows 0..127 | B rows 0..127][4 blocks of 32 k]
  // (+ the L2 prefetch's dummy DMA slots, bf16 only: ONE shared array -- a second __shared__
  // object makes hipcc wait vmcnt(0) before every k-tile's first LDS read)
  constexpr bool PFON = !FP8 && LP_PF > 0;
  __shared__ __attribute__((aligned(1024))) char smem[2 * 2 * LP_IMG + (FP8 ? 2048 : 0) +
                                                      (PFON ? LP_PF_BYTES : 0)];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int t, slice;
  int64_t kbeg, kend;
  // tail-split block (atomic epilogue); the host never pairs a tail split with an epilogue
  // prefetch (PRE), so those instantiations carry no tail code (it cost them 20 % when present)
  const bool tail = PRE == 0 && (int)blockIdx.x >= args.full;
  if (!tail) {
    split_remap(args.full, t, slice);
    kbeg = (int64_t)slice * args.kchunk;
    kend = min(d.K, kbeg + args.kchunk);
  } else {
    const int u = blockIdx.x - args.full;
    slice = u % args.tail_f;
    t = args.tail_t0 + u / args.tail_f;
    kbeg = (int64_t)slice * args.tail_kchunk;
    kend = min(d.K, kbeg + args.tail_kchunk);
  }
  const int tn = t % args.tiles_n, tm = t / args.tiles_n;
  const int64_t m0 = (int64_t)tm * LP_TILE, n0 = (int64_t)tn * LP_TILE;
  constexpr int BKE = FP8 ? 128 : 64;  // k elements per k-tile
  const int nt = (int)((kend - kbeg + BKE - 1) / BKE);
  const int krem = (int)(kend - kbeg - (int64_t)(nt - 1) * BKE);  // k of the last k-tile
  const bool first_split = slice == 0;
  const int esz = FP8 ? 1 : 2;

  LpStage<AT, FP8> sa;
  LpStage<!BT, FP8> sb;
  sa.setup(d.A, d.lda, esz, AT ? nullptr : d.a_rows, m0, d.M, kbeg, wave, lane);
  sb.setup(d.B, d.ldb, esz, nullptr, n0, d.N, kbeg, wave, lane);
  LpPf pf;
  if constexpr (PFON) {
    const int q = 64 * (wave & 1) + lane;
    if (wave < 2) pf.setup<AT>(d.A, d.lda, esz, AT ? nullptr : d.a_rows, m0, d.M, kbeg, d.K, q);
    else pf.setup<!BT>(d.B, d.ldb, esz, nullptr, n0, d.N, kbeg, d.K, q);
  }
  lds_void* const pf_dummy = (lds_void*)(smem + 2 * 2 * LP_IMG + 256 * wave);

  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  LpPre<PRE> pre;
  if constexpr (PRE != 0) {  // (the gate bytes cost 8 registers: loaded before the k-loop)
    if ((nt == 0 || PRE == 3) && !tail) pre.load(d, m0 + wm * 64, n0 + wn * 64, lane);
  }
  // fused bias gradient (savqa_gemm_lp_desc.colsum_a, dW launches): the first column tile of
  // each row block also sums its staged A^T tiles over k, thread (rg, cg) four k rows of 8
  // columns per k-tile (zero-filled past K), folded across the 16 row groups at the end
  const bool do_cs = AT && !FP8 && d.colsum_a != nullptr && tn == 0;
  float cs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = 0.f;

  // fp8 block scales: staged by LDS-DMA with the operand tiles (one 4-byte granule per lane:
  // the 4 blocks of 32 k of one row in a k-tile; wave w stages A rows (w < 2) or B rows
  // 64 (w & 1) + lane), so the k-loop carries no ordinary global loads. Scales loaded into
  // VGPRs per k-tile (8 byte loads per lane, the a_rows gather resolved inside the loop) left
  // the fp8 kernel slower per FLOP than the bf16 one (profiles/r02_lp_diag.txt).
  const uint8_t* scp = nullptr;
  if constexpr (FP8) {
    const int r = 64 * (wave & 1) + lane;
    if (wave < 2) {
      int64_t m = m0 + r;
      m = m < d.M ? m : d.M - 1;
      const int64_t rr = d.a_rows ? d.a_rows[m] : m;
      scp = d.a_scale + rr * d.lds_a + (kbeg >> 5);
    } else {
      int64_t n = n0 + r;
      n = n < d.N ? n : d.N - 1;
      scp = d.b_scale + n * d.lds_b + (kbeg >> 5);
    }
  }
  char* const sc_img = smem + 2 * 2 * LP_IMG;  // fp8 only: [buffer][A 512 B | B 512 B]
  auto stage_scales = [&](int buf, int64_t kt) {
    if constexpr (FP8)
      glds_k<4>(scp + kt * 4, (lds_void*)(sc_img + buf * 1024 + wave * 256));
  };
  int sca[4], scb[4];
  auto read_scales = [&](int buf) {
    if constexpr (FP8) {
      const int g = lane >> 4;
      const uint8_t* si = reinterpret_cast<const uint8_t*>(sc_img + buf * 1024);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sca[i] = si[(wm * 64 + 16 * i + (lane & 15)) * 4 + g];
        scb[i] = si[512 + (wn * 64 + 16 * i + (lane & 15)) * 4 + g];
      }
    }
  };

  auto stage = [&](char* img, int64_t kt) {
    if (kt + 1 == nt && krem < BKE) {
      sa.issue_tail(img, wave, kt, krem);
      sb.issue_tail(img + LP_IMG, wave, kt, krem);
    } else {
      sa.issue(img, wave, kt);
      sb.issue(img + LP_IMG, wave, kt);
    }
  };
  if (nt > 0) {
    stage(smem, 0);
    stage_scales(0, 0);
    lp_wait_vm<0>();  // (asm DMAs: __syncthreads() does not wait for them)
    __syncthreads();  // stage 0 landed for every wave
    for (int kt = 0; kt < nt; ++kt) {
      const char* ia = smem + (kt & 1) * 2 * LP_IMG;
      const char* ib = ia + LP_IMG;
      read_scales(kt & 1);
      if (kt + 1 < nt) {  // next k-tile into the other buffer (read one barrier ago)
        stage(smem + ((kt + 1) & 1) * 2 * LP_IMG, kt + 1);
        stage_scales((kt + 1) & 1, kt + 1);
      } else if constexpr (PRE == 1 || PRE == 2) {  // last k-tile: epilogue operands under its MFMAs
        if (!tail) pre.load(d, m0 + wm * 64, n0 + wn * 64, lane);
      }
      const bool pf_now = PFON && kt + 1 + LP_PF < nt;  // (uniform)
      if constexpr (PFON) {
        if (pf_now) pf.issue(kt + 1 + LP_PF, pf_dummy);
      }
      if constexpr (FP8) {
        i32x8 a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = frag_fp8(ia, wm * 64 + 16 * i, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = frag_fp8(ib, wn * 64 + 16 * j, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                b[j], a[i], acc[i][j], 0, 0, 0, scb[j], 0, sca[i]);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          bf16x8 a[4], b[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) a[i] = frag_bf16<AT>(ia, wm * 64 + 16 * i, kk, lane);
#pragma unroll
          for (int j = 0; j < 4; ++j) b[j] = frag_bf16<!BT>(ib, wn * 64 + 16 * j, kk, lane);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
        }
        if constexpr (AT) {
          if (do_cs) {  // block-uniform
            const int cg = threadIdx.x & 15, rg = threadIdx.x >> 4;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int r = 4 * rg + q;
              const bf16x8 v = *reinterpret_cast<const bf16x8*>(ia + r * 256 + ((16 * cg) ^ (32 * th(r))));
#pragma unroll
              for (int e = 0; e < 8; ++e) cs[e] += (float)v[e];
            }
          }
        }
      }
      // k-tile kt+1 landed (everything but the newest prefetch), this wave's LDS reads of
      // buffer kt done; then the barrier: buffer kt free for k-tile kt+2
      if (pf_now) lp_wait_vm<1>();
      else lp_wait_vm<0>();
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
    }
  }

  // ---------------------------------------------------------------- epilogue
  __syncthreads();  // every wave's last k-tile reads are done: LDS is free
  if constexpr (AT && !FP8) {
    if (do_cs) {  // block-uniform: fold the 16 row groups, one atomic per column
      float* red = reinterpret_cast<float*>(smem);  // [16 row groups][128 columns]
      const int cg = threadIdx.x & 15, rg = threadIdx.x >> 4;
      *reinterpret_cast<f4*>(&red[rg * 128 + 8 * cg]) = f4{cs[0], cs[1], cs[2], cs[3]};
      *reinterpret_cast<f4*>(&red[rg * 128 + 8 * cg + 4]) = f4{cs[4], cs[5], cs[6], cs[7]};
      __syncthreads();
      if (threadIdx.x < 128 && m0 + threadIdx.x < d.M) {
        float v = 0.f;
#pragma unroll
        for (int g = 0; g < 16; ++g) v += red[g * 128 + threadIdx.x];
        if (args.cs_slab && !tail)  // (block-uniform) added in slice order by the slab reduce
          args.cs_slab[(int64_t)slice * d.M + m0 + threadIdx.x] = v;
        else
          atomicAdd(&d.colsum_a[m0 + threadIdx.x], v);
      }
      __syncthreads();  // the epilogue reuses the LDS
    }
  }
  if (PRE == 0 && !FP8 && args.slab && !tail)
    lp_epilogue_slab(d, acc, m0 + wm * 64, n0 + wn * 64, first_split, lane,
                     args.slab + (int64_t)slice * d.M * d.N);
  else if (tail && args.tail_slab)
    lp_epilogue_slab(d, acc, m0 + wm * 64, n0 + wn * 64, first_split, lane,
                     args.tail_slab + (int64_t)slice * (d.M - args.tail_r0) * d.N, args.tail_r0);
  else if (tail)
    lp_epilogue<4, 4>(d, acc, smem + wave * 16384, m0 + wm * 64, n0 + wn * 64, first_split, lane,
                      64, -1, true);
  else if constexpr (PRE != 0)
    lp_epilogue_pre<PRE>(d, acc, smem + wave * 16384, m0 + wm * 64, n0 + wn * 64, pre, lane);
  else
    lp_epilogue<4, 4>(d, acc, smem + wave * 16384, m0 + wm * 64, n0 + wn * 64, first_split, lane);
}

// ---------------------------------------------------------------------------------------
// Large-tile bf16 variants, one 512-thread workgroup (8 waves) per CU:
//   BM x BN = 256 x 256 (waves 2 x 4, 128 x 64 each) or 256 x 128 (waves 4 x 2, 64 x 64),
//   k-tile BK = 32 or 64 bf16 (64-B / 128-B operand rows), an NS-slot LDS-DMA ring
//   (NS = 2: k-tile t+1 in flight while t is computed; NS = 3: t+1 and t+2), counted
//   `s_waitcnt vmcnt` + raw s_barrier once per k-tile, so with NS = 3 a k-tile's DMAs stay
//   in flight across the barrier (cdna_hip_programming.md "Pipelining across barriers").
//   The slot refilled at iteration t was last read in iteration t-1, before the barrier
//   that ended it.
//   R image: [rows][2*BK B], 16-B chunk c of row r at c ^ swz(r): r & 7 for 128-B rows,
//     (r ^ (r >> 1)) & 3 for 64-B rows (both conflict-free for the fragment reads);
//   T image: [BK k rows][cols] bf16, byte b of row r at b ^ 32 h(r) (as above).
template <int BK>
__device__ __forceinline__ int rswz2(int r) {
  return BK == 64 ? (r & 7) : ((r ^ (r >> 1)) & 3);
}

// LDS-DMA sources of one operand tile of R rows (R image) / R columns (T image).
template <bool T, int R, int BK>
struct Lp2Stage {
  static constexpr int INS = R * BK * 2 / 1024 / 8;  // glds per wave per k-tile
  const char* p[INS];
  int koff[INS];  // k of this lane's granule within a k-tile
  int64_t step;

  __device__ __forceinline__ void setup(const __bf16* base, int64_t ld,
                                        const int64_t* __restrict__ rows, int64_t r0, int64_t lim,
                                        int64_t kbeg, int wave, int lane) {
#pragma unroll
    for (int u = 0; u < INS; ++u) {
      const int ins = INS * wave + u;
      if constexpr (!T) {
        constexpr int CPR = BK * 2 / 16, RPI = 64 / CPR;  // chunks per row, rows per instruction
        const int r = RPI * ins + lane / CPR;
        const int lc = (lane % CPR) ^ rswz2<BK>(r);
        int64_t m = r0 + r;
        m = m < lim ? m : lim - 1;
        const int64_t rr = rows ? rows[m] : m;
        p[u] = reinterpret_cast<const char*>(base + rr * ld + kbeg + lc * 8);
        koff[u] = lc * 8;
      } else {
        constexpr int CPR = 2 * R / 16, RPI = 64 / CPR;
        const int r = RPI * ins + lane / CPR;
        const int lc = (lane % CPR) ^ (2 * th(r));
        int64_t c = r0 + lc * 8;
        c = c + 8 <= lim ? c : lim - 8;
        p[u] = reinterpret_cast<const char*>(base + (kbeg + r) * ld + c);
        koff[u] = r;
      }
    }
    step = T ? (int64_t)BK * ld * 2 : BK * 2;
  }

  __device__ __forceinline__ void issue(char* img, int wave, int64_t t) const {
#pragma unroll
    for (int u = 0; u < INS; ++u)
      glds16(p[u] + t * step, (lds_void*)(img + (INS * wave + u) * 1024));
  }

  __device__ __forceinline__ void issue_tail(char* img, int wave, int64_t t, int krem) const {
#pragma unroll
    for (int u = 0; u < INS; ++u)
      glds16(koff[u] < krem ? (const void*)(p[u] + t * step) : (const void*)g_lp_zero,
             (lds_void*)(img + (INS * wave + u) * 1024));
  }
};

// fragment: 16 rows (R image) / 16 columns (T image) x k 32kk + 8g .. +7
template <bool T, int R, int BK>
__device__ __forceinline__ bf16x8 frag2(const char* img, int base, int kk, int lane) {
  const int g = lane >> 4;
  if constexpr (!T) {
    const int r = base + (lane & 15);
    return *reinterpret_cast<const bf16x8*>(img + r * (2 * BK) + ((4 * kk + g) ^ rswz2<BK>(r)) * 16);
  } else {
    const int q = (lane & 15) >> 2, p = lane & 3;
    const int r1 = 32 * kk + 8 * g + q, r2 = r1 + 4;
    const int cb = (base + 4 * p) * 2;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(img + r1 * (2 * R) + (cb ^ (32 * th(r1)))));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) bf16x4*)(img + r2 * (2 * R) + (cb ^ (32 * th(r2)))));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int WM, int BK, int NS, bool AT, bool BT>
__global__ __launch_bounds__(512, 1) void gemm_lp2_kernel(LpArgs args) {
  constexpr int WN = 8 / WM;
  constexpr int TM = BM / WM, TN = BN / WN;  // wave tile
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int IMG_A = BM * BK * 2, IMG_B = BN * BK * 2;
  constexpr int STAGE = IMG_A + IMG_B;
  static_assert(NS * STAGE <= 160 * 1024, "LDS");
  const savqa_gemm_lp_desc& d = args.d;
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  int t, slice;
  split_remap(args.nblk, t, slice);
  const int tn = t % args.tiles_n, tm = t / args.tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)slice * args.kchunk;
  const int64_t kend = min(d.K, kbeg + args.kchunk);
  const int nt = (int)((kend - kbeg + BK - 1) / BK);
  const int krem = (int)(kend - kbeg - (int64_t)(nt - 1) * BK);  // k of the last k-tile
  const bool first_split = slice == 0;

  Lp2Stage<AT, BM, BK> sa;
  Lp2Stage<!BT, BN, BK> sb;
  sa.setup(static_cast<const __bf16*>(d.A), d.lda, AT ? nullptr : d.a_rows, m0, d.M, kbeg, wave, lane);
  sb.setup(static_cast<const __bf16*>(d.B), d.ldb, nullptr, n0, d.N, kbeg, wave, lane);
  constexpr int PER_TILE = Lp2Stage<AT, BM, BK>::INS + Lp2Stage<!BT, BN, BK>::INS;

  f4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](char* img, int64_t kt) {
    if (kt + 1 == nt && krem < BK) {
      sa.issue_tail(img, wave, kt, krem);
      sb.issue_tail(img + IMG_A, wave, kt, krem);
    } else {
      sa.issue(img, wave, kt);
      sb.issue(img + IMG_A, wave, kt);
    }
  };
  if (nt > 0) {
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
      if (s < nt) stage(smem + s * STAGE, s);
    if (NS == 3 && nt > 1) wait_vm<PER_TILE>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    int cur = 0;
    for (int kt = 0; kt < nt; ++kt) {
      const char* ia = smem + cur * STAGE;
      const char* ib = ia + IMG_A;
      const int nxt = kt + NS - 1;
      if (nxt < nt && lp_dbg(args) != 2) {  // into slot nxt % NS, last read in iteration kt-1
        const int sl = cur == 0 ? NS - 1 : cur - 1;
        stage(smem + sl * STAGE, nxt);
      }
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        if (lp_dbg(args) == 1) break;
        bf16x8 a[FM], b[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = frag2<AT, BM, BK>(ia, wm * TM + 16 * i, kk, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) b[j] = frag2<!BT, BN, BK>(ib, wn * TN + 16 * j, kk, lane);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      }
      if (kt + 1 < nt) {  // k-tile kt+1 landed; with NS = 3 the DMAs of kt+2 stay in flight
        if (NS == 3 && kt + 2 < nt) wait_vm<PER_TILE>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
      }
      cur = cur == NS - 1 ? 0 : cur + 1;
    }
  }

  // ---------------------------------------------------------------- epilogue
  static_assert(NS * STAGE >= 8 * 16384, "epilogue images need 16 KB per wave");
  __syncthreads();  // every wave's last k-tile reads are done: LDS is free
  lp_epilogue<FM, FN>(d, acc, smem + wave * 16384, m0 + wm * TM, n0 + wn * TN, first_split, lane);
}

// ---------------------------------------------------------------------------------------
// 256 x 256 bf16 tile in the 8-phase structure (cdna_hip_programming.md "The 256^2 8-phase
// template"): 512 threads = 8 waves, one workgroup per CU, k-tile 64, two LDS buffers of four
// 16-KB half images each (A rows 0-127 / 128-255, B columns 0-127 / 128-255; every half image
// has the format of the 128 x 128 kernel's operand image, so the fragment reads are shared).
// A k-tile is 4 phases; phase q computes block quadrant (i, j) = (0,0), (0,1), (1,1), (1,0) --
// each wave a 64 x 32 piece of it (rows wm*64 of A half i, columns wn*32 of B half j), 16
// MFMAs -- so a phase reads ONE A half and ONE B half, and consecutive phases share a
// register subtile (phase 0 reads A(0) + B(0), 1 B(1), 2 A(1), 3 B(0)). Each phase also
// LDS-DMAs one half of the NEXT k-tile in the order A0, B0, B1, A1, i.e. the order the next
// k-tile's phases first read them, and waits (counted vmcnt) only for the half the next
// phase reads: two halves stay in flight across every barrier. Per phase: subtile ds_reads,
// one half-tile DMA, vmcnt, barrier, lgkmcnt(0), 16 MFMAs at raised priority, barrier.
// RAW: a half is read one phase after the wait that retired it; WAR: a half is restaged
// >= 1 phase (and an lgkmcnt(0)) after its last read in the previous k-tile -- both also
// hold with the two wave rows staggered by one barrier (the row behind waits for its part of
// a half before the barrier the row ahead reads after; it retires its last reads of a half
// before the barrier after which the row ahead restages it).
template <bool T>
struct LpHalf {
  const char* p[2];
  int koff[2];
  int64_t step;

  __device__ __forceinline__ void setup(const void* base, int64_t ld,
                                        const int64_t* __restrict__ rows, int64_t r0, int64_t lim,
                                        int64_t kbeg, int wave, int lane) {
    const char* b = static_cast<const char*>(base);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ins = 2 * wave + u;  // 16 instructions x 1 KB = one 16-KB half image
      if constexpr (!T) {
        const int r = 8 * ins + (lane >> 3);
        const int lc = (lane & 7) ^ rswz<false>(r);
        int64_t m = r0 + r;
        m = m < lim ? m : lim - 1;
        const int64_t rr = rows ? rows[m] : m;
        p[u] = b + (rr * ld + kbeg) * 2 + lc * 16;
        koff[u] = lc * 8;
      } else {
        const int r = 4 * ins + (lane >> 4);
        const int lc = (lane & 15) ^ (2 * th(r));
        int64_t c = r0 + lc * 8;
        c = c + 8 <= lim ? c : lim - 8;
        p[u] = b + ((kbeg + r) * ld + c) * 2;
        koff[u] = r;
      }
    }
    step = T ? (int64_t)64 * ld * 2 : LP_KB;
  }

  __device__ __forceinline__ void issue(char* img, int wave, int64_t t, int krem) const {
#pragma unroll
    for (int u = 0; u < 2; ++u)
      glds_k<16>(krem >= 64 || koff[u] < krem ? (const void*)(p[u] + t * step) : (const void*)g_lp_zero,
             (lds_void*)(img + (2 * wave + u) * 1024));
  }
};

template <bool AT, bool BT>
__global__ __launch_bounds__(512, 1) void gemm_lp3_kernel(LpArgs args) {
  const savqa_gemm_lp_desc& d = args.d;
  __shared__ __attribute__((aligned(1024))) char smem[8 * LP_IMG];  // 2 x {A0, A1, B0, B1}
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  int t, slice;
  split_remap(args.nblk, t, slice);
  const int tn = t % args.tiles_n, tm = t / args.tiles_n;
  const int64_t m0 = (int64_t)tm * 256, n0 = (int64_t)tn * 256;
  const int64_t kbeg = (int64_t)slice * args.kchunk;
  const int64_t kend = min(d.K, kbeg + args.kchunk);
  const int nt = (int)((kend - kbeg + 63) / 64);
  const int krem = (int)(kend - kbeg - (int64_t)(nt - 1) * 64);  // k of the last k-tile
  const bool first_split = slice == 0;

  LpHalf<AT> sa[2];
  LpHalf<!BT> sb[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    sa[h].setup(d.A, d.lda, AT ? nullptr : d.a_rows, m0 + 128 * h, d.M, kbeg, wave, lane);
    sb[h].setup(d.B, d.ldb, nullptr, n0 + 128 * h, d.N, kbeg, wave, lane);
  }
  // half image slots within a buffer: A0 0, A1 1, B0 2, B1 3; DMA order A0, B0, B1, A1
  auto stage = [&](int q, int buf, int64_t kt) {
    const int kr = kt + 1 == nt ? krem : 64;
    char* base = smem + buf * 4 * LP_IMG;
    if (q == 0) sa[0].issue(base + 0 * LP_IMG, wave, kt, kr);
    else if (q == 1) sb[0].issue(base + 2 * LP_IMG, wave, kt, kr);
    else if (q == 2) sb[1].issue(base + 3 * LP_IMG, wave, kt, kr);
    else sa[1].issue(base + 1 * LP_IMG, wave, kt, kr);
  };

  f4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  if (nt > 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) stage(q, 0, 0);
    wait_vm<4>();  // A0 and B0 of k-tile 0 landed (B1, A1 in flight)
    __builtin_amdgcn_s_barrier();
    // the two wave rows run one barrier apart, so on every SIMD one wave issues its MFMAs
    // while the other reads its next subtile (each barrier interval: reads | MFMAs)
    if (wm == 1) __builtin_amdgcn_s_barrier();
    bf16x8 a[4][2], b[2][2];
    for (int kt = 0; kt < nt; ++kt) {
      const char* img = smem + (kt & 1) * 4 * LP_IMG;
      const bool pf = kt + 1 < nt;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = (q == 0 || q == 1) ? 0 : 1;
        const int j = (q == 0 || q == 3) ? 0 : 1;
        if (q == 0 || q == 2) {
#pragma unroll
          for (int fi = 0; fi < 4; ++fi)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
              a[fi][kk] = frag_bf16<AT>(img + i * LP_IMG, wm * 64 + 16 * fi, kk, lane);
        }
        if (q != 2) {
#pragma unroll
          for (int fj = 0; fj < 2; ++fj)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
              b[fj][kk] = frag_bf16<!BT>(img + (2 + j) * LP_IMG, wn * 32 + 16 * fj, kk, lane);
        }
        if (pf && !(lp_dbg(args) & 2)) {
          stage(q, (kt + 1) & 1, kt + 1);
          wait_vm<4>();  // the half the next phase reads has landed
        } else {
          wait_vm<0>();
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this phase's subtile is in VGPRs
        __builtin_amdgcn_s_setprio(1);
        if (!(lp_dbg(args) & 1)) {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int fi = 0; fi < 4; ++fi)
#pragma unroll
              for (int fj = 0; fj < 2; ++fj)
                acc[4 * i + fi][2 * j + fj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    b[fj][kk], a[fi][kk], acc[4 * i + fi][2 * j + fj], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
      }
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();  // re-align the staggered rows
  }

  // ---------------------------------------------------------------- epilogue
  // (every DMA retired in the last k-tile; its last phase ended with a barrier after the
  // final ds_reads were waited for, so LDS is free)
  __syncthreads();
  if (lp_dbg(args) & 4) {  // diagnostics: no epilogue (one store keeps the k-loop alive)
    if (acc[0][0][0] == 12345.f && d.C) d.C[0] = acc[7][3][3];
    return;
  }
  lp_epilogue<8, 4>(d, acc, smem + wave * 16384, m0 + wm * 64, n0 + wn * 32, first_split, lane,
                    128, n0 + 128 + wn * 32);
}

static int lp_slots() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 512;
  if (!cached[dev]) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    cached[dev] = LP_OCC * cus;
  }
  return cached[dev];
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// constraint check (savqa_gemm_lp_supported); msg receives the first violation
static bool lp_ok(const savqa_gemm_lp_desc& d, const char** msg) {
  auto no = [&](const char* m) { *msg = m; return false; };
  if (d.M < 0 || d.N < 0 || d.K < 0) return no("negative dims");
  if (d.M >= (1LL << 31) || d.N >= (1LL << 31)) return no("M/N >= 2^31");
  if (!d.A || !d.B) return no("null operand");
  if (!d.C && !d.Cb) return no("no output");
  const bool fp8 = d.a_type == SAVQA_DT_FP8;
  if (d.a_type != d.b_type) return no("a_type != b_type");
  if (!fp8 && d.a_type != SAVQA_DT_BF16) return no("operand type must be bf16 or fp8");
  if (d.atomic && d.Cb) return no("bf16 output with atomic accumulation");
  if ((d.c_rows || d.n_store > 0) && !d.atomic) return no("c_rows / n_store need atomic = 1");
  if ((d.split_k > 1 || d.split_k < 0) && (!d.atomic || !d.C)) return no("split-K needs atomic fp32 C");
  if (d.a_rows && d.a_trans) return no("a_rows needs a_trans = 0");
  if (d.colsum_a && (!d.a_trans || fp8)) return no("colsum_a needs a_trans = 1 and bf16 operands");
  if (d.mask && d.mask_arows && !d.a_rows) return no("mask_arows needs a_rows");
  if (d.mask && d.mask_type != SAVQA_DT_BF16 && d.mask_type != SAVQA_DT_F32 &&
      d.mask_type != SAVQA_DT_BITS)
    return no("mask_type");
  if (((d.mask && d.mask_type == SAVQA_DT_BITS) || d.bits_out) && !lp_wide_epilogue(d))
    return no("bit masks / bits_out need a bf16-only output (Cb, N % 8 == 0, no C / resid / "
              "rowvec / atomic)");
  if (d.bits_out && d.ldbits < (d.N + 7) / 8) return no("ldbits < N / 8");
  if (d.rowvec && d.rowvec_period <= 0) return no("rowvec_period");
  if (!al16(d.A) || !al16(d.B)) return no("operands must be 16-B aligned");
  if (fp8) {
    if (d.a_trans || !d.b_trans) return no("fp8 needs a_trans = 0, b_trans = 1");
    if (d.K % 128) return no("fp8 needs K % 128 == 0");
    if (d.lda % 16 || d.ldb % 16) return no("fp8 needs ld % 16 == 0");
    if (!d.a_scale || !d.b_scale) return no("fp8 needs block scales");
    if ((d.lds_a % 4) || (d.lds_b % 4) || ((uintptr_t)d.a_scale & 3) || ((uintptr_t)d.b_scale & 3))
      return no("fp8 needs 4-byte aligned scale rows (lds % 4 == 0)");
  } else {
    // 16-B granules run along k only in k-contiguous (R image) operands
    if (d.K % 8 && (!d.a_trans || d.b_trans)) return no("bf16 needs K % 8 == 0");
    if (d.lda % 8 || d.ldb % 8) return no("bf16 needs ld % 8 == 0");
    if (d.a_trans && d.M % 8) return no("a_trans needs M % 8 == 0");
    if (!d.b_trans && d.N % 8) return no("b_trans = 0 needs N % 8 == 0");
  }
  return true;
}

// Launch plan of a supported descriptor: kernel variant (1 = 128x128, two workgroups per
// CU; 3 = 256x256 BK64 NS2, 4 = 256x128 BK64 NS3 -- one per CU), split-K factor, tiles.
struct LpPlan {
  int var, split, nsplit;
  int64_t tiles, per;
  int bn;
  int pre;  // gemm_lp_kernel's epilogue-operand prefetch (LpPre): 0 none, 1 resid, 2 bf16 mask,
            // 3 gate bits
  // tail split (variant 1, unsplit): tiles [tail_t0, tiles) in tail_f k-slices, rows
  // [zero_row0, M) of C zero-filled first; tail_f = 1: none
  int tail_f;
  int64_t tail_t0, tail_per, zero_row0;
  bool tail_slab;  // the tail slices store partial slabs (d.ws) instead of adding atomically
};

// tail splits need >= 64 k-tiles: with atomic adds into a zero-filled C the epilogue and the
// fill cost a third of a K = 512 launch (K = 2048 shapes were 20-40 % slower); with partial
// slabs and one ordered reduce (deterministic, no fill) K = 2048 / 1536 shapes were 0-6 %
// slower and cfg 3 1.2 % (tools/lp_bench.py, interleaved), K = 6144 7 % faster than atomics
#ifndef SAVQA_LP_TAIL_MIN_NK_SLAB
#define SAVQA_LP_TAIL_MIN_NK_SLAB 64
#endif
constexpr int LP_TAIL_MIN_NK = 64, LP_TAIL_MIN_NK_SLAB = SAVQA_LP_TAIL_MIN_NK_SLAB;
constexpr int LP_TAIL_MIN_NK_PLAN = 64;  // (bf16 k-tiles) the 256 x 256 round rule's K bound
#ifndef SAVQA_LP3_ROUND_COST
#define SAVQA_LP3_ROUND_COST 17  // one 256 x 256 round in tenths of a 128 x 128 round
#endif
static bool lp_al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static LpPlan lp_plan(const savqa_gemm_lp_desc& d) {
  LpPlan p{};
  const bool fp8 = d.a_type == SAVQA_DT_FP8;
  // kernel: variants of gemm_lp2_kernel (bf16, one workgroup per CU) when there are enough
  // tiles to fill the chip, else the 128 x 128 kernel (two per CU); d.tile_hint selects one
  // explicitly (tests / tuning): 1 = 128x128, 3 = 256x256 BK64 NS2, 4 = 256x128 BK64 NS3
  // (k-tile 32 with a three-slot ring measured slower: 64-B rows halve each DMA's lines)
  // measured (tools/lp_bench.py --variants, cfg-3 shapes): the two-per-CU 128 x 128 kernel is
  // fastest except for the very wide outputs (N = 6144 forward, M = 6144 split-K dW) and the
  // wide dX of the FFN (NN, N = 2048), where the 8-phase 256 x 256 kernel (5) wins by 1-11%
  // (the NS2 256 x 256 kernel (3) by ~10% over 128 x 128 on the first two). Diagnostic builds
  // of kernel 5 (tile_hint bits 8-10: no MFMA / no k-loop DMA / no epilogue) at the K = 512
  // shapes: the epilogue's HBM writes are ~30% of a launch and are not overlapped (one
  // workgroup per CU), which is why the two-per-CU kernel stays ahead there.
  p.var = 1;
  if (!fp8) {
    const bool split = d.split_k > 1 || d.split_k < 0;
    const int h = d.tile_hint & 255;
    // (round 5, tools/lp_bench.py --variants: the 128 x 128 kernel with split-K slabs beats the
    // 256 x 256 one with atomics on the M = 6144 dW, 322 vs 344 us; the 256 x 256 kernel wins
    // the N = 2048 forward too, 104 vs 109 us)
    const bool slab_dw = split && d.ws && !d.mask && !d.relu && !d.Cb && d.N % 4 == 0;
    if (h == 1 || h == 3 || h == 4 || h == 5) p.var = h;
    else if (d.N >= 4096 || (split && d.a_trans && d.M >= 4096 && d.N >= 256 && !slab_dw) ||
             (!d.a_trans && d.N >= 2048 && d.M >= 8192))
      p.var = 5;
    else if (!split && !d.a_trans && !d.c_rows && (d.K + 63) / 64 < LP_TAIL_MIN_NK_PLAN) {
      // Round 6, with both kernels' LDS-DMAs pipelined (glds_asm): by the rounds each takes
      // (2 x CUs 128 x 128 slots, CUs 256 x 256 slots), the 8-phase kernel wins once
      // 1.7 x its rounds < the 128 x 128 kernel's -- one of its rounds costs ~1.7 of the
      // other's at these K (tools/gemm_replay.py --hints 1,5 on the cfg-3 launches, cold:
      // NN 25600x512x2048 116 -> 98 us, NT 92160x1024x304 176 -> 146, NT 37376x1536x512
      // 112 -> 98; NN 37376x512x2048 stays 128 x 128, 158 vs 175). Long K keeps the
      // 128 x 128 kernel and its tail split.
      const int64_t t1 = ((d.M + 127) / 128) * ((d.N + 127) / 128);
      const int64_t t3 = ((d.M + 255) / 256) * ((d.N + 255) / 256);
      const int64_t s1 = lp_slots(), s3 = std::max(1, lp_slots() / LP_OCC);
      const int64_t r1 = (t1 + s1 - 1) / s1, r3 = (t3 + s3 - 1) / s3;
      if (SAVQA_LP3_ROUND_COST * r3 < 10 * r1) p.var = 5;
    }
  }
  const int bm = p.var == 1 ? 128 : 256;
  p.bn = (p.var == 3 || p.var == 5) ? 256 : 128;
  const int bk = fp8 ? 128 : 64;
  const int slots = p.var == 1 ? lp_slots() : lp_slots() / LP_OCC;
  p.tiles = ((d.M + bm - 1) / bm) * ((d.N + p.bn - 1) / p.bn);
  const int64_t nk = (d.K + bk - 1) / bk;
  p.split = d.split_k > 1 ? d.split_k : 1;
  if (d.split_k < 0) {  // minimise rounds(s) * (k-tiles per slice + per-block overhead)
    int64_t best_cost = INT64_MAX;
    for (int s = 1; s <= 64 && (s == 1 || nk / s >= 4); ++s) {
      const int64_t rounds = (p.tiles * s + slots - 1) / slots;
      const int64_t cost = rounds * ((nk + s - 1) / s + 3);
      if (cost < best_cost) { best_cost = cost; p.split = s; }
    }
  }
  p.per = (nk + p.split - 1) / p.split;
  p.nsplit = nk > 0 ? (int)((nk + p.per - 1) / p.per) : 1;
  // epilogue operand prefetched under the last k-tile (LpPre): one residual or one bf16
  // mask, nothing else to load, whole tiles (no split), vector layout
  p.pre = 0;
  if (p.var == 1 && !fp8 && p.nsplit == 1 && !d.atomic && !d.rowvec && lp_vec_epilogue(d)) {
    if (d.resid && !d.mask) p.pre = 1;
    else if (d.mask && lp_wide_epilogue(d)) p.pre = d.mask_type == SAVQA_DT_BITS ? 3 : 2;
  }
  // Tail split (as savqa_gemm's): the tiles of the last, partial round of workgroups are split
  // over K (zero-filled C, atomic fp32 adds, bias / residual / row vector on slice 0) so that
  // they spread over all CUs instead of leaving most of them idle for a whole tile. Needs a
  // linear epilogue into fp32 C only (no ReLU, no bf16 copy), identity row map, and C not
  // overlapping the residual. Only for long K (>= 64 k-tiles): the atomic epilogue costs about
  // a third of a K = 512 launch (diagnostic builds), and with the zero-fill it made the K = 2048
  // step shapes 20-40 % slower (tools/lp_bench.py); at K = 6144 (dX of the decoder K/V
  // projection) it is 8-10 % faster.
  p.tail_f = 1;
  p.tail_t0 = p.tiles;
  p.tail_per = p.per;
  p.zero_row0 = -1;
  bool tail_ok = p.var == 1 && p.nsplit == 1 && !d.atomic && d.C && !d.Cb && !d.relu &&
                 d.c_group <= 0 && !d.c_rows && d.ldc >= d.N && d.tile_hint == 0;
  if (tail_ok && d.resid) {
    const char* c0 = (const char*)d.C;
    const char* c1 = (const char*)(d.C + (d.M - 1) * d.ldc + d.N);
    const char* r0 = (const char*)d.resid;
    const char* r1 = (const char*)(d.resid + (d.M - 1) * d.ldr + d.N);
    if (r0 < c1 && c0 < r1) tail_ok = false;
  }
  // slabs: a workspace was given (its size is checked below) and the slab rows are whole f4s
  const bool slab_ok = d.ws && d.N % 4 == 0 && lp_al16(d.ws);
  if (tail_ok && p.tiles > slots && nk >= (slab_ok ? LP_TAIL_MIN_NK_SLAB : LP_TAIL_MIN_NK)) {
    const int64_t tn = (d.N + p.bn - 1) / p.bn;
    int64_t r = p.tiles % slots;
    r = (r + tn - 1) / tn * tn;  // whole rows of tiles: one contiguous zero-fill / slab
    if (r > 0 && r < p.tiles) {
      int64_t f = slots / r;
      if (f > nk / 4) f = nk / 4;
      if (f >= 2) {
        const int64_t per = (nk + f - 1) / f;
        const int tf = (int)((nk + per - 1) / per);
        const int64_t r0 = ((p.tiles - r) / tn) * bm;
        // (the slab epilogue is linear only -- no ReLU-backward gate: a masked launch keeps
        // the atomic tail, whose epilogue applies the mask)
        const bool slab = slab_ok && !d.mask && d.ws_elems >= (int64_t)tf * (d.M - r0) * d.N;
        if (slab || nk >= LP_TAIL_MIN_NK) {
          p.tail_per = per;
          p.tail_f = tf;
          p.tail_t0 = p.tiles - r;
          p.zero_row0 = r0;
          p.tail_slab = slab;
          p.pre = 0;  // the prefetching instantiations have no tail path
        }
      }
    }
  }
  return p;
}

// fp32 workspace elements the plan of d can use for partial slabs (split-K and tail split)
static int64_t lp_ws_need(const savqa_gemm_lp_desc& d0) {
  savqa_gemm_lp_desc d = d0;
  static float probe[4] __attribute__((aligned(16)));
  d.ws = probe;                 // any aligned non-null pointer: the plan only tests it
  d.ws_elems = INT64_MAX;
  const LpPlan p = lp_plan(d);
  int64_t need = 0;
  if (p.var == 1 && d.a_type != SAVQA_DT_FP8 && p.nsplit > 1 && d.C && !d.Cb && !d.relu &&
      !d.mask && !d.c_rows && d.n_store % 4 == 0 && d.c_group <= 0 && d.N % 4 == 0)
    need = (int64_t)p.nsplit * d.M * (d.N + (d.colsum_a ? 1 : 0));
  if (p.tail_slab) need = std::max(need, (int64_t)p.tail_f * (d.M - p.zero_row0) * d.N);
  return need;
}

}  // namespace savqa

using namespace savqa;

extern "C" int savqa_gemm_lp_supported(const savqa_gemm_lp_desc* d) {
  const char* msg = nullptr;
  return d && lp_ok(*d, &msg) ? 1 : 0;
}

extern "C" int64_t savqa_gemm_lp_ws_elems(const savqa_gemm_lp_desc* d) {
  const char* msg = nullptr;
  if (!d || !lp_ok(*d, &msg)) return 0;
  return lp_ws_need(*d);
}

extern "C" int savqa_gemm_lp_plan(const savqa_gemm_lp_desc* d, int32_t* out) {
  if (!d || !out) return fail(SAVQA_EINVAL, "savqa_gemm_lp_plan: null argument");
  const char* msg = nullptr;
  if (!lp_ok(*d, &msg)) return fail(SAVQA_EUNSUP, std::string("savqa_gemm_lp_plan: ") + msg);
  const LpPlan p = lp_plan(*d);
  out[0] = p.var;
  out[1] = p.nsplit;
  out[2] = (int32_t)(p.tail_t0 * p.nsplit + (p.tiles - p.tail_t0) * p.tail_f);
  out[3] = p.pre;
  return 0;
}

extern "C" int savqa_gemm_lp(void* stream, const savqa_gemm_lp_desc* dp) {
  if (!dp) return fail(SAVQA_EINVAL, "savqa_gemm_lp: null descriptor");
  LpArgs a{};
  a.d = *dp;
  savqa_gemm_lp_desc& d = a.d;
  if (d.M == 0 || d.N == 0) return 0;
  const char* msg = nullptr;
  if (!lp_ok(d, &msg)) return fail(SAVQA_EUNSUP, std::string("savqa_gemm_lp: ") + msg);
  if (d.c_group <= 0) d.c_group = 0;
  const bool fp8 = d.a_type == SAVQA_DT_FP8;
  const LpPlan p = lp_plan(d);
  const int var = p.var;
  const int bk = fp8 ? 128 : 64;
  a.kchunk = p.per * bk;
  a.tiles_n = (int)((d.N + p.bn - 1) / p.bn);
  a.dbg = SAVQA_LP_DIAG ? d.tile_hint >> 8 : 0;
  a.nblk = (int)p.tiles;
  a.ntiles_k = (int)p.per;
  a.full = (int)p.tail_t0;
  a.tail_t0 = (int)p.tail_t0;
  a.tail_f = p.tail_f;
  a.tail_kchunk = p.tail_per * bk;
  if (d.K == 0) a.kchunk = 0;
  // split-K slabs instead of atomics (savqa_gemm_lp_desc.ws): 128 x 128 kernel, plain
  // accumulation into fp32 C with a linear epilogue
  const bool slabs = d.ws && var == 1 && !fp8 && p.nsplit > 1 && d.C && !d.Cb && !d.relu &&
                     !d.mask && !d.c_rows && d.n_store % 4 == 0 && d.c_group <= 0 &&
                     d.N % 4 == 0 && ((uintptr_t)d.ws & 15) == 0 &&
                     d.ws_elems >= (int64_t)p.nsplit * d.M * (d.N + (d.colsum_a ? 1 : 0));
  a.slab = slabs ? d.ws : nullptr;
  a.cs_slab = slabs && d.colsum_a ? d.ws + (int64_t)p.nsplit * d.M * d.N : nullptr;
  a.tail_slab = p.tail_slab ? d.ws : nullptr;
  a.tail_r0 = p.tail_slab ? p.zero_row0 : 0;
  hipStream_t s = as_stream(stream);
  if (p.zero_row0 >= 0 && !p.tail_slab &&
      hipMemset2DAsync(d.C + p.zero_row0 * d.ldc, d.ldc * sizeof(float), 0, d.N * sizeof(float),
                       d.M - p.zero_row0, s) != hipSuccess)
    return fail(SAVQA_EUNSUP, "savqa_gemm_lp: tail zero-fill failed");
  const dim3 grid((unsigned)(p.tail_t0 + (p.tiles - p.tail_t0) * p.tail_f), (unsigned)p.nsplit),
      block(LP_NT);
  if (var == 5) {
    const dim3 b3(512);
    if (!d.a_trans && d.b_trans)
      hipLaunchKernelGGL((gemm_lp3_kernel<false, true>), grid, b3, 0, s, a);
    else if (!d.a_trans)
      hipLaunchKernelGGL((gemm_lp3_kernel<false, false>), grid, b3, 0, s, a);
    else if (!d.b_trans)
      hipLaunchKernelGGL((gemm_lp3_kernel<true, false>), grid, b3, 0, s, a);
    else
      hipLaunchKernelGGL((gemm_lp3_kernel<true, true>), grid, b3, 0, s, a);
  } else if (var != 1) {
    const dim3 b2(512);
#define SAVQA_LP2(BN_, WM_, BK_, NS_)                                                              \
  do {                                                                                             \
    if (!d.a_trans && d.b_trans)                                                                   \
      hipLaunchKernelGGL((gemm_lp2_kernel<256, BN_, WM_, BK_, NS_, false, true>), grid, b2, 0, s, a);  \
    else if (!d.a_trans)                                                                           \
      hipLaunchKernelGGL((gemm_lp2_kernel<256, BN_, WM_, BK_, NS_, false, false>), grid, b2, 0, s, a); \
    else if (!d.b_trans)                                                                           \
      hipLaunchKernelGGL((gemm_lp2_kernel<256, BN_, WM_, BK_, NS_, true, false>), grid, b2, 0, s, a);  \
    else                                                                                           \
      hipLaunchKernelGGL((gemm_lp2_kernel<256, BN_, WM_, BK_, NS_, true, true>), grid, b2, 0, s, a);   \
  } while (0)
    if (var == 3) SAVQA_LP2(256, 2, 64, 2);
    else SAVQA_LP2(128, 4, 64, 3);
#undef SAVQA_LP2
  } else if (fp8) {
    hipLaunchKernelGGL((gemm_lp_kernel<false, true, true, 0>), grid, block, 0, s, a);
  } else {
    const int pre = p.pre;
#define SAVQA_LP1(AT_, BT_)                                                                   \
  do {                                                                                        \
    if (pre == 1) hipLaunchKernelGGL((gemm_lp_kernel<AT_, BT_, false, 1>), grid, block, 0, s, a); \
    else if (pre == 2) hipLaunchKernelGGL((gemm_lp_kernel<AT_, BT_, false, 2>), grid, block, 0, s, a); \
    else if (pre == 3) hipLaunchKernelGGL((gemm_lp_kernel<AT_, BT_, false, 3>), grid, block, 0, s, a); \
    else hipLaunchKernelGGL((gemm_lp_kernel<AT_, BT_, false, 0>), grid, block, 0, s, a);     \
  } while (0)
    if (!d.a_trans && d.b_trans) SAVQA_LP1(false, true);
    else if (!d.a_trans && !d.b_trans) SAVQA_LP1(false, false);
    else if (d.a_trans && !d.b_trans) SAVQA_LP1(true, false);
    else SAVQA_LP1(true, true);
#undef SAVQA_LP1
  }
  if (d.colsum_a && var != 1) {  // the fused column sum lives in the 128 x 128 kernel only
    if (int rc = savqa_colsum_bf16(stream, d.A, d.K, d.M, d.lda, d.colsum_a)) return rc;
  }
  if (slabs || p.tail_slab) {
    if (int rc = check_launch("savqa_gemm_lp")) return rc;
    const int vec = (d.ldc % 4 == 0) && (((uintptr_t)d.C & 15) == 0);
    const int64_t r0 = p.tail_slab ? p.zero_row0 : 0, rows = d.M - r0;
    const int64_t n = rows * (d.N / 4), blk = (n + 255) / 256;
    const int64_t cs_blk = a.cs_slab ? (d.M + 255) / 256 : 0;
    hipLaunchKernelGGL(lp_slab_reduce_kernel, dim3((unsigned)(blk + cs_blk)), dim3(256), 0, s,
                       d.ws, p.tail_slab ? p.tail_f : p.nsplit, rows, d.N,
                       d.n_store > 0 ? d.n_store : d.N, d.C, d.ldc, vec, r0, p.tail_slab ? 1 : 0,
                       blk, a.cs_slab, d.M, d.colsum_a);
  }
  return check_launch("savqa_gemm_lp");
}
