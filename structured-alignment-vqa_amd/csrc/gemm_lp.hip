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

struct LpArgs {
  savqa_gemm_lp_desc d;
  int tiles_n, ntiles_k;  // k-tiles per split slice
  int64_t kchunk;         // elements of k per split slice
  int nblk;               // tiles (grid.x)
};

// Per-lane LDS-DMA sources of one operand, resolved once per workgroup.
//   R image: instruction u of wave w covers tile rows 8(4w+u) .. +7; lane L -> row
//     8(4w+u) + L/8, physical chunk L%8, logical chunk (L%8) ^ swz(row).
//   T image: instruction u covers k rows 4(4w+u) .. +3; lane L -> row 4(4w+u) + L/16,
//     physical chunk L%16, logical chunk (L%16) ^ 2h(row); advances by whole rows.
template <bool T, bool FP8>
struct LpStage {
  const char* p[4];
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
      } else {
        const int r = 4 * ins + (lane >> 4);
        const int lc = (lane & 15) ^ (2 * th(r));
        int64_t c = r0 + lc * 8;
        c = c + 8 <= lim ? c : lim - 8;
        p[u] = b + ((kbeg + r) * ld + c) * esz;
      }
    }
    step = T ? (int64_t)64 * ld * esz : LP_KB;
  }

  __device__ __forceinline__ void issue(char* img, int wave, int64_t t) const {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      glds16(p[u] + t * step, (lds_void*)(img + (4 * wave + u) * 1024));
  }
};

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

template <bool AT, bool BT, bool FP8>
__global__ __launch_bounds__(LP_NT, LP_OCC) void gemm_lp_kernel(LpArgs args) {
  const savqa_gemm_lp_desc& d = args.d;
  __shared__ __attribute__((aligned(1024))) char smem[2 * 2 * LP_IMG];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int t = xcd_remap(blockIdx.x, args.nblk);
  const int tn = t % args.tiles_n, tm = t / args.tiles_n;
  const int64_t m0 = (int64_t)tm * LP_TILE, n0 = (int64_t)tn * LP_TILE;
  const int64_t kbeg = (int64_t)blockIdx.y * args.kchunk;
  const int64_t kend = min(d.K, kbeg + args.kchunk);
  const int nt = (int)((kend - kbeg) / (FP8 ? 128 : 64));
  const bool first_split = blockIdx.y == 0;
  const int esz = FP8 ? 1 : 2;

  LpStage<AT, FP8> sa;
  LpStage<!BT, FP8> sb;
  sa.setup(d.A, d.lda, esz, AT ? nullptr : d.a_rows, m0, d.M, kbeg, wave, lane);
  sb.setup(d.B, d.ldb, esz, nullptr, n0, d.N, kbeg, wave, lane);

  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // fp8 block scales of this lane's rows: A rows (m), B rows (n), block k/32 + g
  int sca[4], scb[4];
  const int g = lane >> 4;
  auto load_scales = [&](int64_t kt) {
    if constexpr (FP8) {
      const int64_t blk = (kbeg >> 5) + kt * 4 + g;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int64_t m = m0 + wm * 64 + 16 * i + (lane & 15);
        m = m < d.M ? m : d.M - 1;
        const int64_t rr = d.a_rows ? d.a_rows[m] : m;
        sca[i] = d.a_scale[rr * d.lds_a + blk];
        int64_t n = n0 + wn * 64 + 16 * i + (lane & 15);
        n = n < d.N ? n : d.N - 1;
        scb[i] = d.b_scale[n * d.lds_b + blk];
      }
    }
  };

  if (nt > 0) {
    sa.issue(smem, wave, 0);
    sb.issue(smem + LP_IMG, wave, 0);
    load_scales(0);
    __syncthreads();  // vmcnt(0) + barrier: stage 0 landed for every wave
    for (int kt = 0; kt < nt; ++kt) {
      const char* ia = smem + (kt & 1) * 2 * LP_IMG;
      const char* ib = ia + LP_IMG;
      int sca_c[4], scb_c[4];
      if constexpr (FP8) {
#pragma unroll
        for (int i = 0; i < 4; ++i) { sca_c[i] = sca[i]; scb_c[i] = scb[i]; }
      }
      if (kt + 1 < nt) {  // next k-tile into the other buffer (read one barrier ago)
        char* nx = smem + ((kt + 1) & 1) * 2 * LP_IMG;
        sa.issue(nx, wave, kt + 1);
        sb.issue(nx + LP_IMG, wave, kt + 1);
        load_scales(kt + 1);
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
                b[j], a[i], acc[i][j], 0, 0, 0, scb_c[j], 0, sca_c[i]);
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
      }
      __syncthreads();  // k-tile kt+1 landed; buffer kt free for k-tile kt+2
    }
  }

  // ---------------------------------------------------------------- epilogue
  // acc[i][j][r] = C(m = m0 + 64wm + 16i + (lane & 15), n = n0 + 64wn + 16j + 4g + r)
  const bool ident = d.c_group <= 0;
  const bool vec_c = d.C && (d.ldc & 3) == 0 && (((uintptr_t)d.C) & 15) == 0;
  float bv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t n = min(n0 + wn * 64 + 16 * j + 4 * g + r, d.N - 1);
      bv[j][r] = (first_split && d.bias) ? d.bias[n] : 0.f;
    }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = m0 + wm * 64 + 16 * i + (lane & 15);
    const int64_t mc = m < d.M ? m : d.M - 1;
    // this row's epilogue operands, loaded before its first store (vmcnt counts stores)
    float rv[4][4], mk[4][4], pv[4][4];
    const int64_t mr = d.mask_arows ? d.a_rows[mc] : mc;
    const int64_t pr = d.rowvec ? (mc % d.rowvec_period) : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t n = min(n0 + wn * 64 + 16 * j + 4 * g + r, d.N - 1);
        rv[j][r] = (first_split && d.resid) ? d.resid[mc * d.ldr + n] : 0.f;
        pv[j][r] = (first_split && d.rowvec) ? d.rowvec[pr * d.ldrv + n] : 0.f;
        if (d.mask)
          mk[j][r] = d.mask_type == SAVQA_DT_BF16
                         ? bf2f(static_cast<const __bf16*>(d.mask)[mr * d.ldmask + n])
                         : static_cast<const float*>(d.mask)[mr * d.ldmask + n];
        else
          mk[j][r] = 1.f;
      }
    if (m >= d.M) continue;
    int64_t cr;
    if (ident) {
      cr = m;
    } else {
      const uint32_t mu = (uint32_t)m, cg = (uint32_t)d.c_group;
      cr = (int64_t)(mu / cg) * d.c_stride + (int64_t)(mu % cg) + d.c_offset;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t nb = n0 + wn * 64 + 16 * j + 4 * g;
      if (nb >= d.N) continue;
      f4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = acc[i][j][r] * d.alpha + bv[j][r] + pv[j][r];
        if (d.relu) x = fmaxf(x, 0.f);
        if (!(mk[j][r] > 0.f)) x = 0.f;
        v[r] = x + rv[j][r];
      }
      const bool full = nb + 4 <= d.N;
      if (d.C) {
        float* cp = d.C + cr * d.ldc + nb;
        if (d.atomic) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (nb + r < d.N) atomicAdd(cp + r, v[r]);
        } else if (full && vec_c) {
          *reinterpret_cast<f4*>(cp) = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (nb + r < d.N) cp[r] = v[r];
        }
      }
      if (d.Cb) {
        __bf16* cp = static_cast<__bf16*>(d.Cb) + cr * d.ldcb + nb;
        const bf16x4 h = __builtin_convertvector(v, bf16x4);
        if (full && (d.ldcb & 3) == 0 && (((uintptr_t)d.Cb) & 7) == 0) {
          *reinterpret_cast<bf16x4*>(cp) = h;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (nb + r < d.N) cp[r] = h[r];
        }
      }
    }
  }
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
  if ((d.split_k > 1 || d.split_k < 0) && (!d.atomic || !d.C)) return no("split-K needs atomic fp32 C");
  if (d.a_rows && d.a_trans) return no("a_rows needs a_trans = 0");
  if (d.mask && d.mask_arows && !d.a_rows) return no("mask_arows needs a_rows");
  if (d.mask && d.mask_type != SAVQA_DT_BF16 && d.mask_type != SAVQA_DT_F32) return no("mask_type");
  if (d.rowvec && d.rowvec_period <= 0) return no("rowvec_period");
  if (!al16(d.A) || !al16(d.B)) return no("operands must be 16-B aligned");
  if (fp8) {
    if (d.a_trans || !d.b_trans) return no("fp8 needs a_trans = 0, b_trans = 1");
    if (d.K % 128) return no("fp8 needs K % 128 == 0");
    if (d.lda % 16 || d.ldb % 16) return no("fp8 needs ld % 16 == 0");
    if (!d.a_scale || !d.b_scale) return no("fp8 needs block scales");
  } else {
    if (d.K % 64) return no("bf16 needs K % 64 == 0");
    if (d.lda % 8 || d.ldb % 8) return no("bf16 needs ld % 8 == 0");
    if (d.a_trans && d.M % 8) return no("a_trans needs M % 8 == 0");
    if (!d.b_trans && d.N % 8) return no("b_trans = 0 needs N % 8 == 0");
  }
  return true;
}

}  // namespace savqa

using namespace savqa;

extern "C" int savqa_gemm_lp_supported(const savqa_gemm_lp_desc* d) {
  const char* msg = nullptr;
  return d && lp_ok(*d, &msg) ? 1 : 0;
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
  const int bk = fp8 ? 128 : 64;
  const int64_t tiles = ((d.M + 127) / 128) * ((d.N + 127) / 128);
  const int64_t nk = d.K / bk;
  int split = d.split_k > 1 ? d.split_k : 1;
  if (d.split_k < 0) {  // minimise rounds(s) * (k-tiles per slice + per-block overhead)
    const int slots = lp_slots();
    int64_t best_cost = INT64_MAX;
    for (int s = 1; s <= 64 && (s == 1 || nk / s >= 4); ++s) {
      const int64_t rounds = (tiles * s + slots - 1) / slots;
      const int64_t cost = rounds * ((nk + s - 1) / s + 3);
      if (cost < best_cost) { best_cost = cost; split = s; }
    }
  }
  const int64_t per = (nk + split - 1) / split;
  a.kchunk = per * bk;
  const int nsplit = nk > 0 ? (int)((nk + per - 1) / per) : 1;
  a.tiles_n = (int)((d.N + 127) / 128);
  a.nblk = (int)tiles;
  a.ntiles_k = (int)per;
  if (d.K == 0) a.kchunk = 0;
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)tiles, (unsigned)nsplit), block(LP_NT);
  if (fp8)
    hipLaunchKernelGGL((gemm_lp_kernel<false, true, true>), grid, block, 0, s, a);
  else if (!d.a_trans && d.b_trans)
    hipLaunchKernelGGL((gemm_lp_kernel<false, true, false>), grid, block, 0, s, a);
  else if (!d.a_trans && !d.b_trans)
    hipLaunchKernelGGL((gemm_lp_kernel<false, false, false>), grid, block, 0, s, a);
  else if (d.a_trans && !d.b_trans)
    hipLaunchKernelGGL((gemm_lp_kernel<true, false, false>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((gemm_lp_kernel<true, true, false>), grid, block, 0, s, a);
  return check_launch("savqa_gemm_lp");
}
