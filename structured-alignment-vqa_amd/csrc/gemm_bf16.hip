// 3xbf16-MFMA GEMM for the 128x128-tile shapes (v_mfma_f32_32x32x16_bf16, fp32 accumulate):
// the "bf16x3" precision mode (savqa_gemm_desc.prec = 3).
//
// Same operator, operand layouts, epilogues and launch grid as gemm_f32_kernel (gemm.hip);
// only the products run on the bf16 matrix path (16x the fp32 MFMA rate per clock):
//   a = ah + al, b = bh + bl (ah = bf16(a), al = bf16(a - ah)), a*b ~ ah*bh + ah*bl + al*bh
//   (three MFMAs, ~2^-16 relative per product; fp32 storage and accumulation throughout).
// (The plain bf16 training mode, BASELINE cfg 3, runs on bf16-RESIDENT operands in
// gemm_lp.hip; the P template parameter below only ever takes 3 in the library.)
// Operands stay fp32 in HBM: each 128x32 tile is loaded as float4s, converted while it is
// staged, and kept in LDS as [row][k] bf16 planes (hi, and lo for prec 3) with 80-B rows,
// so every MFMA fragment (8 consecutive k of one row) is ONE conflict-free ds_read_b128,
// for k-contiguous operands (X, W of the forward; dY of dX) and m-contiguous ones alike
// (W of dX, dY^T and X of dW: a thread loads a 4k x 4m block and transposes it in
// registers before its ds_write_b64s). Register prefetch of the next tile during the
// MFMAs, double-buffered LDS, one barrier per k-tile, XCD-aware block order.
#include "gemm_common.h"

namespace savqa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int BF_BM = 128;              // block tile (rows and columns)
constexpr int BF_BK = 32;               // k per tile (two MFMA k-steps of 16)
constexpr int BF_LD = BF_BK + 8;        // bf16 per LDS row: 80 B (conflict-free b128 reads)
constexpr int BF_PLANE = BF_BM * BF_LD; // bf16 per operand plane

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// hi = bf16(v) (round to nearest even), lo = bf16(v - hi)
template <int P>
__device__ __forceinline__ void split4(f4 v, bf16x4& hi, bf16x4& lo) {
  hi = __builtin_convertvector(v, bf16x4);
  if constexpr (P == 3) {
    const f4 hf = __builtin_convertvector(hi, f4);
    lo = __builtin_convertvector(v - hf, bf16x4);
  }
}

// One operand's share of a 128 x 32 tile: 4 float4 per thread.
//   ROW (k contiguous in memory): float4 u = tid + 256*it covers row u/8, k 4*(u%8).
//   COL (m contiguous): the thread owns rows (m) 4*(tid%32) .. +3 and k 4*(tid/32) .. +3,
//        float4 it = row k 4*(tid/32) + it; transposed in registers at store time.
template <bool ROW>
struct BfOperand {
  f4 r[4];
  const float* rp[4];

  __device__ __forceinline__ void setup_fast(const float* __restrict__ base, int64_t ld,
                                             const int64_t* __restrict__ rows, int64_t m0, int tid) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      if constexpr (ROW) {
        const int u = tid + 256 * it;
        const int64_t m = m0 + u / 8;
        const int64_t rr = rows ? rows[m] : m;
        rp[it] = base + rr * ld + 4 * (u % 8);
      } else {
        rp[it] = base + (int64_t)(4 * (tid / 32) + it) * ld + m0 + 4 * (tid % 32);
      }
    }
  }

  __device__ __forceinline__ void load_fast(int64_t ld, int64_t k0) {
#pragma unroll
    for (int it = 0; it < 4; ++it)
      r[it] = *reinterpret_cast<const f4*>(ROW ? rp[it] + k0 : rp[it] + k0 * ld);
  }

  // guarded: clamped addresses, out-of-range elements selected to 0 (branch-free); rows
  // gathers the m index (ROW) or the k index (COL)
  __device__ __forceinline__ void load_slow(const float* __restrict__ base, int64_t ld,
                                            const int64_t* __restrict__ rows, int64_t mlim,
                                            int64_t m0, int64_t k0, int64_t kend, int tid) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      int64_t row, col, rlim, clim;
      if constexpr (ROW) {
        const int u = tid + 256 * it;
        row = m0 + u / 8;
        col = k0 + 4 * (u % 8);
        rlim = mlim;
        clim = kend;
      } else {
        row = k0 + 4 * (tid / 32) + it;
        col = m0 + 4 * (tid % 32);
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
      r[it] = f4{e[0], e[1], e[2], e[3]};
    }
  }

  // colsum_a (dW bias gradient, COL operand only): cs[q] += sum over this thread's 4 k of
  // A(m = 4*(tid%32) + q, k)
  __device__ __forceinline__ void accum(f4& cs) const {
    cs += (r[0] + r[1]) + (r[2] + r[3]);
  }

  template <int P>
  __device__ __forceinline__ void store(__bf16* __restrict__ hi_plane, int tid) const {
    __bf16* lo_plane = hi_plane + BF_PLANE;
    if constexpr (ROW) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int u = tid + 256 * it;
        const int off = (u / 8) * BF_LD + 4 * (u % 8);
        bf16x4 h, l;
        split4<P>(r[it], h, l);
        *reinterpret_cast<bf16x4*>(hi_plane + off) = h;
        if constexpr (P == 3) *reinterpret_cast<bf16x4*>(lo_plane + off) = l;
      }
    } else {
      const int g = tid % 32, kg = tid / 32;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int q = (s + g) & 3;  // staggered: lanes 4 rows apart would hit one bank
        const f4 v = f4{r[0][q], r[1][q], r[2][q], r[3][q]};  // k = 4kg .. 4kg+3 of row 4g+q
        const int off = (4 * g + q) * BF_LD + 4 * kg;
        bf16x4 h, l;
        split4<P>(v, h, l);
        *reinterpret_cast<bf16x4*>(hi_plane + off) = h;
        if constexpr (P == 3) *reinterpret_cast<bf16x4*>(lo_plane + off) = l;
      }
    }
  }
};

// fragment: 32 rows x 16 k of a plane, lane (i = lane&31, h = lane>>5) holds row i, k 8h..8h+7
__device__ __forceinline__ bf16x8 frag(const __bf16* __restrict__ plane, int row0, int kk, int lane) {
  return *reinterpret_cast<const bf16x8*>(plane + (row0 + (lane & 31)) * BF_LD + kk * 16 + 8 * (lane >> 5));
}

template <int P>
__device__ __forceinline__ void bf_compute_tile(const __bf16* __restrict__ As, const __bf16* __restrict__ Bs,
                                                int wm, int wn, int lane, f32x16 (&acc)[2][2]) {
#pragma unroll
  for (int kk = 0; kk < BF_BK / 16; ++kk) {
    bf16x8 ah[2], bh[2], al[2], bl[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ah[i] = frag(As, wm * 64 + i * 32, kk, lane);
      bh[i] = frag(Bs, wn * 64 + i * 32, kk, lane);
      if constexpr (P == 3) {
        al[i] = frag(As + BF_PLANE, wm * 64 + i * 32, kk, lane);
        bl[i] = frag(Bs + BF_PLANE, wn * 64 + i * 32, kk, lane);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (P == 3) {  // small terms first
          acc[i][j] = mfma_bf16(al[i], bh[j], acc[i][j]);
          acc[i][j] = mfma_bf16(ah[i], bl[j], acc[i][j]);
        }
        acc[i][j] = mfma_bf16(ah[i], bh[j], acc[i][j]);
      }
  }
}

template <bool AT, bool BT, int P, bool FAST>
__device__ __forceinline__ void bf_mainloop(const savqa_gemm_desc& d, __bf16* smem, int64_t m0,
                                            int64_t n0, int64_t kbeg, int64_t kend, int ntiles,
                                            f32x16 (&acc)[2][2], bool do_cs, f4& cs) {
  constexpr int NPL = P == 3 ? 2 : 1;
  constexpr int STAGE = 2 * NPL * BF_PLANE;  // A planes then B planes
  BfOperand<!AT> la;
  BfOperand<BT> lb;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  if constexpr (FAST) {
    la.setup_fast(d.A, d.lda, d.a_rows, m0, tid);
    lb.setup_fast(d.B, d.ldb, d.b_rows, n0, tid);
  }
  auto load = [&](int64_t k0) {
    if constexpr (FAST) {
      la.load_fast(d.lda, k0);
      lb.load_fast(d.ldb, k0);
    } else {
      la.load_slow(d.A, d.lda, d.a_rows, d.M, m0, k0, kend, tid);
      lb.load_slow(d.B, d.ldb, d.b_rows, d.N, n0, k0, kend, tid);
    }
  };
  load(kbeg);
  if (do_cs) la.accum(cs);
  la.template store<P>(smem, tid);
  lb.template store<P>(smem + NPL * BF_PLANE, tid);
  __syncthreads();
  int cur = 0;
  for (int tt = 0; tt < ntiles; ++tt) {
    const bool more = tt + 1 < ntiles;
    if (more) load(kbeg + (int64_t)(tt + 1) * BF_BK);
    const __bf16* st = smem + cur * STAGE;
    bf_compute_tile<P>(st, st + NPL * BF_PLANE, wm, wn, lane, acc);
    if (more) {
      if (do_cs) la.accum(cs);
      __bf16* nx = smem + (cur ^ 1) * STAGE;
      la.template store<P>(nx, tid);
      lb.template store<P>(nx + NPL * BF_PLANE, tid);
    }
    __syncthreads();
    cur ^= 1;
  }
}

template <bool AT, bool BT, int P>
__global__ __launch_bounds__(GEMM_NT, 2) void gemm_bf16_kernel(savqa_gemm_desc d, GemmGrid gg,
                                                               int avec, int bvec) {
  constexpr int NPL = P == 3 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * NPL * BF_PLANE];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int bid = blockIdx.x;
  int t;
  int64_t kbeg, kend;
  bool first_split, atomic;
  if (bid < gg.full) {
    int slice;
    split_remap(gg.full, t, slice);
    kbeg = (int64_t)slice * gg.kchunk;
    kend = min(d.K, kbeg + gg.kchunk);
    first_split = slice == 0;
    atomic = d.atomic || gridDim.y > 1;
  } else {
    const int u = bid - gg.full;
    const int part = u % gg.tail_f;
    t = gg.tail_t0 + u / gg.tail_f;
    kbeg = (int64_t)part * gg.tail_kchunk;
    kend = min(d.K, kbeg + gg.tail_kchunk);
    first_split = part == 0;
    atomic = true;
  }
  const int tn = t % gg.tiles_n, tm = t / gg.tiles_n;
  const int64_t m0 = (int64_t)tm * BF_BM, n0 = (int64_t)tn * BF_BM;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const bool a_kgather = AT && d.a_rows;
  const bool b_kgather = !BT && d.b_rows;
  const bool fast = (m0 + BF_BM <= d.M) && (n0 + BF_BM <= d.N) && ((kend - kbeg) % BF_BK == 0) &&
                    avec && bvec && !a_kgather && !b_kgather;
  const int ntiles = kend > kbeg ? (int)((kend - kbeg + BF_BK - 1) / BF_BK) : 0;
  const bool do_cs = AT && d.colsum_a != nullptr && tn == 0;
  f4 cs = {0.f, 0.f, 0.f, 0.f};
  if (ntiles > 0) {
    if (fast)
      bf_mainloop<AT, BT, P, true>(d, smem, m0, n0, kbeg, kend, ntiles, acc, do_cs, cs);
    else
      bf_mainloop<AT, BT, P, false>(d, smem, m0, n0, kbeg, kend, ntiles, acc, do_cs, cs);
  }
  if constexpr (AT) {
    if (do_cs) {  // block-uniform; smem is free after the main loop's last barrier
      // thread rows tid/32 hold partials of columns 4*(tid%32)..+3: plain LDS rows, then
      // one thread per column (no LDS float atomics)
      float* red = reinterpret_cast<float*>(smem);
      *reinterpret_cast<f4*>(&red[(threadIdx.x / 32) * BF_BM + 4 * (threadIdx.x % 32)]) = cs;
      __syncthreads();
      for (int i = threadIdx.x; i < BF_BM; i += GEMM_NT) {
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < GEMM_NT / 32; ++r) v += red[r * BF_BM + i];
        if (m0 + i < d.M) atomicAdd(&d.colsum_a[m0 + i], v);
      }
    }
  }
  // epilogue: the 32x32 accumulator layout of every v_mfma_f32_32x32x* form
  const bool ident = d.c_rows == nullptr && d.c_group >= d.M && d.c_offset == 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (m >= d.M) continue;
      const EpiRow er = epi_row(d, m, ident);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t n = n0 + wn * 64 + j * 32 + (lane & 31);
        if (n >= d.N) continue;
        epi_store(d, er, m, n, acc[i][j][r], first_split, atomic);
      }
    }
  }
}

}  // namespace savqa

// Launch of the bf16 kernels on a plan made by savqa_gemm (gemm.hip): grid (grid_x, nsplit).
int savqa_launch_gemm_bf16(const savqa_gemm_desc& d, const savqa::GemmGrid& gg, int grid_x,
                           int nsplit, hipStream_t s, int avec, int bvec) {
  using namespace savqa;
  const dim3 g(grid_x, nsplit), b(GEMM_NT);
#define SAVQA_BF_LAUNCH(AT, BT)                                                              \
  do {                                                                                       \
    hipLaunchKernelGGL((gemm_bf16_kernel<AT, BT, 3>), g, b, 0, s, d, gg, avec, bvec);        \
  } while (0)
  if (!d.a_trans && d.b_trans) SAVQA_BF_LAUNCH(false, true);
  else if (!d.a_trans && !d.b_trans) SAVQA_BF_LAUNCH(false, false);
  else if (d.a_trans && !d.b_trans) SAVQA_BF_LAUNCH(true, false);
  else SAVQA_BF_LAUNCH(true, true);
#undef SAVQA_BF_LAUNCH
  return 0;
}
