// fp32 GEMM on gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact f32, 64 FLOP/clk/SIMD).
//
// Replaces every nn.Linear of the SA-VQA model_v=3 path and the two backward GEMMs of
// each (dX = dY W, dW = dY^T X). One kernel template covers the three operand
// layouts the path needs:
//   forward  C = X W^T        A [M][K] (a_trans=0), B [N][K] (b_trans=1)
//   dX       C = dY W         A [M][K] (a_trans=0), B [K][N] (b_trans=0)
//   dW      C += dY^T X       A [K][M] (a_trans=1), B [K][N] (b_trans=0), split-K + atomics
// Fused epilogues: bias, periodic row vector (learned position table), residual,
// ReLU, ReLU-backward mask, beta-accumulate, atomic scatter to indexed rows
// (embedding-table gradient) -- see include/savqa.h for the exact formula.
//
// Tiling: 256 threads = 4 waves (2x2), block tile BMxBN (128x128 or 64x64), BK = 32,
// LDS k-major [BK][BM+pad] so every MFMA operand read is 32 consecutive floats per
// half-wave (conflict-free ds_read_b32). Global loads are float4 along the
// contiguous dimension; register-staged double buffering with the LDS write after the
// compute of the current tile (cdna_hip_programming.md T14), one barrier per k-tile.
#include "common.h"

namespace savqa {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GEMM_BK = 32;
constexpr int GEMM_NT = 256;

template <int BM, bool KCONTIG>
struct TileLoader {
  // KCONTIG: the operand's k index is the contiguous one in global memory
  //   (A stored [M][K], or B stored [N][K]) -> float4 along k, scalar transposed LDS writes.
  // else: the operand's m/n index is contiguous ([K][M] / [K][N]) -> float4 along m/n.
  static constexpr int LD = KCONTIG ? BM + 1 : BM + 4;
  static constexpr int ITERS = BM * GEMM_BK / 4 / GEMM_NT;  // float4 per thread
  float4 r[ITERS];
  const float* rp[ITERS];  // FAST + KCONTIG: row pointers, resolved once per block

  // FAST path (block-uniform): the whole tile is in range, the k range is a multiple of
  // GEMM_BK and the operand is 16-B aligned -> branch-free float4 loads.
  __device__ __forceinline__ void setup_fast(const float* __restrict__ base, int64_t ld,
                                             const int64_t* __restrict__ rows, int64_t m0,
                                             int tid) {
    if (KCONTIG) {
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int idx = tid + it * GEMM_NT;
        const int64_t m = m0 + (idx >> 3);
        const int64_t rr = rows ? rows[m] : m;
        rp[it] = base + rr * ld + (idx & 7) * 4;
      }
    }
  }

  __device__ __forceinline__ void load_fast(const float* __restrict__ base, int64_t ld,
                                            int64_t m0, int64_t k0, int tid) {
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int idx = tid + it * GEMM_NT;
      if (KCONTIG) {
        r[it] = *reinterpret_cast<const float4*>(rp[it] + k0);
      } else {
        constexpr int PER_K = BM / 4;
        const int kr = idx / PER_K;
        const int mq = (idx % PER_K) * 4;
        r[it] = *reinterpret_cast<const float4*>(base + (k0 + kr) * ld + m0 + mq);
      }
    }
  }

  // guarded path for edge tiles, k tails, unaligned operands and k-row gathers
  __device__ __forceinline__ void load_slow(const float* __restrict__ base, int64_t ld,
                                            const int64_t* __restrict__ rows, int64_t mlim,
                                            int64_t m0, int64_t k0, int64_t kend, bool vec,
                                            int tid) {
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int idx = tid + it * GEMM_NT;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (KCONTIG) {
        const int row = idx >> 3;
        const int kq = (idx & 7) * 4;
        const int64_t m = m0 + row;
        const int64_t k = k0 + kq;
        if (m < mlim) {
          const int64_t rr = rows ? rows[m] : m;
          const float* p = base + rr * ld + k;
          if (vec && k + 3 < kend) {
            v = *reinterpret_cast<const float4*>(p);
          } else {
            if (k + 0 < kend) v.x = p[0];
            if (k + 1 < kend) v.y = p[1];
            if (k + 2 < kend) v.z = p[2];
            if (k + 3 < kend) v.w = p[3];
          }
        }
      } else {
        constexpr int PER_K = BM / 4;
        const int kr = idx / PER_K;
        const int mq = (idx % PER_K) * 4;
        const int64_t k = k0 + kr;
        const int64_t m = m0 + mq;
        if (k < kend) {
          const int64_t kk = rows ? rows[k] : k;
          const float* p = base + kk * ld + m;
          if (vec && m + 3 < mlim) {
            v = *reinterpret_cast<const float4*>(p);
          } else {
            if (m + 0 < mlim) v.x = p[0];
            if (m + 1 < mlim) v.y = p[1];
            if (m + 2 < mlim) v.z = p[2];
            if (m + 3 < mlim) v.w = p[3];
          }
        }
      }
      r[it] = v;
    }
  }

  __device__ __forceinline__ void store(float* __restrict__ s, int tid) const {
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int idx = tid + it * GEMM_NT;
      if (KCONTIG) {
        const int row = idx >> 3;
        const int kq = (idx & 7) * 4;
        s[(kq + 0) * LD + row] = r[it].x;
        s[(kq + 1) * LD + row] = r[it].y;
        s[(kq + 2) * LD + row] = r[it].z;
        s[(kq + 3) * LD + row] = r[it].w;
      } else {
        constexpr int PER_K = BM / 4;
        const int kr = idx / PER_K;
        const int mq = (idx % PER_K) * 4;
        *reinterpret_cast<float4*>(&s[kr * LD + mq]) = r[it];
      }
    }
  }
};

template <int BM, int BN, bool AT, bool BT>
struct GemmTile {
  using LA = TileLoader<BM, !AT>;
  using LB = TileLoader<BN, BT>;
  static constexpr int SA = GEMM_BK * LA::LD;
  static constexpr int SB = GEMM_BK * LB::LD;
  static constexpr int WM = BM / 2, WN = BN / 2;
  static constexpr int FM = WM / 32, FN = WN / 32;
};

template <int BM, int BN, bool AT, bool BT, bool FAST>
__device__ __forceinline__ void gemm_mainloop(const savqa_gemm_desc& d, float* smem, int64_t m0,
                                              int64_t n0, int64_t kbeg, int64_t kend, bool avec,
                                              bool bvec,
                                              f32x16 (&acc)[GemmTile<BM, BN, AT, BT>::FM]
                                                           [GemmTile<BM, BN, AT, BT>::FN]) {
  using GT = GemmTile<BM, BN, AT, BT>;
  typename GT::LA la;
  typename GT::LB lb;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntiles = kend > kbeg ? (int)((kend - kbeg + GEMM_BK - 1) / GEMM_BK) : 0;
  if (ntiles == 0) return;
  if (FAST) {
    la.setup_fast(d.A, d.lda, d.a_rows, m0, tid);
    lb.setup_fast(d.B, d.ldb, d.b_rows, n0, tid);
    la.load_fast(d.A, d.lda, m0, kbeg, tid);
    lb.load_fast(d.B, d.ldb, n0, kbeg, tid);
  } else {
    la.load_slow(d.A, d.lda, d.a_rows, d.M, m0, kbeg, kend, avec, tid);
    lb.load_slow(d.B, d.ldb, d.b_rows, d.N, n0, kbeg, kend, bvec, tid);
  }
  la.store(smem, tid);
  lb.store(smem + 2 * GT::SA, tid);
  __syncthreads();

  int cur = 0;
  const int kl = lane >> 5;
  const int il = lane & 31;
  for (int tt = 0; tt < ntiles; ++tt) {
    const bool more = tt + 1 < ntiles;
    if (more) {
      const int64_t kn = kbeg + (int64_t)(tt + 1) * GEMM_BK;
      if (FAST) {
        la.load_fast(d.A, d.lda, m0, kn, tid);
        lb.load_fast(d.B, d.ldb, n0, kn, tid);
      } else {
        la.load_slow(d.A, d.lda, d.a_rows, d.M, m0, kn, kend, avec, tid);
        lb.load_slow(d.B, d.ldb, d.b_rows, d.N, n0, kn, kend, bvec, tid);
      }
    }
    const float* As = smem + cur * GT::SA + kl * GT::LA::LD + wm * GT::WM + il;
    const float* Bs = smem + 2 * GT::SA + cur * GT::SB + kl * GT::LB::LD + wn * GT::WN + il;
#pragma unroll
    for (int kk = 0; kk < GEMM_BK; kk += 2) {
      float a[GT::FM], b[GT::FN];
#pragma unroll
      for (int i = 0; i < GT::FM; ++i) a[i] = As[kk * GT::LA::LD + i * 32];
#pragma unroll
      for (int j = 0; j < GT::FN; ++j) b[j] = Bs[kk * GT::LB::LD + j * 32];
#pragma unroll
      for (int i = 0; i < GT::FM; ++i)
#pragma unroll
        for (int j = 0; j < GT::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      la.store(smem + (cur ^ 1) * GT::SA, tid);
      lb.store(smem + 2 * GT::SA + (cur ^ 1) * GT::SB, tid);
    }
    __syncthreads();
    cur ^= 1;
  }
}

template <int BM, int BN, bool AT, bool BT>
__global__ __launch_bounds__(GEMM_NT, 2) void gemm_f32_kernel(savqa_gemm_desc d, int tiles_m,
                                                             int tiles_n, int64_t kchunk,
                                                             int avec, int bvec) {
  using GT = GemmTile<BM, BN, AT, BT>;
  constexpr int FM = GT::FM, FN = GT::FN, WM = GT::WM, WN = GT::WN;
  __shared__ __attribute__((aligned(16))) float smem[2 * (GT::SA + GT::SB)];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int nblk = tiles_m * tiles_n;
  const int t = xcd_remap(blockIdx.x, nblk);
  const int tn = t % tiles_n;
  const int tm = t / tiles_n;
  const int64_t m0 = (int64_t)tm * BM;
  const int64_t n0 = (int64_t)tn * BN;
  const int64_t kbeg = (int64_t)blockIdx.y * kchunk;
  const int64_t kend = min(d.K, kbeg + kchunk);

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // block-uniform choice of the branch-free main loop
  const bool a_kgather = AT && d.a_rows;
  const bool b_kgather = !BT && d.b_rows;
  const bool fast = (m0 + BM <= d.M) && (n0 + BN <= d.N) && ((kend - kbeg) % GEMM_BK == 0) &&
                    avec && bvec && !a_kgather && !b_kgather;
  if (fast)
    gemm_mainloop<BM, BN, AT, BT, true>(d, smem, m0, n0, kbeg, kend, avec, bvec, acc);
  else
    gemm_mainloop<BM, BN, AT, BT, false>(d, smem, m0, n0, kbeg, kend, avec, bvec, acc);

  // ---------------------------------------------------------------- epilogue
  const bool first_split = blockIdx.y == 0;
  const bool atomic = d.atomic || gridDim.y > 1;
  const bool ident = d.c_rows == nullptr && d.c_group >= d.M && d.c_offset == 0;
  const uint32_t cg = (uint32_t)d.c_group;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (m >= d.M) continue;
      int64_t cr;
      if (ident) {
        cr = m;
      } else if (d.c_rows) {
        cr = d.c_rows[m];
      } else {
        const uint32_t mu = (uint32_t)m;
        cr = (int64_t)(mu / cg) * d.c_stride + (int64_t)(mu % cg) + d.c_offset;
      }
      float* crow = d.C + cr * d.ldc;
      const float rs = d.rowscale ? d.rowscale[m] : 1.f;
      const int64_t mr = d.mask_arows ? d.a_rows[m] : m;
      const int64_t pr = d.rowvec ? (int64_t)((uint32_t)m % (uint32_t)d.rowvec_period) : 0;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int64_t n = n0 + wn * WN + j * 32 + (lane & 31);
        if (n >= d.N) continue;
        float v = acc[i][j][r] * d.alpha;
        if (first_split) {
          if (d.bias) v += d.bias[n];
          if (d.rowvec) v += d.rowvec[pr * d.ldrv + n];
        }
        if (d.relu) v = fmaxf(v, 0.f);
        v *= rs;
        if (d.mask && !(d.mask[mr * d.ldmask + n] > 0.f)) v = 0.f;
        if (first_split && d.resid) v += d.resid[m * d.ldr + n];
        float* cp = crow + n;
        if (atomic) {
          atomicAdd(cp, v);
        } else if (d.beta != 0.f) {
          *cp = v + d.beta * *cp;
        } else {
          *cp = v;
        }
      }
    }
  }
}

template <int BM, int BN, bool AT, bool BT>
static void launch_gemm(const savqa_gemm_desc& d, hipStream_t s, int split, int avec, int bvec) {
  const int tm = (int)((d.M + BM - 1) / BM);
  const int tn = (int)((d.N + BN - 1) / BN);
  int64_t kchunk = (d.K + split - 1) / split;
  kchunk = (kchunk + GEMM_BK - 1) / GEMM_BK * GEMM_BK;
  const int nsplit = (int)((d.K + kchunk - 1) / kchunk);
  dim3 grid(tm * tn, nsplit > 0 ? nsplit : 1);
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, AT, BT>), grid, dim3(GEMM_NT), 0, s, d, tm, tn,
                     kchunk, avec, bvec);
}

template <int BM, int BN>
static void dispatch_layout(const savqa_gemm_desc& d, hipStream_t s, int split, int avec, int bvec) {
  if (!d.a_trans && d.b_trans) launch_gemm<BM, BN, false, true>(d, s, split, avec, bvec);
  else if (!d.a_trans && !d.b_trans) launch_gemm<BM, BN, false, false>(d, s, split, avec, bvec);
  else if (d.a_trans && !d.b_trans) launch_gemm<BM, BN, true, false>(d, s, split, avec, bvec);
  else launch_gemm<BM, BN, true, true>(d, s, split, avec, bvec);
}

}  // namespace savqa

using namespace savqa;

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

extern "C" int savqa_gemm(void* stream, const savqa_gemm_desc* dp) {
  if (!dp) return fail(SAVQA_EINVAL, "savqa_gemm: null descriptor");
  savqa_gemm_desc d = *dp;
  if (d.M < 0 || d.N < 0 || d.K < 0) return fail(SAVQA_EINVAL, "savqa_gemm: negative dims");
  if (d.M == 0 || d.N == 0) return 0;
  if (!d.A || !d.B || !d.C) return fail(SAVQA_EINVAL, "savqa_gemm: null operand");
  if (d.mask && d.mask_arows && (d.a_trans || !d.a_rows))
    return fail(SAVQA_EINVAL, "savqa_gemm: mask_arows needs a_trans=0 and a_rows");
  if (d.c_group <= 0) { d.c_group = d.M; d.c_stride = d.M; }
  if (d.rowvec && d.rowvec_period <= 0) return fail(SAVQA_EINVAL, "savqa_gemm: rowvec_period");
  int split = d.split_k > 1 ? d.split_k : 1;
  const int avec = (d.lda % 4 == 0) && aligned16(d.A);
  const int bvec = (d.ldb % 4 == 0) && aligned16(d.B);
  hipStream_t s = as_stream(stream);
  // 128x128 tiles once there is enough parallelism (split-K counts), else 64x64
  const int64_t big_tiles = ((d.M + 127) / 128) * ((d.N + 127) / 128) * split;
  if (big_tiles >= 160)
    dispatch_layout<128, 128>(d, s, split, avec, bvec);
  else
    dispatch_layout<64, 64>(d, s, split, avec, bvec);
  return check_launch("savqa_gemm");
}

// ---------------------------------------------------------------- column sums
namespace savqa {
// out[c] += sum_r X[r][c]: 256 threads = 64 columns x 4 row-slices per block; grid
// (ceil(cols/64), row chunks); one atomicAdd per (column, block).
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ X, int64_t rows,
                                                     int64_t cols, int64_t ldx, int64_t rchunk,
                                                     float* __restrict__ out) {
  __shared__ float part[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sl = threadIdx.x >> 6;
  const int64_t r0 = blockIdx.y * rchunk;
  const int64_t r1 = min(rows, r0 + rchunk);
  float s = 0.f;
  if (c < cols)
    for (int64_t r = r0 + sl; r < r1; r += 4) s += X[r * ldx + c];
  part[sl][threadIdx.x & 63] = s;
  __syncthreads();
  if (sl == 0 && c < cols) {
    s = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
    atomicAdd(&out[c], s);
  }
}
}  // namespace savqa

extern "C" int savqa_colsum_acc(void* stream, const float* X, int64_t rows, int64_t cols,
                                int64_t ldx, float* out) {
  if (rows <= 0 || cols <= 0) return 0;
  const int64_t cb = (cols + 63) / 64;
  int64_t chunks = (2048 + cb - 1) / cb;
  int64_t rchunk = (rows + chunks - 1) / chunks;
  if (rchunk < 64) rchunk = 64;
  chunks = (rows + rchunk - 1) / rchunk;
  hipLaunchKernelGGL(colsum_kernel, dim3(cb, chunks), dim3(256), 0, as_stream(stream), X, rows,
                     cols, ldx, rchunk, out);
  return check_launch("savqa_colsum_acc");
}
