// fp32 GEMM on gfx950 matrix cores (v_mfma_f32_16x16x4_f32: exact f32, 64 FLOP/clk/SIMD).
//
// Replaces every nn.Linear of the SA-VQA model_v=3 path and the two backward GEMMs of
// each (dX = dY W, dW = dY^T X). One kernel template covers the operand layouts:
//   forward  C = X W^T        A [M][K] (a_trans=0), B [N][K] (b_trans=1)
//   dX       C = dY W         A [M][K] (a_trans=0), B [K][N] (b_trans=0)
//   dW      C += dY^T X       A [K][M] (a_trans=1), B [K][N] (b_trans=0), split-K + atomics
// Fused epilogues: bias, periodic row vector (learned position table), residual,
// ReLU, row scale, ReLU-backward mask, beta-accumulate, atomic scatter to indexed rows
// (embedding-table gradient) -- see include/savqa.h for the exact formula.
//
// Tiling: 256 threads = 4 waves (2x2), block tile 128x128, BK 16.
// Each operand tile keeps its global orientation in LDS, so every global->LDS move is a
// float4 load + one ds_write_b128 (no transposition):
//   ROW operand (k contiguous: X, W of the forward, dY of dX) -> LDS [m][BK+4]; the
//     MFMA's 2-wide k slot is fed from ONE ds_read_b128 per 8 k: lane half q reads
//     k = 8c+4q .. 8c+4q+3 and four successive MFMAs consume its 4 values (k order
//     permuted consistently for A and B; +4-float row pad = conflict-free b128 reads);
//   COL operand (m contiguous: W of dX, dY^T / X of dW) -> LDS [k][m+4], ds_read_b32 of
//     32 consecutive floats per half-wave in the same permuted k order.
// Interior tiles run a branch-free loop (row pointers resolved once per block, gathers
// included); edge tiles, k tails and k-row gathers take a clamped, branch-free guarded
// loader. One register-staged prefetch, LDS write after the barrier (forward, dX) or
// after the compute (dW) -- see gemm_t14 --, one barrier
// per k-tile, XCD-aware block order (T1).
#include "gemm_common.h"

#include <algorithm>

namespace savqa {

// Workgroups (= waves per SIMD) per CU the launch bounds ask for (VGPRs capped at 512 / OCC;
// 40 KB of LDS per workgroup admits 3), and the slots per CU the launch planner counts per
// round (split-K factors, the tail split of the last partial round).
#ifndef SAVQA_GEMM_OCC
#define SAVQA_GEMM_OCC 3
#endif
#ifndef SAVQA_GEMM_PLAN_OCC
#define SAVQA_GEMM_PLAN_OCC 3
#endif
#ifndef SAVQA_GEMM_CU_TAIL
#define SAVQA_GEMM_CU_TAIL 1
#endif
constexpr int GEMM_OCC = SAVQA_GEMM_OCC;
constexpr int GEMM_PLAN_OCC = SAVQA_GEMM_PLAN_OCC;
constexpr int GEMM_BK = 16;   // k-tile; 16 beats 32 on the K=512 step shapes (shorter prologue)
constexpr int GEMM_BK_DW = 16;  // k-tile of the dW layouts (A = dY^T, K = B*T rows); 32 no better


// MFMA of the 128x128 path: v_mfma_f32_16x16x4_f32 (fp32 in, fp32 accumulate, 64
// FLOP/clk/SIMD), 16-row fragments, 4 accumulator VGPRs each. A fragment's operand lane
// (i, q) feeds k = 16c + 4q + j in MFMA step j of k-chunk c (the b128 trick).
// (v_mfma_f32_32x32x2_f32 measured 5-10% slower on every cfg-2 shape: DESIGN.md 6.)
struct GemmMi {
  static constexpr int FR = 16, KCH = 16, NACC = 4;
  using Acc = f4;
  static __device__ __forceinline__ Acc mma(float a, float b, Acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int lane_i(int lane) { return lane & 15; }
  static __device__ __forceinline__ int lane_q(int lane) { return lane >> 4; }
  static __device__ __forceinline__ int row(int r, int lane) { return 4 * (lane >> 4) + r; }
  static __device__ __forceinline__ int col(int lane) { return lane & 15; }
};

template <int BMX, int BK, bool ROW>
struct Operand {
  static constexpr int LD = ROW ? BK + 4 : BMX + 4;
  static constexpr int SIZE = ROW ? BMX * LD : BK * LD;
  static constexpr int PER = ROW ? BK / 4 : BMX / 4;  // float4 per stored row
  static constexpr int ITERS = BMX * BK / 4 / GEMM_NT;
  static_assert(ITERS * GEMM_NT * 4 == BMX * BK, "tile not divisible by the block");
  f4 r[ITERS];
  const float* rp[ITERS];  // FAST path: per-float4 source pointers, resolved once per block

  // Stored row of staging slot q. ds_write_b128 serves 8 contiguous lanes per LDS cycle
  // with banks (a/4) mod 32: at BK = 16 a ROW tile row is 80 B, so two consecutive rows
  // share a 16-B slot (2-way conflict on every store); pairing rows r and r+4 in one
  // lane group makes their slots disjoint. (The ds_read_b128 fetch stays conflict-free.)
  static __device__ __forceinline__ int row_of(int q) {
    if constexpr (ROW && PER == 4)
      return (q & ~7) | ((q & 7) >> 1) | ((q & 1) << 2);
    else return q;
  }

  // ROW: stored row = m (tile row), contiguous col = k.  COL: stored row = k, col = m.
  // mlim: rows (ROW) / columns (COL) of the operand. Edge tiles clamp: a ROW operand's
  // rows past mlim re-read row mlim-1, a COL operand's float4 groups past mlim re-read the
  // last group (mlim % 4 == 0); those LDS rows / columns only reach output rows / columns
  // the epilogue never stores.
  __device__ __forceinline__ void setup_fast(const float* __restrict__ base, int64_t ld,
                                             const int64_t* __restrict__ rows, int64_t m0,
                                             int64_t mlim, int tid) {
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int idx = tid + it * GEMM_NT;
      if constexpr (ROW) {
        const int64_t m = min(m0 + row_of(idx / PER), mlim - 1);
        const int64_t rr = rows ? rows[m] : m;
        rp[it] = base + rr * ld + (idx % PER) * 4;
      } else {
        rp[it] = base + (int64_t)(idx / PER) * ld + min(m0 + (idx % PER) * 4, mlim - 4);
      }
    }
  }

  // k0: first k of the tile. ROW advances along the row, COL by whole rows.
  __device__ __forceinline__ void load_fast(int64_t ld, int64_t k0) {
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const float* p = ROW ? rp[it] + k0 : rp[it] + k0 * ld;
      r[it] = *reinterpret_cast<const f4*>(p);
    }
  }

  // k-row gathers of a COL operand (an embedding table read through the token ids of
  // a dW GEMM): setup_kg drops the row term of the pointers, load_fast_kg adds the
  // gathered row of each k per tile
  __device__ __forceinline__ void setup_kg(int64_t ld, int tid) {
    if constexpr (!ROW) {
#pragma unroll
      for (int it = 0; it < ITERS; ++it) rp[it] -= (int64_t)((tid + it * GEMM_NT) / PER) * ld;
    }
  }
  __device__ __forceinline__ void load_fast_kg(int64_t ld, const int64_t* __restrict__ rows,
                                               int64_t k0, int tid) {
    if constexpr (ROW) {
      load_fast(ld, k0);
    } else {
      int64_t rr[ITERS];
#pragma unroll
      for (int it = 0; it < ITERS; ++it) rr[it] = rows[k0 + (tid + it * GEMM_NT) / PER];
#pragma unroll
      for (int it = 0; it < ITERS; ++it) r[it] = *reinterpret_cast<const f4*>(rp[it] + rr[it] * ld);
    }
  }

  // guarded path: clamped addresses, out-of-range elements selected to 0 (branch-free)
  __device__ __forceinline__ void load_slow(const float* __restrict__ base, int64_t ld,
                                            const int64_t* __restrict__ rows, int64_t mlim,
                                            int64_t m0, int64_t k0, int64_t kend, int tid) {
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int idx = tid + it * GEMM_NT;
      int64_t row, col, rlim, clim;
      if constexpr (ROW) {
        row = m0 + row_of(idx / PER);
        col = k0 + (idx % PER) * 4;
        rlim = mlim;
        clim = kend;
      } else {
        row = k0 + idx / PER;
        col = m0 + (idx % PER) * 4;
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

  __device__ __forceinline__ void accum(f4 (&cs)[ITERS]) const {
#pragma unroll
    for (int it = 0; it < ITERS; ++it) cs[it] += r[it];
  }

  __device__ __forceinline__ void store(float* __restrict__ s, int tid) const {
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int idx = tid + it * GEMM_NT;
      *reinterpret_cast<f4*>(&s[row_of(idx / PER) * LD + (idx % PER) * 4]) = r[it];
    }
  }

  // MFMA operand values of k-chunk c (MI::KCH wide) for fragment rows [f*FR, f*FR+FR) of
  // this wave's sub-tile (wbase): v[j] feeds MFMA step j (k = KCH*c + 4*q + j).
  template <class MI>
  static __device__ __forceinline__ void fetch(const float* __restrict__ s, int wbase, int f,
                                               int c, int lane, float (&v)[4]) {
    const int q = MI::lane_q(lane), i = MI::lane_i(lane);
    if constexpr (ROW) {
      const f4 t = *reinterpret_cast<const f4*>(&s[(wbase + f * MI::FR + i) * LD + c * MI::KCH + 4 * q]);
      v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = s[(c * MI::KCH + 4 * q + j) * LD + wbase + f * MI::FR + i];
    }
  }
};

template <int BM, int BN, int BK, bool AT, bool BT>
struct GemmCfg {
  using OA = Operand<BM, BK, !AT>;
  using OB = Operand<BN, BK, BT>;
  using MI = GemmMi;
  using Acc = typename MI::Acc;
  static constexpr int WM = BM / 2, WN = BN / 2;
  static constexpr int FM = WM / MI::FR, FN = WN / MI::FR;
};

template <int BM, int BN, int BK, bool AT, bool BT>
__device__ __forceinline__ void gemm_compute_tile(
    const float* __restrict__ As, const float* __restrict__ Bs, int wm, int wn, int lane,
    typename GemmCfg<BM, BN, BK, AT, BT>::Acc (&acc)[GemmCfg<BM, BN, BK, AT, BT>::FM][GemmCfg<BM, BN, BK, AT, BT>::FN]) {
  using G = GemmCfg<BM, BN, BK, AT, BT>;
  using MI = typename G::MI;
  constexpr int NC = BK / MI::KCH;
  // operands of k-chunk c+1 are read from LDS while chunk c's MFMAs run
  float a[2][G::FM][4], b[2][G::FN][4];
#pragma unroll
  for (int i = 0; i < G::FM; ++i) G::OA::template fetch<MI>(As, wm * G::WM, i, 0, lane, a[0][i]);
#pragma unroll
  for (int j = 0; j < G::FN; ++j) G::OB::template fetch<MI>(Bs, wn * G::WN, j, 0, lane, b[0][j]);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int cur = c & 1;
    if (c + 1 < NC) {
#pragma unroll
      for (int i = 0; i < G::FM; ++i) G::OA::template fetch<MI>(As, wm * G::WM, i, c + 1, lane, a[cur ^ 1][i]);
#pragma unroll
      for (int j = 0; j < G::FN; ++j) G::OB::template fetch<MI>(Bs, wn * G::WN, j, c + 1, lane, b[cur ^ 1][j]);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < G::FM; ++i)
#pragma unroll
        for (int j = 0; j < G::FN; ++j)
          acc[i][j] = MI::mma(a[cur][i][s], b[cur][j][s], acc[i][j]);
  }
}

// k-loop order. Measured (tools/gemm_bench.py, cfg-2 shapes): storing the staged tile
// right after the barrier (T14) is +1-4% on the k-contiguous-A layouts (forward, dX) and
// -1..-4% on dW (A = dY^T, m-contiguous), so dW keeps the store-after-compute order.
template <bool AT>
__host__ __device__ constexpr bool gemm_t14() { return !AT; }

// k-loop load mode of a block (block-uniform): 0 = guarded loads everywhere (unaligned
// operands, odd edge widths), 1 = branch-free loads on every k-tile, 2 = branch-free
// except a guarded last k-tile (K not a multiple of BK, e.g. the 300-d GloVe
// projections), 3 = as 2 with k-row gathers (the GloVe-table dW: rows by token id).
template <int BM, int BN, int BK, bool AT, bool BT>
__device__ __forceinline__ int gemm_mode(const savqa_gemm_desc& d, int64_t m0, int64_t n0,
                                         int64_t kbeg, int64_t kend, int avec, int bvec) {
  const bool a_kgather = AT && d.a_rows;
  const bool b_kgather = !BT && d.b_rows;
  if (!avec || !bvec) return 0;
  if (m0 + BM > d.M && AT && (d.M & 3)) return 0;   // COL edge needs whole float4 groups
  if (n0 + BN > d.N && !BT && (d.N & 3)) return 0;
  if (a_kgather || b_kgather) return 3;
  return ((kend - kbeg) % BK == 0) ? 1 : 2;
}

template <int BM, int BN, int BK, bool AT, bool BT, int MODE>
__device__ __forceinline__ void gemm_mainloop(
    const savqa_gemm_desc& d, float* smem, int64_t m0, int64_t n0, int64_t kbeg, int64_t kend,
    int ntiles,
    typename GemmCfg<BM, BN, BK, AT, BT>::Acc (&acc)[GemmCfg<BM, BN, BK, AT, BT>::FM][GemmCfg<BM, BN, BK, AT, BT>::FN],
    bool do_cs, f4 (&cs)[GemmCfg<BM, BN, BK, AT, BT>::OA::ITERS]) {
  using G = GemmCfg<BM, BN, BK, AT, BT>;
  using OA = typename G::OA;
  using OB = typename G::OB;
  OA la;
  OB lb;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const bool agk = AT && d.a_rows, bgk = !BT && d.b_rows;  // MODE 3: k-row gathers
  if constexpr (MODE != 0) {
    la.setup_fast(d.A, d.lda, AT ? nullptr : d.a_rows, m0, d.M, tid);
    lb.setup_fast(d.B, d.ldb, BT ? d.b_rows : nullptr, n0, d.N, tid);
    if (MODE == 3 && agk) la.setup_kg(d.lda, tid);
    if (MODE == 3 && bgk) lb.setup_kg(d.ldb, tid);
  }
#define SAVQA_GEMM_LOAD(k0)                                          \
  do {                                                               \
    const int64_t k0_ = (k0);                                        \
    if (MODE == 1 || (MODE == 2 && k0_ + BK <= kend)) {              \
      la.load_fast(d.lda, k0_);                                      \
      lb.load_fast(d.ldb, k0_);                                      \
    } else if (MODE == 3 && k0_ + BK <= kend) {                      \
      if (agk) la.load_fast_kg(d.lda, d.a_rows, k0_, tid);           \
      else la.load_fast(d.lda, k0_);                                 \
      if (bgk) lb.load_fast_kg(d.ldb, d.b_rows, k0_, tid);           \
      else lb.load_fast(d.ldb, k0_);                                 \
    } else {                                                         \
      la.load_slow(d.A, d.lda, d.a_rows, d.M, m0, k0_, kend, tid);   \
      lb.load_slow(d.B, d.ldb, d.b_rows, d.N, n0, k0_, kend, tid);   \
    }                                                                \
  } while (0)
  SAVQA_GEMM_LOAD(kbeg);
  if (do_cs) la.accum(cs);  // colsum_a: the staged A tile summed over its k rows
  la.store(smem, tid);
  lb.store(smem + 2 * OA::SIZE, tid);
  if constexpr (gemm_t14<AT>()) {
  // write-after-barrier order: per k-tile  barrier -> store tile t+1 (its loads landed
  // during compute t-1) -> issue loads of t+2 -> compute t
  if (ntiles > 1) SAVQA_GEMM_LOAD(kbeg + BK);
  for (int tt = 0; tt < ntiles; ++tt) {
    __syncthreads();
    const int cur = tt & 1;
    if (tt + 1 < ntiles) {
      if (do_cs) la.accum(cs);
      la.store(smem + (cur ^ 1) * OA::SIZE, tid);
      lb.store(smem + 2 * OA::SIZE + (cur ^ 1) * OB::SIZE, tid);
      if (tt + 2 < ntiles) SAVQA_GEMM_LOAD(kbeg + (int64_t)(tt + 2) * BK);
    }
    gemm_compute_tile<BM, BN, BK, AT, BT>(smem + cur * OA::SIZE,
                                          smem + 2 * OA::SIZE + cur * OB::SIZE, wm, wn, lane,
                                          acc);
  }
  __syncthreads();  // the caller's epilogue helpers reuse smem
  } else {
  __syncthreads();
  int cur = 0;
  for (int tt = 0; tt < ntiles; ++tt) {
    const bool more = tt + 1 < ntiles;
    if (more) SAVQA_GEMM_LOAD(kbeg + (int64_t)(tt + 1) * BK);
    gemm_compute_tile<BM, BN, BK, AT, BT>(smem + cur * OA::SIZE,
                                          smem + 2 * OA::SIZE + cur * OB::SIZE, wm, wn, lane,
                                          acc);
    if (more) {
      if (do_cs) la.accum(cs);
      la.store(smem + (cur ^ 1) * OA::SIZE, tid);
      lb.store(smem + 2 * OA::SIZE + (cur ^ 1) * OB::SIZE, tid);
    }
    __syncthreads();
    cur ^= 1;
  }
  }
#undef SAVQA_GEMM_LOAD
}

// colsum_a fold (bias gradient of a dW GEMM): every thread's staged-A partials share one
// column group q = tid % PER (GEMM_NT is a multiple of PER); rows of threads write plain
// LDS rows and one thread per column sums them (LDS float atomics serialise: ~us per block)
template <int PER, int ITERS, int BM>
__device__ __forceinline__ void cs_fold(const f4 (&cs)[ITERS], float* smem, int64_t m0,
                                        const savqa_gemm_desc& d, float* slab_cs) {
  static_assert(GEMM_NT % PER == 0 && 4 * PER == BM, "colsum layout");
  constexpr int ROWS = GEMM_NT / PER;
  f4 t = cs[0];
#pragma unroll
  for (int it = 1; it < ITERS; ++it) t += cs[it];
  __syncthreads();
  *reinterpret_cast<f4*>(&smem[(threadIdx.x / PER) * BM + 4 * (threadIdx.x % PER)]) = t;
  __syncthreads();
  for (int i = threadIdx.x; i < BM; i += GEMM_NT) {
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) v += smem[r * BM + i];
    if (m0 + i < d.M) {
      if (slab_cs) slab_cs[m0 + i] = v;  // slab mode: this slice's row of column sums
      else atomicAdd(&d.colsum_a[m0 + i], v);
    }
  }
}

template <int BM, int BN, int BK, bool AT, bool BT>
__global__ __launch_bounds__(GEMM_NT, GEMM_OCC) __attribute__((amdgpu_waves_per_eu(GEMM_OCC, GEMM_OCC))) void gemm_f32_kernel(savqa_gemm_desc d, GemmGrid gg,
                                                             int avec, int bvec) {
  using G = GemmCfg<BM, BN, BK, AT, BT>;
  constexpr int FM = G::FM, FN = G::FN, WM = G::WM, WN = G::WN;
  __shared__ __attribute__((aligned(16))) float smem[2 * (G::OA::SIZE + G::OB::SIZE)];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int bid = blockIdx.x;
  int t, slice;
  int64_t kbeg, kend;
  bool first_split, atomic;
  float* slab = nullptr;  // slab mode (GemmGrid): this block's partial-tile slab
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
  const int tn = t % gg.tiles_n;
  const int tm = t / gg.tiles_n;
  const int64_t m0 = (int64_t)tm * BM;
  const int64_t n0 = (int64_t)tn * BN;

  using MI = typename G::MI;
  typename G::Acc acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < MI::NACC; ++r) acc[i][j][r] = 0.f;

  const int mode = gemm_mode<BM, BN, BK, AT, BT>(d, m0, n0, kbeg, kend, avec, bvec);
  const int ntiles = kend > kbeg ? (int)((kend - kbeg + BK - 1) / BK) : 0;
  // colsum_a (a_trans only): column tile 0 also sums its A tiles over k (bias gradient)
  const bool do_cs = AT && d.colsum_a != nullptr && tn == 0;
  f4 cs[G::OA::ITERS];
#pragma unroll
  for (int it = 0; it < G::OA::ITERS; ++it) cs[it] = f4{0.f, 0.f, 0.f, 0.f};
  if (ntiles > 0) {
    if (mode == 1)
      gemm_mainloop<BM, BN, BK, AT, BT, 1>(d, smem, m0, n0, kbeg, kend, ntiles, acc, do_cs, cs);
    else if (mode == 2)
      gemm_mainloop<BM, BN, BK, AT, BT, 2>(d, smem, m0, n0, kbeg, kend, ntiles, acc, do_cs, cs);
    else if (mode == 3)
      gemm_mainloop<BM, BN, BK, AT, BT, 3>(d, smem, m0, n0, kbeg, kend, ntiles, acc, do_cs, cs);
    else
      gemm_mainloop<BM, BN, BK, AT, BT, 0>(d, smem, m0, n0, kbeg, kend, ntiles, acc, do_cs, cs);
  }
  if constexpr (AT) {
    if (do_cs) {  // block-uniform; smem is free after the main loop's last barrier
      cs_fold<G::OA::PER, G::OA::ITERS, BM>(cs, smem, m0, d,
                                            gg.slab_cs ? gg.slab_cs + slice * d.M : nullptr);
    }
  }

  // ---------------------------------------------------------------- epilogue
  static_assert(MI::FR == 16 && MI::NACC == 4, "16x16 accumulator layout");
  gemm_epilogue16<FM, FN, WM, WN>(d, acc, m0, n0, wm, wn, lane, first_split, atomic, slab,
                                  gg.slab_r0);
}

// ---------------------------------------------------------------------------------------
// Small-M / small-N GEMMs (the decoder and head Linears at M = B = 256 rows, their dW at
// K = 256): one 32x32 output tile per 512-thread workgroup, the 8 waves split K eight ways
// and fold their accumulators through LDS, so a 256x512x512 GEMM runs as 128 workgroups of
// 8 short MFMA chains instead of 32 workgroups of one long one. Operands go straight from
// global memory (L2) into MFMA registers: lane half q of an 8-k group takes k = 8g+4q+s,
// s = 0..3 -- one b128 load on a k-contiguous operand, 4 coalesced scalars otherwise.
constexpr int SK_WAVES = 8;
constexpr int SK_DEPTH = 2;  // 4 and 8 measured no faster

template <bool KCONTIG>
__device__ __forceinline__ void sk_load4(const float* __restrict__ P, int64_t ld,
                                         const int64_t* __restrict__ rows, int64_t x, int64_t xlim,
                                         int64_t k, int64_t kend, bool vec, float (&v)[4]) {
  // KCONTIG: value(x, k) = P[r(x)*ld + k]; else value(x, k) = P[r(k)*ld + x]
  if constexpr (KCONTIG) {
    const bool xok = x < xlim;
    const int64_t rx = xok ? (rows ? rows[x] : x) : 0;
    const float* p = P + rx * ld;
    if (vec && xok && k + 3 < kend) {
      const f4 t = *reinterpret_cast<const f4*>(p + k);
      v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = xok && k + j < kend;
        const float t = p[ok ? k + j : 0];
        v[j] = ok ? t : 0.f;
      }
    }
  } else {
    const bool xok = x < xlim;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool ok = xok && k + j < kend;
      const int64_t kk = ok ? k + j : 0;
      const int64_t rk = rows ? rows[kk] : kk;
      const float t = P[rk * ld + (xok ? x : 0)];
      v[j] = ok ? t : 0.f;
    }
  }
}

// Branch-free loads of whole k-groups (every k in range, the lane's row / column clamped to a
// valid one and its values masked at use): the guarded sk_load4 above branches per element,
// and hipcc then waits vmcnt(0) at every join -- it serialised the skinny kernels' loads
// (63-75 s_waitcnt vmcnt(0) per kernel body, one global round trip per load). The guarded
// form now only runs the (at most one) partial group at the end of K.
//   KCONTIG: value(x, k) = base[k] with base = P + r(x) * ld (VEC: one b128 load)
//   else:    value(x, k) = base[k * ld] with base = P + x (4 coalesced scalars)
template <bool KCONTIG, bool VEC>
__device__ __forceinline__ void sk_full4(const float* __restrict__ base, int64_t ld, int64_t k,
                                         float (&v)[4]) {
  if constexpr (KCONTIG) {
    if constexpr (VEC) {
      const f4 t = *reinterpret_cast<const f4*>(base + k);
      v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = base[k + j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = base[(k + j) * ld];
  }
}

// D-slot register ring over ng whole k-groups starting at g0: a steady loop whose body is
// straight-line (every slot's MFMAs, then its reload D groups ahead), so hipcc's counted
// vmcnt waits for exactly the slot it consumes; guards only in the drain. Fewer than D
// groups: all loads first, then the MFMAs (one round trip).
template <int D, int W, class LD, class MM>
__device__ __forceinline__ void sk_ring(int64_t g0, int ng, float (&a)[D][W], float (&b)[D][W],
                                        LD&& load, MM&& mma) {
  if (ng >= D) {
#pragma unroll
    for (int u = 0; u < D; ++u) load(g0 + u, a[u], b[u]);
    int it = 0;
    for (; it + 2 * D <= ng; it += D) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        mma(a[u], b[u]);
        load(g0 + it + D + u, a[u], b[u]);
        // keep slot order: left alone, the scheduler hoists every MFMA above every reload
        // and the loop then waits vmcnt(0) at its head
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int u = 0; u < D; ++u) {
      mma(a[u], b[u]);
      if (it + D + u < ng) load(g0 + it + D + u, a[u], b[u]);
    }
#pragma unroll
    for (int u = 0; u < D; ++u)
      if (it + D + u < ng) mma(a[u], b[u]);
  } else {
#pragma unroll
    for (int u = 0; u < D; ++u)
      if (u < ng) load(g0 + u, a[u], b[u]);
#pragma unroll
    for (int u = 0; u < D; ++u)
      if (u < ng) mma(a[u], b[u]);
  }
}

// per-lane operand base of sk_full4 (row / column clamped into range)
template <bool KCONTIG>
__device__ __forceinline__ const float* sk_base(const float* P, int64_t ld,
                                                const int64_t* __restrict__ rows, int64_t x,
                                                int64_t xlim) {
  const int64_t xc = x < xlim ? x : xlim - 1;
  if constexpr (KCONTIG) return P + (rows ? rows[xc] : xc) * ld;
  else return P + xc;
}

template <bool AT, bool BT, int NW, bool AV, bool BV>
__global__ __launch_bounds__(64 * NW) void gemm_skinny_kernel(savqa_gemm_desc d, int tiles_n,
                                                                   int avec, int bvec) {
  __shared__ float red[NW][32][33];
  // the wave index in an SGPR: every k-range bound below is then wave-uniform to the
  // compiler, so the ring's guards are scalar branches, not exec masks (an exec-masked guard
  // makes hipcc wait vmcnt(0) at its join and serialises the loads)
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = blockIdx.x;
  const int64_t m0 = (int64_t)(t / tiles_n) * 32, n0 = (int64_t)(t % tiles_n) * 32;
  // this wave's k range, in whole 8-k groups
  const int64_t ngrp = (d.K + 7) / 8;
  const int64_t g0 = ngrp * w / NW, g1 = ngrp * (w + 1) / NW;
  const int64_t gf = min(g1, max(g0, d.K / 8));  // [g0, gf): groups wholly inside K
  const int i = lane & 31, q = lane >> 5;
  const int64_t am = m0 + i, bn = n0 + i;
  const int64_t* arows = d.a_rows;  // !AT: gather on m; AT: gather on k
  const int64_t* brows = d.b_rows;  // BT: gather on n; !BT: gather on k
  // k-row gathers (AT a_rows / !BT b_rows) keep the guarded per-element loads
  const bool kgather = (AT && arows) || (!BT && brows);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float cs = 0.f;  // colsum_a partial (AT): sum over this wave's k of A(m0 + i, k), half q
  // out-of-range rows / columns (clamped loads) contribute zeros: masked here, at the use,
  // so no load result is needed before the MFMA that consumes it
  const bool aok = am < d.M, bok = bn < d.N;
  auto mma = [&](const float (&aa)[4], const float (&bb)[4]) {
    float x[4], y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = aok ? aa[j] : 0.f;
      y[j] = bok ? bb[j] : 0.f;
    }
    cs += (x[0] + x[1]) + (x[2] + x[3]);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[s], y[s], acc, 0, 0, 0);
  };
  if (!kgather) {
    const float* ab = sk_base<!AT>(d.A, d.lda, AT ? nullptr : arows, am, d.M);
    const float* bb_ = sk_base<BT>(d.B, d.ldb, BT ? brows : nullptr, bn, d.N);
    constexpr int D = 4;  // k-groups in flight per wave (a ring of compile-time slots)
    float a[D][4], b[D][4];
    auto load = [&](int64_t g, float (&aa)[4], float (&bx)[4]) {
      const int64_t k = g * 8 + 4 * q;
      sk_full4<!AT, AV>(ab, d.lda, k, aa);
      sk_full4<BT, BV>(bb_, d.ldb, k, bx);
    };
    sk_ring<D>(g0, (int)(gf - g0), a, b, load, mma);
    if (gf < g1) {  // the partial group at the end of K (one wave at most)
      float aa[4], bx[4];
      const int64_t k = gf * 8 + 4 * q;
      sk_load4<!AT>(d.A, d.lda, arows, am, d.M, k, d.K, avec, aa);
      sk_load4<BT>(d.B, d.ldb, brows, bn, d.N, k, d.K, bvec, bx);
      mma(aa, bx);
    }
  } else {
    float a[SK_DEPTH][2][4], b[SK_DEPTH][2][4];
    auto load_pair = [&](int64_t gg, float (&aa)[2][4], float (&bb)[2][4]) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t k = (gg + u) * 8 + 4 * q;
        const int64_t kl = gg + u < g1 ? d.K : 0;  // groups past this wave's range load zeros
        sk_load4<!AT>(d.A, d.lda, arows, am, d.M, k, kl, avec, aa[u]);
        sk_load4<BT>(d.B, d.ldb, brows, bn, d.N, k, kl, bvec, bb[u]);
      }
    };
    const int npair = (int)((g1 - g0 + 1) / 2);
#pragma unroll
    for (int q2 = 0; q2 < SK_DEPTH; ++q2)
      if (q2 < npair) load_pair(g0 + 2 * q2, a[q2], b[q2]);
    for (int pi = 0; pi < npair; pi += SK_DEPTH) {
#pragma unroll
      for (int q2 = 0; q2 < SK_DEPTH; ++q2) {
        if (pi + q2 < npair) {
          mma(a[q2][0], b[q2][0]);
          mma(a[q2][1], b[q2][1]);
          if (pi + q2 + SK_DEPTH < npair) load_pair(g0 + 2 * (pi + q2 + SK_DEPTH), a[q2], b[q2]);
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[w][(r & 3) + 8 * (r >> 2) + 4 * q][i] = acc[r];
  __syncthreads();
  const bool ident = d.c_rows == nullptr && d.c_group >= d.M && d.c_offset == 0;
  for (int e = threadIdx.x; e < 32 * 32; e += 64 * NW) {
    const int r = e >> 5, c = e & 31;
    const int64_t m = m0 + r, n = n0 + c;
    if (m >= d.M || n >= d.N) continue;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += red[ww][r][c];
    const EpiRow er = epi_row(d, m, ident);
    epi_store(d, er, m, n, v, true, d.atomic != 0);
  }
  if constexpr (AT) {
    if (d.colsum_a && n0 == 0) {
      __syncthreads();
      float* flat = &red[0][0][0];
      flat[threadIdx.x] = cs;  // 64 * NW partials: (wave, half q, i)
      __syncthreads();
      if (threadIdx.x < 32 && m0 + threadIdx.x < d.M) {
        float sum = 0.f;
        for (int j = 0; j < 2 * NW; ++j) sum += flat[j * 32 + threadIdx.x];
        atomicAdd(&d.colsum_a[m0 + threadIdx.x], sum);
      }
    }
  }
}

// bf16-product variant of gemm_skinny_kernel (savqa_gemm_desc.prec = 1: the low-precision
// modes' decoder / head Linears at M = B rows, whose operands are fp32 activations): the same
// 32x32 tile, K split over the 8 waves and LDS fold, but groups of 16 k -- lane half q takes
// k = 16g + 8q .. +7 of its row (two b128 loads on a k-contiguous operand), rounds them to
// bf16 (RNE, autocast's rounding of a Linear's operands) and issues ONE
// v_mfma_f32_32x32x16_bf16 per group instead of eight v_mfma_f32_32x32x2_f32 (32 against 512
// SIMD cycles); fp32 accumulation, the fp32 epilogue. The bias-gradient column sums (AT) add
// the fp32 values.
template <bool AT, bool BT, int NW, bool AV, bool BV>
__global__ __launch_bounds__(64 * NW) void gemm_skinny_bf_kernel(savqa_gemm_desc d, int tiles_n,
                                                                 int avec, int bvec) {
  typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
  __shared__ float red[NW][32][33];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = blockIdx.x;
  const int64_t m0 = (int64_t)(t / tiles_n) * 32, n0 = (int64_t)(t % tiles_n) * 32;
  const int64_t ngrp = (d.K + 15) / 16;
  const int64_t g0 = ngrp * w / NW, g1 = ngrp * (w + 1) / NW;
  const int64_t gf = min(g1, max(g0, d.K / 16));  // [g0, gf): groups wholly inside K
  const int i = lane & 31, q = lane >> 5;
  const int64_t am = m0 + i, bn = n0 + i;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float cs = 0.f;
  const bool aok = am < d.M, bok = bn < d.N;
  auto mma = [&](const float (&aa)[8], const float (&bb)[8]) {
    bfx8 x, y;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xa = aok ? aa[j] : 0.f;
      cs += xa;
      x[j] = (__bf16)xa;
      y[j] = (__bf16)(bok ? bb[j] : 0.f);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, acc, 0, 0, 0);
  };
  const float* ab = sk_base<!AT>(d.A, d.lda, AT ? nullptr : d.a_rows, am, d.M);
  const float* bb_ = sk_base<BT>(d.B, d.ldb, BT ? d.b_rows : nullptr, bn, d.N);
  constexpr int D = 4;
  float a[D][8], b[D][8];
  auto load = [&](int64_t g, float (&aa)[8], float (&bx)[8]) {
    const int64_t k = g * 16 + 8 * q;
    float t4[4];
    sk_full4<!AT, AV>(ab, d.lda, k, t4);
    aa[0] = t4[0]; aa[1] = t4[1]; aa[2] = t4[2]; aa[3] = t4[3];
    sk_full4<!AT, AV>(ab, d.lda, k + 4, t4);
    aa[4] = t4[0]; aa[5] = t4[1]; aa[6] = t4[2]; aa[7] = t4[3];
    sk_full4<BT, BV>(bb_, d.ldb, k, t4);
    bx[0] = t4[0]; bx[1] = t4[1]; bx[2] = t4[2]; bx[3] = t4[3];
    sk_full4<BT, BV>(bb_, d.ldb, k + 4, t4);
    bx[4] = t4[0]; bx[5] = t4[1]; bx[6] = t4[2]; bx[7] = t4[3];
  };
  sk_ring<D>(g0, (int)(gf - g0), a, b, load, mma);
  if (gf < g1) {  // the partial group at the end of K (one wave at most)
    float aa[8], bx[8], t4[4];
    const int64_t k = gf * 16 + 8 * q;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      sk_load4<!AT>(d.A, d.lda, d.a_rows, am, d.M, k + 4 * h, d.K, avec, t4);
#pragma unroll
      for (int j = 0; j < 4; ++j) aa[4 * h + j] = t4[j];
      sk_load4<BT>(d.B, d.ldb, d.b_rows, bn, d.N, k + 4 * h, d.K, bvec, t4);
#pragma unroll
      for (int j = 0; j < 4; ++j) bx[4 * h + j] = t4[j];
    }
    mma(aa, bx);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[w][(r & 3) + 8 * (r >> 2) + 4 * q][i] = acc[r];
  __syncthreads();
  const bool ident = d.c_rows == nullptr && d.c_group >= d.M && d.c_offset == 0;
  for (int e = threadIdx.x; e < 32 * 32; e += 64 * NW) {
    const int r = e >> 5, c = e & 31;
    const int64_t m = m0 + r, n = n0 + c;
    if (m >= d.M || n >= d.N) continue;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += red[ww][r][c];
    const EpiRow er = epi_row(d, m, ident);
    epi_store(d, er, m, n, v, true, d.atomic != 0);
  }
  if constexpr (AT) {
    if (d.colsum_a && n0 == 0) {
      __syncthreads();
      float* flat = &red[0][0][0];
      flat[threadIdx.x] = cs;  // 64 * NW partials: (wave, half q, i)
      __syncthreads();
      if (threadIdx.x < 32 && m0 + threadIdx.x < d.M) {
        float sum = 0.f;
        for (int j = 0; j < 2 * NW; ++j) sum += flat[j * 32 + threadIdx.x];
        atomicAdd(&d.colsum_a[m0 + threadIdx.x], sum);
      }
    }
  }
}

// 16x16-tile variant (v_mfma_f32_16x16x4_f32) for the skinny shapes with too few 32x32
// tiles to fill the chip (a 256x512 output is 128 32x32 tiles for 256 CUs, 512 16x16
// ones): same K split over the waves and LDS fold. Lane (i, q) = (lane % 16, lane / 16)
// takes k = 16g + 4q + s in MFMA step s of 16-k group g: one b128 load on a k-contiguous
// operand, 4 coalesced scalars otherwise; accumulator row 4q + r, column i.
constexpr int SK16_DEPTH = 4;

template <bool AT, bool BT, int NW, bool AV, bool BV>
__global__ __launch_bounds__(64 * NW) void gemm_skinny16_kernel(savqa_gemm_desc d,
                                                                     int tiles_n, int avec,
                                                                     int bvec) {
  __shared__ float red[NW][16][17];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = blockIdx.x;
  const int64_t m0 = (int64_t)(t / tiles_n) * 16, n0 = (int64_t)(t % tiles_n) * 16;
  const int64_t ngrp = (d.K + 15) / 16;
  const int64_t g0 = ngrp * w / NW, g1 = ngrp * (w + 1) / NW;
  const int64_t gf = min(g1, max(g0, d.K / 16));  // [g0, gf): groups wholly inside K
  const int i = lane & 15, q = lane >> 4;
  const int64_t am = m0 + i, bn = n0 + i;
  const bool kgather = (AT && d.a_rows) || (!BT && d.b_rows);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  float cs = 0.f;
  const bool aok = am < d.M, bok = bn < d.N;  // clamped loads masked at the use
  auto mma = [&](const float (&aa)[4], const float (&bb)[4]) {
    float x[4], y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = aok ? aa[j] : 0.f;
      y[j] = bok ? bb[j] : 0.f;
    }
    cs += (x[0] + x[1]) + (x[2] + x[3]);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[s], y[s], acc, 0, 0, 0);
  };
  auto load_guarded = [&](int64_t gg, float (&aa)[4], float (&bb)[4]) {
    const int64_t k = gg * 16 + 4 * q;
    sk_load4<!AT>(d.A, d.lda, d.a_rows, am, d.M, k, d.K, avec, aa);
    sk_load4<BT>(d.B, d.ldb, d.b_rows, bn, d.N, k, d.K, bvec, bb);
  };
  if (!kgather) {
    const float* ab = sk_base<!AT>(d.A, d.lda, AT ? nullptr : d.a_rows, am, d.M);
    const float* bb_ = sk_base<BT>(d.B, d.ldb, BT ? d.b_rows : nullptr, bn, d.N);
    float a[SK16_DEPTH][4], b[SK16_DEPTH][4];
    auto load = [&](int64_t gg, float (&aa)[4], float (&bx)[4]) {
      const int64_t k = gg * 16 + 4 * q;
      sk_full4<!AT, AV>(ab, d.lda, k, aa);
      sk_full4<BT, BV>(bb_, d.ldb, k, bx);
    };
    sk_ring<SK16_DEPTH>(g0, (int)(gf - g0), a, b, load, mma);
    if (gf < g1) {
      float aa[4], bx[4];
      load_guarded(gf, aa, bx);
      mma(aa, bx);
    }
  } else {
    float a[SK16_DEPTH][4], b[SK16_DEPTH][4];
    const int ng = (int)(g1 - g0);
#pragma unroll
    for (int q2 = 0; q2 < SK16_DEPTH; ++q2)
      if (q2 < ng) load_guarded(g0 + q2, a[q2], b[q2]);
    for (int pi = 0; pi < ng; pi += SK16_DEPTH) {
#pragma unroll
      for (int q2 = 0; q2 < SK16_DEPTH; ++q2) {
        if (pi + q2 < ng) {
          mma(a[q2], b[q2]);
          if (pi + q2 + SK16_DEPTH < ng) load_guarded(g0 + pi + q2 + SK16_DEPTH, a[q2], b[q2]);
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[w][4 * q + r][i] = acc[r];
  __syncthreads();
  const bool ident = d.c_rows == nullptr && d.c_group >= d.M && d.c_offset == 0;
  for (int e = threadIdx.x; e < 16 * 16; e += 64 * NW) {
    const int r = e >> 4, c = e & 15;
    const int64_t m = m0 + r, n = n0 + c;
    if (m >= d.M || n >= d.N) continue;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += red[ww][r][c];
    const EpiRow er = epi_row(d, m, ident);
    epi_store(d, er, m, n, v, true, d.atomic != 0);
  }
  if constexpr (AT) {
    if (d.colsum_a && n0 == 0) {
      __syncthreads();
      float* flat = &red[0][0][0];
      flat[threadIdx.x] = cs;  // 64 * NW partials: ((wave, q), i)
      __syncthreads();
      if (threadIdx.x < 16 && m0 + threadIdx.x < d.M) {
        float sum = 0.f;
        for (int j = 0; j < 4 * NW; ++j) sum += flat[j * 16 + threadIdx.x];
        atomicAdd(&d.colsum_a[m0 + threadIdx.x], sum);
      }
    }
  }
}

// skinny launches: the operands' vector-load eligibility picks the instantiation
#define SAVQA_SK_LAUNCH(K_, AT_, BT_)                                                          \
  do {                                                                                         \
    if (avec && bvec) hipLaunchKernelGGL((K_<AT_, BT_, SK_WAVES, true, true>), g, b, 0, s, d, tn, avec, bvec);    \
    else if (avec) hipLaunchKernelGGL((K_<AT_, BT_, SK_WAVES, true, false>), g, b, 0, s, d, tn, avec, bvec);      \
    else if (bvec) hipLaunchKernelGGL((K_<AT_, BT_, SK_WAVES, false, true>), g, b, 0, s, d, tn, avec, bvec);      \
    else hipLaunchKernelGGL((K_<AT_, BT_, SK_WAVES, false, false>), g, b, 0, s, d, tn, avec, bvec);               \
  } while (0)

static int cu_count() {
  // the CU count of the current device
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    cached[dev] = cus;
  }
  return cached[dev];
}

// split-K factor minimising  rounds(s) * (k-tiles per slice + per-block overhead)
static int auto_split(int64_t tiles, int64_t K, int BK, int slots) {
  const int64_t nch = (K + BK - 1) / BK;
  int best = 1;
  int64_t best_cost = INT64_MAX;
  for (int s = 1; s <= 64 && (s == 1 || nch / s >= 8); ++s) {
    const int64_t rounds = (tiles * s + slots - 1) / slots;
    const int64_t cost = rounds * ((nch + s - 1) / s + 4);
    if (cost < best_cost) { best_cost = cost; best = s; }
  }
  return best;
}

// Launch plan: tile size, split-K, tail split (shared by savqa_gemm / savqa_gemm_plan).
struct GemmPlan {
  int tile, split;
  GemmGrid gg;
  int grid_x, nsplit;
  int64_t zero_row0;  // >= 0: rows [zero_row0, M) of C are zero-filled before the launch
  int64_t ws_need;    // slab mode: workspace floats (0: the plan does not split K / cannot)
};

// Slab mode's second pass (savqa_gemm_desc.ws): rows [r0, rows) of C get the sum of the ns
// partial slabs in slice order -- added to C (split-K: the atomic "C +=" semantics) or
// assigned (tail split: those rows are written by the tail blocks only) -- and colsum_a the
// ns rows of per-slice column sums. Four columns per thread when rows are 16-B vectors.
__global__ __launch_bounds__(256) void gemm_slab_reduce_kernel(
    float* __restrict__ C, int64_t ldc, const float* __restrict__ slab, int ns, int64_t stride,
    int64_t r0, int64_t rows, int64_t N, int accumulate, int vec, float* __restrict__ colsum,
    const float* __restrict__ slab_cs, int64_t M) {
  const int64_t nr = rows - r0;
  const int64_t per = vec ? N / 4 : N;
  const int64_t total = nr * per;
  const int64_t ncs = colsum ? M : 0;  // column sums: the last ncs work items
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total + ncs;
       u += (int64_t)gridDim.x * blockDim.x) {
    if (u >= total) {
      const int64_t m = u - total;
      float v = slab_cs[m];
      for (int s = 1; s < ns; ++s) v += slab_cs[s * M + m];
      colsum[m] += v;
      continue;
    }
    const int64_t r = u / per, c = u - r * per;
    if (vec) {
      const float* sp = slab + r * N + 4 * c;
      f4 v = *reinterpret_cast<const f4*>(sp);
      for (int s = 1; s < ns; ++s) v += *reinterpret_cast<const f4*>(sp + s * stride);
      f4* cp = reinterpret_cast<f4*>(C + (r0 + r) * ldc + 4 * c);
      *cp = accumulate ? *cp + v : v;
    } else {
      const float* sp = slab + r * N + c;
      float v = *sp;
      for (int s = 1; s < ns; ++s) v += sp[s * stride];
      float* cp = C + (r0 + r) * ldc + c;
      *cp = accumulate ? *cp + v : v;
    }
  }
}

}  // namespace savqa

using namespace savqa;

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }


// skinny shapes with fewer 32x32 tiles than this run on 16x16 tiles (measured: 256x512
// outputs (128 tiles) 1.25-1.55x faster at K=2048, 256x914 (232) slower; thresholds 192 /
// 257 / 1100 A/B'd in-step, 192 best)
constexpr int64_t SK16_MAX_TILES = 192;

// 128x128-tile launches with fewer workgroups than this (tiles x split-K slices) take the
// skinny kernels; SAVQA_SK_TILES overrides it (tuning runs)
static int64_t sk_min_tiles() {
  static int64_t v = [] {
    const char* e = getenv("SAVQA_SK_TILES");
    return e ? (int64_t)atoll(e) : (int64_t)160;
  }();
  return v;
}
// ... except tall launches (M >= SK_TALL_M, not the M = B decoder / head rows the skinny
// kernels are tuned for) with at least SK_TALL_TILES workgroups: the cfg-2 M = 3584 launches of
// 84 / 112 tiles (the question tokens' dX and GloVe-row gradients) run faster on 128 x 128
// tiles. Round 6, interleaved (profiles/r06_ab_sk_tiles.txt): a plain threshold of 80 gave
// cfg 2 7689 / 7682 -> 7749 / 7689 but cfg 5 24725 / 24674 -> 24590 / 24489 (its M = 1024
// decoder launches of 128 tiles moved too); the tall rule: cfg 2 7558 / 7646 -> 7688 / 7730,
// cfg 5 24652 / 24714 -> 24664 / 24753.
constexpr int64_t SK_TALL_M = 2048, SK_TALL_TILES = 80;
static bool sk_tiles_overridden() {
  static const bool v = getenv("SAVQA_SK_TILES") != nullptr;
  return v;
}

static int plan_gemm(savqa_gemm_desc& d, GemmPlan& p) {
  if (d.M < 0 || d.N < 0 || d.K < 0) return fail(SAVQA_EINVAL, "savqa_gemm: negative dims");
  if (d.M >= (1LL << 31) || d.N >= (1LL << 31)) return fail(SAVQA_EUNSUP, "savqa_gemm: M/N >= 2^31");
  if (d.mask && d.mask_arows && (d.a_trans || !d.a_rows))
    return fail(SAVQA_EINVAL, "savqa_gemm: mask_arows needs a_trans=0 and a_rows");
  if (d.c_group <= 0) { d.c_group = d.M; d.c_stride = d.M; }
  if (d.rowvec && d.rowvec_period <= 0) return fail(SAVQA_EINVAL, "savqa_gemm: rowvec_period");
  if (d.split_k < 0 && !d.atomic) return fail(SAVQA_EINVAL, "savqa_gemm: auto split-K needs atomic=1");
  if (d.colsum_a && !d.a_trans) return fail(SAVQA_EINVAL, "savqa_gemm: colsum_a needs a_trans=1");
  if (d.prec == 1 || d.prec == 5) d.prec = 6;  // 1: bf16 products on the skinny launches only,
                                                // 5: x6 two-level (savqa_gemm); x6 else
  if (d.prec != 0 && d.prec != 3 && d.prec != 6)
    return fail(SAVQA_EINVAL, "savqa_gemm: prec must be 0 (fp32), 1 (bf16 skinny, x6 "
                              "otherwise), 3 (3xbf16), 5 (x6 two-level) or 6 (fp32 x6)");
  // gemm_bf16_kernel / gemm_x6_kernel k-tile: 32; workgroups per CU the planner counts
  const int BK = d.prec ? 32 : (d.a_trans ? GEMM_BK_DW : GEMM_BK);
  const int occ = d.prec == 6 ? 2 : GEMM_PLAN_OCC;
  const int slots = occ * cu_count();
  const int64_t tiles128 = ((d.M + 127) / 128) * ((d.N + 127) / 128);
  int split = d.split_k > 1 ? d.split_k : 1;
  if (d.split_k < 0) split = auto_split(tiles128, d.K, BK, slots);
  // 128x128 tiles once there is enough parallelism (split-K counts), else the skinny
  // kernel (32x32 tiles, K split over the 8 waves of a workgroup; no split-K launch),
  // 16x16 tiles while 32x32 ones would leave CUs idle (< SK16_MAX_TILES tiles)
  if (tiles128 * split < sk_min_tiles() &&
      !(d.M >= SK_TALL_M && tiles128 * split >= SK_TALL_TILES && !sk_tiles_overridden())) {
    const int64_t tiles32 = ((d.M + 31) / 32) * ((d.N + 31) / 32);
    p.tile = tiles32 < SK16_MAX_TILES ? 16 : 32;
    p.split = 1;
    p.nsplit = 1;
    p.gg.tiles_n = (int)((d.N + p.tile - 1) / p.tile);
    p.grid_x = (int)((d.M + p.tile - 1) / p.tile) * p.gg.tiles_n;
    p.zero_row0 = -1;
    p.gg.tail_f = 1;
    return 0;
  }
  p.tile = 128;
  const int tm = (int)((d.M + p.tile - 1) / p.tile);
  const int tn = (int)((d.N + p.tile - 1) / p.tile);
  const int T = tm * tn;
  int64_t kchunk = (d.K + split - 1) / split;
  kchunk = (kchunk + BK - 1) / BK * BK;
  p.nsplit = kchunk > 0 ? (int)((d.K + kchunk - 1) / kchunk) : 1;
  if (p.nsplit < 1) p.nsplit = 1;
  p.split = p.nsplit;
  p.gg.tiles_n = tn;
  p.gg.kchunk = kchunk;
  p.gg.full = T;
  p.gg.tail_t0 = T;
  p.gg.tail_f = 1;
  p.gg.tail_kchunk = kchunk;
  p.grid_x = T;
  p.zero_row0 = -1;
  // tail split: linear epilogue, identity row map, plain store, C not overlapping resid
  const bool ident = d.c_rows == nullptr && d.c_group >= d.M && d.c_offset == 0;
  bool tail_ok = p.tile == 128 && !d.atomic && p.nsplit == 1 && !d.relu && d.beta == 0.f &&
                 ident && d.ldc >= d.N;
  if (tail_ok && d.resid) {
    const char* c0 = (const char*)d.C;
    const char* c1 = (const char*)(d.C + (d.M - 1) * d.ldc + d.N);
    const char* r0 = (const char*)d.resid;
    const char* r1 = (const char*)(d.resid + (d.M - 1) * d.ldr + d.N);
    if (r0 < c1 && c0 < r1) tail_ok = false;
  }
  // Underfilled single round (SAVQA_GEMM_CU_TAIL): T tiles over `cus` CUs put
  // ceil(T / cus) tiles on some CUs while the average is T / cus (the N = 512 step shapes:
  // 584 tiles = 2.28 per CU, so 3 tile-times per launch). Whole tiles for k = floor(T / cus)
  // per CU, the r left over split into f <= cus / r k-slices dispatched after them: at most
  // k tiles + one slice per CU. With T <= cus (k = 0: the relation workload's 5256-row
  // stack, 168 tiles) every tile is split, for K >= 64 k-tiles only: 5256x512x2048 175 ->
  // 130 us, x1536 129 -> 101 us, but x512 53 -> 56 us (the zero fill and atomics dominate).
  const int cus = slots / occ;
  const bool cu_tail = SAVQA_GEMM_CU_TAIL && tail_ok && T <= slots &&
                       (T > cus || (d.K + BK - 1) / BK >= 64);
  if (tail_ok && (T > slots || cu_tail)) {
    const int64_t nch = (d.K + BK - 1) / BK;
    const int cap = cu_tail ? cus : slots;
    int r = cu_tail ? T - (T / cus) * cus : T % slots;
    r = (r + tn - 1) / tn * tn;  // whole rows of tiles: one contiguous zero-fill
    if (r > 0 && (r < T || cu_tail)) {
      int f = cap / r;
      if (cu_tail) {
        // slices per left-over tile minimising the per-CU time k + ceil(r f / cus) / f
        // (in whole-tile times) within one round of slots, e.g. 400 tiles = 256 + 144 x 3
        // slices: 1.67 instead of 2 tile-times
        const int k = T / cus;
        double best = k + 1.0;
        f = 1;
        for (int g = 2; g <= 8 && g <= nch / 4; ++g) {
          if ((int64_t)k * cus + (int64_t)r * g > slots) break;
          const double t = k + (double)((r * g + cus - 1) / cus) / g;
          if (t < best - 1e-9) { best = t; f = g; }
        }
      }
      if (f > nch / 4) f = (int)(nch / 4);
      if (f >= 2) {
        p.gg.full = T - r;
        p.gg.tail_t0 = T - r;
        p.gg.tail_f = f;
        const int64_t tk = (d.K + f - 1) / f;
        p.gg.tail_kchunk = (tk + BK - 1) / BK * BK;
        p.grid_x = p.gg.full + r * f;
        p.zero_row0 = (int64_t)(p.gg.tail_t0 / tn) * p.tile;
      }
    }
  }
  // slab mode: the partials of a K split go to the caller's workspace and are summed in a
  // fixed order (fp32 / x6 kernels; identity row map and an epilogue linear in the
  // accumulator -- row scale and ReLU-backward mask included, no ReLU / beta)
  const bool slab_ok = (d.prec == 0 || d.prec == 6) && ident && !d.relu && d.beta == 0.f;
  p.ws_need = 0;
  if (slab_ok && p.nsplit > 1 && d.atomic)
    p.ws_need = (int64_t)p.nsplit * d.M * d.N + (d.colsum_a ? (int64_t)p.nsplit * d.M : 0);
  else if (slab_ok && p.gg.tail_f > 1)
    p.ws_need = (int64_t)p.gg.tail_f * (d.M - p.zero_row0) * d.N;
  if (p.ws_need > 0 && d.ws && d.ws_elems >= p.ws_need) {
    p.gg.slab = d.ws;
    if (p.nsplit > 1) {
      p.gg.slab_stride = d.M * d.N;
      p.gg.slab_r0 = 0;
      p.gg.slab_cs = d.colsum_a ? d.ws + (int64_t)p.nsplit * d.M * d.N : nullptr;
    } else {
      p.gg.slab_r0 = p.zero_row0;
      p.gg.slab_stride = (d.M - p.zero_row0) * d.N;
      p.zero_row0 = -1;  // the reduce pass assigns the tail rows: no zero fill
    }
  }
  return 0;
}

template <int BM, int BN, int BK, bool AT, bool BT>
static void launch_gemm(const savqa_gemm_desc& d, const GemmPlan& p, hipStream_t s, int avec,
                        int bvec) {
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, BK, AT, BT>), dim3(p.grid_x, p.nsplit), dim3(GEMM_NT),
                     0, s, d, p.gg, avec, bvec);
}

template <int BM, int BN, int BK>
static void dispatch_layout(const savqa_gemm_desc& d, const GemmPlan& p, hipStream_t s, int avec,
                            int bvec) {
  constexpr int BKW = GEMM_BK_DW;
  if (!d.a_trans && d.b_trans) launch_gemm<BM, BN, BK, false, true>(d, p, s, avec, bvec);
  else if (!d.a_trans && !d.b_trans) launch_gemm<BM, BN, BK, false, false>(d, p, s, avec, bvec);
  else if (d.a_trans && !d.b_trans) launch_gemm<BM, BN, BKW, true, false>(d, p, s, avec, bvec);
  else launch_gemm<BM, BN, BKW, true, true>(d, p, s, avec, bvec);
}

extern "C" int savqa_gemm_plan(const savqa_gemm_desc* dp, int32_t* out) {
  if (!dp || !out) return fail(SAVQA_EINVAL, "savqa_gemm_plan: null argument");
  savqa_gemm_desc d = *dp;
  GemmPlan p{};
  if (int rc = plan_gemm(d, p)) return rc;
  out[0] = p.tile;
  out[1] = p.split;
  out[2] = p.gg.tail_f > 1 ? p.gg.tail_f : 0;
  out[3] = p.grid_x * p.nsplit;
  return 0;
}

extern "C" int64_t savqa_gemm_ws_elems(const savqa_gemm_desc* dp) {
  if (!dp) return fail(SAVQA_EINVAL, "savqa_gemm_ws_elems: null descriptor");
  savqa_gemm_desc d = *dp;
  GemmPlan p{};
  if (int rc = plan_gemm(d, p)) return rc;
  const bool vecs = (d.lda % 4 == 0) && aligned16(d.A) && (d.ldb % 4 == 0) && aligned16(d.B);
  if (p.tile == 128 && d.prec == 6 && !vecs) {  // savqa_gemm's fallback to the fp32 kernel
    d.prec = 0;
    if (int rc = plan_gemm(d, p)) return rc;
  }
  return p.ws_need;
}

extern "C" int savqa_gemm(void* stream, const savqa_gemm_desc* dp) {
  if (!dp) return fail(SAVQA_EINVAL, "savqa_gemm: null descriptor");
  savqa_gemm_desc d = *dp;
  if (d.M == 0 || d.N == 0) return 0;
  if (!d.A || !d.B || !d.C) return fail(SAVQA_EINVAL, "savqa_gemm: null operand");
  const bool bf_skinny = d.prec == 1;  // (plan_gemm maps it to 6 for the 128 x 128 tiles)
  const bool x6_two_level = d.prec == 5;
  if (bf_skinny || x6_two_level) d.prec = 6;
  GemmPlan p{};
  if (int rc = plan_gemm(d, p)) return rc;
  const int avec = (d.lda % 4 == 0) && aligned16(d.A);
  const int bvec = (d.ldb % 4 == 0) && aligned16(d.B);
  hipStream_t s = as_stream(stream);
  if (p.tile == 128 && d.prec == 6 && (!avec || !bvec)) {
    // operands that are not 16-B vectors (guarded loads only in the x6 kernel) take the fp32
    // kernel
    d.prec = 0;
    if (int rc = plan_gemm(d, p)) return rc;
  }
  if (p.zero_row0 >= 0 &&
      hipMemset2DAsync(d.C + p.zero_row0 * d.ldc, d.ldc * sizeof(float), 0, d.N * sizeof(float),
                       d.M - p.zero_row0, s) != hipSuccess)
    return fail(SAVQA_EUNSUP, "savqa_gemm: tail zero-fill failed");
  // pre-split B planes (savqa_gemm_desc.b_planes): x6 128x128 launches with a k-contiguous,
  // 16-B-vector A and no B row gather; anything else ignores them
  if (d.b_planes && !(p.tile == 128 && d.prec == 6 && !d.a_trans && !d.b_rows && avec &&
                      aligned16(d.b_planes)))
    d.b_planes = nullptr;
  if (p.tile == 128 && d.prec == 6) {
    savqa_launch_gemm_x6(d, p.gg, p.grid_x, p.nsplit, s, x6_two_level);
  } else if (p.tile == 128 && d.prec != 0) {
    savqa_launch_gemm_bf16(d, p.gg, p.grid_x, p.nsplit, s, avec, bvec);
  } else if (p.tile == 128) {
    dispatch_layout<128, 128, GEMM_BK>(d, p, s, avec, bvec);
  }
  if (p.tile == 128 && p.gg.slab) {  // slab mode: add the slices in order
    const bool split = p.nsplit > 1;
    const int64_t r0 = p.gg.slab_r0;
    const int ns = split ? p.nsplit : p.gg.tail_f;
    const int vec = (d.N % 4 == 0) && (d.ldc % 4 == 0) && aligned16(d.C);
    const int64_t work = (d.M - r0) * (vec ? d.N / 4 : d.N) + (split && d.colsum_a ? d.M : 0);
    const int blocks = (int)std::min<int64_t>(std::max<int64_t>((work + 255) / 256, 1),
                                              (int64_t)cu_count() * 8);
    hipLaunchKernelGGL(gemm_slab_reduce_kernel, dim3(blocks), dim3(256), 0, s, d.C, d.ldc,
                       p.gg.slab, ns, p.gg.slab_stride, r0, d.M, d.N, split ? 1 : 0, vec,
                       split ? d.colsum_a : nullptr, p.gg.slab_cs, d.M);
  }
  if (p.tile == 128) {
  } else if (p.tile == 16) {
    const int tn = p.gg.tiles_n;
    const dim3 g(p.grid_x), b(64 * SK_WAVES);
    if (!d.a_trans && d.b_trans) SAVQA_SK_LAUNCH(gemm_skinny16_kernel, false, true);
    else if (!d.a_trans) SAVQA_SK_LAUNCH(gemm_skinny16_kernel, false, false);
    else if (!d.b_trans) SAVQA_SK_LAUNCH(gemm_skinny16_kernel, true, false);
    else SAVQA_SK_LAUNCH(gemm_skinny16_kernel, true, true);
  } else if (bf_skinny && !((d.a_trans && d.a_rows) || (!d.b_trans && d.b_rows))) {
    const dim3 g(p.grid_x), b(64 * SK_WAVES);
    const int tn = p.gg.tiles_n;
    if (!d.a_trans && d.b_trans) SAVQA_SK_LAUNCH(gemm_skinny_bf_kernel, false, true);
    else if (!d.a_trans) SAVQA_SK_LAUNCH(gemm_skinny_bf_kernel, false, false);
    else if (!d.b_trans) SAVQA_SK_LAUNCH(gemm_skinny_bf_kernel, true, false);
    else SAVQA_SK_LAUNCH(gemm_skinny_bf_kernel, true, true);
  } else {
    const dim3 g(p.grid_x), b(64 * SK_WAVES);
    const int tn = p.gg.tiles_n;
    if (!d.a_trans && d.b_trans) SAVQA_SK_LAUNCH(gemm_skinny_kernel, false, true);
    else if (!d.a_trans) SAVQA_SK_LAUNCH(gemm_skinny_kernel, false, false);
    else if (!d.b_trans) SAVQA_SK_LAUNCH(gemm_skinny_kernel, true, false);
    else SAVQA_SK_LAUNCH(gemm_skinny_kernel, true, true);
  }
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

// Wide form (cols % 4 == 0, 16-B aligned rows): each lane sums 4 consecutive columns with
// 16-B loads (a wave covers 256 columns of a row, four rows in flight per lane), the 4 waves
// of a block take interleaved rows of its row chunk and fold through LDS before one atomicAdd
// per column and block (the 4-B-per-lane form above: 25.7 us for the 37376 x 512 bias
// gradients of cfg 3, ~3 TB/s).
namespace savqa {
__global__ __launch_bounds__(256) void colsum_wide_kernel(const float* __restrict__ X, int64_t rows,
                                                          int64_t cols, int64_t ldx, int64_t rchunk,
                                                          float* __restrict__ out) {
  __shared__ f4 part[4][64];
  const int lane = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 256 + 4 * lane;
  const int64_t r0 = (int64_t)blockIdx.y * rchunk;
  const int64_t r1 = min(rows, r0 + rchunk);
  f4 s = {0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int64_t r = r0 + sl;
    for (; r + 12 < r1; r += 16) {
      f4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f4*>(X + (r + 4 * u) * ldx + c);
#pragma unroll
      for (int u = 0; u < 4; ++u) s += v[u];
    }
    for (; r < r1; r += 4) s += *reinterpret_cast<const f4*>(X + r * ldx + c);
  }
  part[sl][lane] = s;
  __syncthreads();
  if (sl == 0 && c < cols) {
    const f4 t = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
#pragma unroll
    for (int q = 0; q < 4; ++q) atomicAdd(&out[c + q], t[q]);
  }
}
}  // namespace savqa

extern "C" int savqa_colsum_acc(void* stream, const float* X, int64_t rows, int64_t cols,
                                int64_t ldx, float* out) {
  if (rows <= 0 || cols <= 0) return 0;
  if (cols % 4 == 0 && ldx % 4 == 0 && aligned16(X)) {
    const int64_t cb = (cols + 255) / 256;
    int64_t chunks = (2048 + cb - 1) / cb;
    int64_t rchunk = (rows + chunks - 1) / chunks;
    if (rchunk < 64) rchunk = 64;
    chunks = (rows + rchunk - 1) / rchunk;
    hipLaunchKernelGGL(colsum_wide_kernel, dim3((unsigned)cb, (unsigned)chunks), dim3(256), 0,
                       as_stream(stream), X, rows, cols, ldx, rchunk, out);
    return check_launch("savqa_colsum_acc");
  }
  const int64_t cb = (cols + 63) / 64;
  int64_t chunks = (2048 + cb - 1) / cb;
  int64_t rchunk = (rows + chunks - 1) / chunks;
  if (rchunk < 64) rchunk = 64;
  chunks = (rows + rchunk - 1) / rchunk;
  hipLaunchKernelGGL(colsum_kernel, dim3(cb, chunks), dim3(256), 0, as_stream(stream), X, rows,
                     cols, ldx, rchunk, out);
  return check_launch("savqa_colsum_acc");
}
