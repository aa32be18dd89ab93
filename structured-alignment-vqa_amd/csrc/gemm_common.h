// Shared pieces of the GEMM kernels (gemm.hip: fp32 MFMA; gemm_bf16.hip: bf16 / 3xbf16
// MFMA): vector types, the launch-grid descriptor and the fused epilogue. gfx950 only.
#pragma once
#include "common.h"

namespace savqa {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));  // native vector (HIP float4 copies
                                                          // lower to memcpy and block SROA)

constexpr int GEMM_NT = 256;

// Block -> (tile, k range). Blocks [0, full) own whole tiles (or split-K slices along
// blockIdx.y); blocks [full, gridDim.x) are the "tail": tiles [tail_t0, T) each cut into
// tail_f k-slices so the last partial wave of tiles spreads over every CU.
// Slab mode (savqa_gemm_desc.ws; gemm_f32_kernel / gemm_x6_kernel): split-K slice s stores its
// partial tile to slab + s * slab_stride, a tail block of part p to slab + p * slab_stride,
// as rows m - slab_r0 of N floats (plain stores), and slice s's column sums (colsum_a) to
// slab_cs + s * M; gemm_slab_reduce_kernel then adds them in slice order.
struct GemmGrid {
  int tiles_n, full, tail_t0, tail_f;
  int64_t kchunk, tail_kchunk;
  float* slab;
  float* slab_cs;
  int64_t slab_stride, slab_r0;
};

// Epilogue of one output element (include/savqa.h formula), split per row / element.
struct EpiRow {
  float* crow;
  float rs;
  int64_t mr, pr;
};

__device__ __forceinline__ EpiRow epi_row(const savqa_gemm_desc& d, int64_t m, bool ident) {
  EpiRow e;
  int64_t cr;
  if (ident) {
    cr = m;
  } else if (d.c_rows) {
    cr = d.c_rows[m];
  } else {
    const uint32_t mu = (uint32_t)m, cg = (uint32_t)d.c_group;
    cr = (int64_t)(mu / cg) * d.c_stride + (int64_t)(mu % cg) + d.c_offset;
  }
  e.crow = d.C + cr * d.ldc;
  e.rs = d.rowscale ? d.rowscale[m] : 1.f;
  e.mr = d.mask_arows ? d.a_rows[m] : m;
  e.pr = d.rowvec ? (int64_t)((uint32_t)m % (uint32_t)d.rowvec_period) : 0;
  return e;
}

// keep: < 0 = read the mask from memory, 0 / 1 = the caller's prefetched mask bit
__device__ __forceinline__ void epi_store_t(const savqa_gemm_desc& d, const EpiRow& e, int64_t m,
                                            int64_t n, float acc, bool first_split, bool atomic,
                                            int keep) {
  float v = acc * d.alpha;
  if (first_split) {
    if (d.bias) v += d.bias[n];
    if (d.rowvec) v += d.rowvec[e.pr * d.ldrv + n];
  }
  if (d.relu) v = fmaxf(v, 0.f);
  v *= e.rs;
  if (keep == 0 || (keep < 0 && d.mask && !(d.mask[e.mr * d.ldmask + n] > 0.f))) v = 0.f;
  if (first_split && d.resid) v += d.resid[m * d.ldr + n];
  float* cp = e.crow + n;
  if (atomic) {
    atomicAdd(cp, v);
  } else if (d.beta != 0.f) {
    *cp = v + d.beta * *cp;
  } else {
    *cp = v;
  }
}

__device__ __forceinline__ void epi_store(const savqa_gemm_desc& d, const EpiRow& e, int64_t m,
                                          int64_t n, float acc, bool first_split, bool atomic) {
  epi_store_t(d, e, m, n, acc, first_split, atomic, -1);
}

// Epilogue of a 128x128 tile held as 16x16 MFMA accumulators (every v_mfma_f32_16x16x*
// form: lane l holds rows 4(l/16) + r, r < 4, of column l % 16), FM x FN fragments per wave,
// the wave's sub-tile at (m0 + wm*WM, n0 + wn*WN). Used by gemm_f32_kernel (gemm.hip) and
// gemm_x6_kernel (gemm_x6.hip).
// Operands of the epilogue are fetched before a fragment's first store: vmcnt also counts
// stores, so a load issued after a store waits for it, and one load per element (bias,
// ReLU-backward mask, residual) serialised a memory round trip per element.
//   bias: FN values per lane and the mask bits (rows indexed by m) per fragment row, the
//   residual per 16-row fragment (a whole tile's would spill).
// slab != nullptr: the partial of this K slice goes to slab[(m - slab_r0) * N + n] with a
// plain store (identity row map, linear epilogue: host-checked).
template <int FM, int FN, int WM, int WN>
__device__ __forceinline__ void gemm_epilogue16(const savqa_gemm_desc& d, const f4 (&acc)[FM][FN],
                                                int64_t m0, int64_t n0, int wm, int wn, int lane,
                                                bool first_split, bool atomic,
                                                float* slab = nullptr, int64_t slab_r0 = 0) {
  constexpr int FR = 16, NACC = 4;
  auto row = [&](int r) { return 4 * (lane >> 4) + r; };
  const int col = lane & 15;
  const bool ident = d.c_rows == nullptr && d.c_group >= d.M && d.c_offset == 0;
  const bool mask_pre = d.mask && !d.mask_arows;
  const bool res_pre = first_split && d.resid != nullptr;
  float bv[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int64_t n = min(n0 + wn * WN + j * FR + col, (int64_t)d.N - 1);
    bv[j] = (first_split && d.bias) ? d.bias[n] : 0.f;
  }
  uint32_t keep[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    keep[i] = 0xffffffffu;
    if (mask_pre) {  // this fragment's mask bits (a whole tile's up front spilled)
      float mv[NACC][FN];
#pragma unroll
      for (int r = 0; r < NACC; ++r) {
        const int64_t m = min(m0 + wm * WM + i * FR + row(r), (int64_t)d.M - 1);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int64_t n = min(n0 + wn * WN + j * FR + col, (int64_t)d.N - 1);
          mv[r][j] = d.mask[m * d.ldmask + n];
        }
      }
      keep[i] = 0;
#pragma unroll
      for (int r = 0; r < NACC; ++r)
#pragma unroll
        for (int j = 0; j < FN; ++j) keep[i] |= (mv[r][j] > 0.f ? 1u : 0u) << (r * FN + j);
    }
    float rv[NACC][FN];  // this fragment's residual values
#pragma unroll
    for (int r = 0; r < NACC; ++r) {
      const int64_t m = min(m0 + wm * WM + i * FR + row(r), (int64_t)d.M - 1);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int64_t n = min(n0 + wn * WN + j * FR + col, (int64_t)d.N - 1);
        rv[r][j] = res_pre ? d.resid[m * d.ldr + n] : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < NACC; ++r) {
      const int64_t m = m0 + wm * WM + i * FR + row(r);
      if (m >= d.M) continue;
      const EpiRow er = epi_row(d, m, ident);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int64_t n = n0 + wn * WN + j * FR + col;
        if (n >= d.N) continue;
        // savqa_gemm epilogue (include/savqa.h), operands prefetched above
        float v = acc[i][j][r] * d.alpha + bv[j];
        if (first_split && d.rowvec) v += d.rowvec[er.pr * d.ldrv + n];
        if (d.relu) v = fmaxf(v, 0.f);
        v *= er.rs;
        if (d.mask && (mask_pre ? !((keep[i] >> (r * FN + j)) & 1u)
                                : !(d.mask[er.mr * d.ldmask + n] > 0.f)))
          v = 0.f;
        v += rv[r][j];
        if (slab) {
          slab[(m - slab_r0) * d.N + n] = v;
          continue;
        }
        float* cp = er.crow + n;
        if (atomic) atomicAdd(cp, v);
        else if (d.beta != 0.f) *cp = v + d.beta * *cp;
        else *cp = v;
      }
    }
  }
}

}  // namespace savqa

// gemm_bf16.hip: bf16 / 3xbf16 MFMA kernels on a plan made by savqa_gemm (desc.prec == 3)
int savqa_launch_gemm_bf16(const savqa_gemm_desc& d, const savqa::GemmGrid& gg, int grid_x,
                           int nsplit, hipStream_t s, int avec, int bvec);
// gemm_x6.hip: fp32 GEMM on bf16 matrix cores from exact three-term splits (desc.prec == 6)
int savqa_launch_gemm_x6(const savqa_gemm_desc& d, const savqa::GemmGrid& gg, int grid_x,
                         int nsplit, hipStream_t s, bool two_level);
