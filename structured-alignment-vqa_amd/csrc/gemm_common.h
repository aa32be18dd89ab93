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
struct GemmGrid {
  int tiles_n, full, tail_t0, tail_f;
  int64_t kchunk, tail_kchunk;
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

}  // namespace savqa

// gemm_bf16.hip: bf16 / 3xbf16 MFMA kernels on a plan made by savqa_gemm (desc.prec != 0)
int savqa_launch_gemm_bf16(const savqa_gemm_desc& d, const savqa::GemmGrid& gg, int grid_x,
                           int nsplit, hipStream_t s, int avec, int bvec);
