// Shared helpers for the libsavqa HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/savqa.h"

namespace savqa {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);

constexpr int kWave = 64;

// Wave-wide reductions with DPP row ops + 4 readlanes (all VALU/SALU, no LDS round
// trips): quad_perm [1,0,3,2], [2,3,0,1], row_ror:4, row_ror:8 leave every lane of a
// 16-lane row holding that row's total; the four row totals are then read as scalars.
// (__shfl_xor lowers to ds_bpermute: ~100 cycles of LDS latency per step, 6 steps.)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}

__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x128>(v);  // row_ror:8
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}

__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x124>(v));
  v = fmaxf(v, dpp_f<0x128>(v));
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

// bijective XCD-aware remap (cdna_hip_programming.md T1): blocks b and b+8 share an
// XCD under round-robin dispatch, so give each XCD a contiguous run of logical tiles.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int xcd = bid & 7;
  const int q = nblk >> 3, r = nblk & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace savqa
