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

// (tile, k-slice) of a split-K launch (grid = tiles x slices), XCD-aware over the WHOLE grid
// in slice-major order: each XCD runs a contiguous run of (slice, tile) items, i.e. whole
// k-slices, so a slice's operand rows are fetched into one XCD's L2 and shared by every tile
// of that slice there. (Remapping only the tile index gave every XCD the same tiles of
// every slice: each XCD then streamed all k-slices of its tiles' operand columns, and the
// N-side operand was fetched by all eight L2s.) Unsplit launches: xcd_remap of the tile.
__device__ __forceinline__ void split_remap(int nblk, int& tile, int& slice) {
  if (gridDim.y == 1) {
    tile = xcd_remap(blockIdx.x, nblk);
    slice = 0;
    return;
  }
  const int item = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  slice = item / gridDim.x;
  tile = item - slice * gridDim.x;
}

// Dropout keep bits (nn.Dropout sites of the path, AttModel_x3.py:71-72, 102, 147, 227, 274,
// 482-500). torch's Philox stream cannot be reproduced bit-for-bit, so the library defines
// its own counter-based stream: element idx of dropout site `site` under step seed `seed`
// is the SplitMix64 output for counter (seed + site*K1 + (idx+1)*K2). Stateless, so the
// backward regenerates the forward's masks instead of storing them. Restated in
// oracle/savqa_oracle.py:dropout_keep for the parity tests.
__device__ __forceinline__ uint32_t drop_bits(uint64_t seed, uint32_t site, uint64_t idx) {
  uint64_t z = seed + (uint64_t)site * 0xD1B54A32D192ED03ull + (idx + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

// keep iff bits >= thr, thr = floor(p * 2^32); kept values are scaled by 1/(1-p).
struct DropParam {
  uint64_t seed;
  uint32_t thr;
  float scale;
  int drop_all;
};

inline DropParam make_drop(uint64_t seed, float p) {
  DropParam d;
  d.seed = seed;
  d.drop_all = p >= 1.f;
  const double t = (double)p * 4294967296.0;
  d.thr = p <= 0.f ? 0u : (t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t);
  d.scale = d.drop_all ? 0.f : 1.f / (1.f - p);
  return d;
}

__device__ __forceinline__ float drop_mul(const DropParam& d, uint32_t site, uint64_t idx) {
  return (!d.drop_all && drop_bits(d.seed, site, idx) >= d.thr) ? d.scale : 0.f;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Buffer-resource view of one operand from a wave-uniform origin (cdna_hip_programming.md T8 /
// T20): every lane address is a 32-bit byte offset from the origin, wave-uniform parts go to
// the instruction's SGPR soffset, and the hardware range check returns 0 for reads at or past
// `n_bytes` (writes there are dropped) -- so a (sample, head) origin turns the 64-bit
// row * ld address arithmetic of each load into one 32-bit lane offset per access pattern,
// and rows past the end of the tensor need no clamped addresses.
struct BView {
  __amdgpu_buffer_rsrc_t r;
  uint32_t ld;  // bytes per row
};

__device__ __forceinline__ BView bview(const void* origin, int64_t ld_bytes, int64_t n_bytes) {
  BView v;
  const int64_t nb = n_bytes < 0 ? 0 : (n_bytes > 0xFFFFFFFFll ? 0xFFFFFFFFll : n_bytes);
  v.r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(origin), (short)0, (int)(uint32_t)nb,
                                          0x00020000);
  v.ld = (uint32_t)ld_bytes;
  return v;
}

__device__ __forceinline__ float bld1(const BView& v, uint32_t vo, uint32_t so) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(v.r, vo, so, 0));
}
__device__ __forceinline__ unsigned short bld16(const BView& v, uint32_t vo, uint32_t so) {
  return __builtin_amdgcn_raw_buffer_load_b16(v.r, vo, so, 0);
}
template <class V>  // 8 bytes
__device__ __forceinline__ V bld8b(const BView& v, uint32_t vo, uint32_t so) {
  return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(v.r, vo, so, 0));
}
template <class V>  // 16 bytes
__device__ __forceinline__ V bld16b(const BView& v, uint32_t vo, uint32_t so) {
  return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(v.r, vo, so, 0));
}
__device__ __forceinline__ void bst16(const BView& v, unsigned short x, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_buffer_store_b16(x, v.r, vo, so, 0);
}
__device__ __forceinline__ void bst32(const BView& v, float x, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, x), v.r, vo, so, 0);
}
template <class V>
__device__ __forceinline__ void bst8b(const BView& v, V x, uint32_t vo, uint32_t so) {
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, x), v.r, vo, so, 0);
}
template <class V>
__device__ __forceinline__ void bst16b(const BView& v, V x, uint32_t vo, uint32_t so) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, x), v.r, vo, so, 0);
}

}  // namespace savqa
