// Shared pieces of the graph-attention kernels (attn.hip: T <= 128 MFMA strip / single-query kernels,
// attn_flash.hip: key-tiled kernels for long sequences). gfx950 only.
#pragma once
#include "common.h"

namespace savqa {

constexpr int ATT_DK = 64;
constexpr int ATT_KLD = 68;  // padded K/V row (floats), 16-B aligned
constexpr float ATT_MASKED = -4294967296.0f;  // fp32(-2**32 + 1)

// TQ / TKV: storage types of Q, dQ and of K, V, dK, dV (float, or __bf16 in the bf16
// training mode); O, dO, the graph and the flags stay fp32, and every kernel computes in fp32.
template <typename TQ, typename TKV = TQ>
struct AttnArgsT {
  const TQ* q; int64_t ldq;
  const TKV* k; int64_t ldk;
  const TKV* v; int64_t ldv;
  const float* G;
  const float* kflag;
  const float* qflag;
  int B, Tq, Tk, H;
  float* o; int64_t ldo;
  float* att;
  // backward
  const float* dout; int64_t lddo;
  TQ* dq; int64_t lddq;
  TKV* dk; int64_t lddk;
  TKV* dv; int64_t lddv;
};
using AttnArgs = AttnArgsT<float>;

using f4v = float __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v mfma16(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// sum / max over the 16 lanes of a DPP row. Butterfly partners (quad_perm [1,0,3,2],
// [2,3,0,1], row_half_mirror, row_mirror) pair every lane with a lane holding the same
// operand set, so all 16 lanes end with bitwise-identical totals (a row_ror ladder
// leaves quads with different association orders: T=1 softmax would then give a != 1
// in some lanes and break the reference's exact-zero Q/K gradients).
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  return v;
}

__device__ __forceinline__ f4v ld4(const float* p) { return *reinterpret_cast<const f4v*>(p); }

// 4 consecutive values of a Q/K/V row (fp32 or bf16 storage) as fp32; one value; a store
typedef __bf16 att_bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4v ldx4(const float* p) { return ld4(p); }
__device__ __forceinline__ f4v ldx4(const __bf16* p) {
  return __builtin_convertvector(*reinterpret_cast<const att_bf16x4*>(p), f4v);
}
__device__ __forceinline__ float ldx1(const float* p) { return *p; }
__device__ __forceinline__ float ldx1(const __bf16* p) { return (float)*p; }
__device__ __forceinline__ void stx1(float* p, float v) { *p = v; }
__device__ __forceinline__ void stx1(__bf16* p, float v) { *p = (__bf16)v; }

// 4 consecutive outputs of one lane: one 16-B (fp32) / 8-B (bf16) store when the row is
// vector-aligned (vec: wave-uniform), else 4 element stores (4 / 8 x the store instructions)
__device__ __forceinline__ void stx4(float* p, f4v v, bool vec) {
  if (vec) {
    *reinterpret_cast<f4v*>(p) = v;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) p[e] = v[e];
  }
}
__device__ __forceinline__ void stx4(__bf16* p, f4v v, bool vec) {
  if (vec) {
    *reinterpret_cast<att_bf16x4*>(p) = __builtin_convertvector(v, att_bf16x4);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) p[e] = (__bf16)v[e];
  }
}
template <typename T>
__device__ __forceinline__ bool vec_rows(const T* p, int64_t ld) {
  return (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(p) & (4 * sizeof(T) - 1)) == 0;
}

// (sample b, head h) views (common.h BView) of the attention operands: a row-major [rows][ld]
// operand of `rows` rows seen from row r0, column c0; the range ends at the tensor's last
// (row, 64-column head) element, so reads past it return 0.
template <typename T>
__device__ __forceinline__ BView head_view(const T* p, int64_t ld, int64_t rows, int64_t r0,
                                           int64_t c0) {
  return bview(p + r0 * ld + c0, ld * (int64_t)sizeof(T),
               ((rows - 1 - r0) * ld + ATT_DK) * (int64_t)sizeof(T));
}
// graph G[b] ([Tq][Tk] fp32) and the key / query flags of sample b
template <class A>
__device__ __forceinline__ BView graph_view(const A& a, int b) {
  const int64_t tt = (int64_t)a.Tq * a.Tk;
  return bview(a.G + b * tt, (int64_t)a.Tk * 4, (int64_t)(a.B - b) * tt * 4);
}
__device__ __forceinline__ BView flag_view(const float* f, int64_t T, int64_t B, int b) {
  return bview(f + b * T, 4, (B - b) * T * 4);
}

// the views every attention kernel of (sample b, head h) reads
template <class A>
struct StripViews {
  BView q, k, v, g, kf, qf;
  __device__ __forceinline__ StripViews(const A& a, int b, int h) {
    const int64_t nq = (int64_t)a.B * a.Tq, nk = (int64_t)a.B * a.Tk;
    q = head_view(a.q, a.ldq, nq, (int64_t)b * a.Tq, h * ATT_DK);
    k = head_view(a.k, a.ldk, nk, (int64_t)b * a.Tk, h * ATT_DK);
    v = head_view(a.v, a.ldv, nk, (int64_t)b * a.Tk, h * ATT_DK);
    g = graph_view(a, b);
    kf = flag_view(a.kflag, a.Tk, a.B, b);
    qf = flag_view(a.qflag, a.Tq, a.B, b);
  }
};

// 4 consecutive Q/K/V values (fp32 or bf16 storage) as fp32 through a view; one value
template <typename T>
__device__ __forceinline__ f4v bldx4(const BView& v, uint32_t vo, uint32_t so) {
  if constexpr (sizeof(T) == 4) {
    return bld16b<f4v>(v, vo, so);
  } else {
    return __builtin_convertvector(bld8b<att_bf16x4>(v, vo, so), f4v);
  }
}
template <typename T>
__device__ __forceinline__ float bldx1(const BView& v, uint32_t vo, uint32_t so) {
  if constexpr (sizeof(T) == 4) {
    return bld1(v, vo, so);
  } else {
    return (float)__builtin_bit_cast(__bf16, bld16(v, vo, so));
  }
}
template <typename T>
__device__ __forceinline__ void bstx1(const BView& v, float x, uint32_t vo, uint32_t so) {
  if constexpr (sizeof(T) == 4) {
    bst32(v, x, vo, so);
  } else {
    bst16(v, __builtin_bit_cast(unsigned short, (__bf16)x), vo, so);
  }
}
// 4 consecutive outputs of one lane through a view: one 16-B (fp32) / 8-B (bf16) store when
// the rows are vector-aligned (vec: wave-uniform), else 4 element stores
template <typename T>
__device__ __forceinline__ void bstx4(const BView& v, f4v x, uint32_t vo, uint32_t so, bool vec) {
  if (vec) {
    if constexpr (sizeof(T) == 4) bst16b(v, x, vo, so);
    else bst8b(v, __builtin_convertvector(x, att_bf16x4), vo, so);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) bstx1<T>(v, x[e], vo + e * (uint32_t)sizeof(T), so);
  }
}

// softmax exponent in base 2: x2 = s * (log2(e) / 8), e = 2^(x2 - max x2) on v_exp_f32 (the
// masked score keeps the reference's "all keys masked -> uniform" behaviour: every masked key
// gets the same value, and any unmasked key's 2^(x2 - max) underflows it to 0)
constexpr float ATT_SCALE2 = 0.18033688011112042f;  // log2(e) / sqrt(64)
__device__ __forceinline__ float att_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Same with Y staged in LDS ([TK][ATT_KLD], rows >= Tk zero): b128 reads, lanes 0-15 of a
// read phase hit 16 disjoint bank quads (row stride 68 floats).
template <int NJT>
__device__ __forceinline__ void strip_dots_lds(const f4v (&x)[4], const float* Ys, int col, int g,
                                               f4v (&acc)[NJT]) {
#pragma unroll
  for (int jt = 0; jt < NJT; ++jt) {
    const float* yr = Ys + (jt * 16 + col) * ATT_KLD + 4 * g;
    f4v s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f4v yv = ld4(yr + 16 * c);
      s = mfma16(x[c].x, yv.x, s);
      s = mfma16(x[c].y, yv.y, s);
      s = mfma16(x[c].z, yv.z, s);
      s = mfma16(x[c].w, yv.w, s);
    }
    acc[jt] = s;
  }
}

}  // namespace savqa
