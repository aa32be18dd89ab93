// MIL-NCE relation branch (only_obj = False), AttModel_x3.py:382-437, gfx950.
//
// Entries ("slots") come from the loader's loc tables (dataloader/
// data_loader_itp_bbox_super_node.py:208-246, collate :437-449):
//   positive [b][k] = [obj_i, obj_j, rel_category, macro_rel_loc, micro_rel_loc], negative
//   [b][k] = [obj_i, obj_j, rel_category, macro_rel_loc]; macro_rel_loc < 0 = padding.
// The reference evaluates x_i^T R_r x_j for ALL (b, r, i, j) (an N x #rel x H x H einsum,
// :393-401, materialising R repeated N times) and then gathers the listed entries. Here
// the caller runs ONE MFMA GEMM V = X_all Rmat^T (X_all = the batch's object rows,
// Rmat = R viewed as [nrel*H][H]: V[(b,j)][r*H+l] = (R_r x_j)_l), every listed entry is a
// contiguous 4*H-byte dot (rel_entries_*), and the backward is the entries' scatter into
// dV plus two more GEMMs (dR += dV^T X_all, dX_all += dV Rmat).
// The scalar chain (two logsumexps over the batch's positives / negatives, the softmax
// over the positives, :405-420) and the ordered macro-node update (:418-436: zero the
// relation nodes, then add softmax[micro_rel_loc] * rel_feature[micro_rel_loc] entry by
// entry, in the reference's loop order) run in single-workgroup kernels: their order
// is the reference's, so the result does not depend on scheduling.
#include <algorithm>

#include "common.h"

namespace savqa {

struct RelSlots {
  const int64_t* loc;  // [B][L][W]
  int W, B, L;
};

__device__ __forceinline__ bool slot_valid(const RelSlots& s, int slot) {
  return s.loc[(int64_t)slot * s.W + 3] >= 0;
}

// Bilinear entries through the dense product V = X R^T-stacked (csrc: a GEMM by the caller):
//   V[(b,j)][r*H + l] = sum_k obj[b,j][k] R[r][l][k] = (R_r x_j)_l,  ldv = nrel*H
// so an entry is one contiguous dot: val = sum_l x_i[l] V[(b,j)][r*H + l]. One wave per slot.
__global__ __launch_bounds__(256) void rel_entries_fwd_kernel(RelSlots s, const float* __restrict__ obj,
                                                             int Nv, int H,
                                                             const float* __restrict__ V,
                                                             int64_t ldv, float* __restrict__ val) {
  const int lane = threadIdx.x & 63;
  const int slot = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (slot >= s.B * s.L) return;
  const int64_t* lr = s.loc + (int64_t)slot * s.W;
  if (lr[3] < 0) {
    if (lane == 0) val[slot] = 0.f;
    return;
  }
  // bounds (the host checks them too): a bad row scores NaN instead of reading outside
  if (lr[0] < 0 || lr[0] >= Nv || lr[1] < 0 || lr[1] >= Nv || lr[2] < 0 || (lr[2] + 1) * H > ldv) {
    if (lane == 0) val[slot] = __builtin_nanf("");
    return;
  }
  const int b = slot / s.L;
  const float* xi = obj + ((int64_t)b * Nv + lr[0]) * H;
  const float* vr = V + ((int64_t)b * Nv + lr[1]) * ldv + lr[2] * (int64_t)H;
  float acc = 0.f;
  for (int l = lane; l < H; l += 64) acc += xi[l] * vr[l];
  acc = wave_sum(acc);
  if (lane == 0) val[slot] = acc;
}

// backward of one entry with g = dval[slot]: dobj[b,i] += g V[(b,j)][rH:], dV[(b,j)][rH:] += g x_i
__global__ __launch_bounds__(256) void rel_entries_bwd_kernel(RelSlots s, const float* __restrict__ obj,
                                                             int Nv, int H,
                                                             const float* __restrict__ V,
                                                             int64_t ldv,
                                                             const float* __restrict__ dval,
                                                             float* __restrict__ dobj,
                                                             float* __restrict__ dV) {
  const int lane = threadIdx.x & 63;
  const int slot = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (slot >= s.B * s.L) return;
  const int64_t* lr = s.loc + (int64_t)slot * s.W;
  if (lr[3] < 0 || lr[0] < 0 || lr[0] >= Nv || lr[1] < 0 || lr[1] >= Nv || lr[2] < 0 ||
      (lr[2] + 1) * H > ldv)
    return;
  const float g = dval[slot];
  if (g == 0.f) return;
  const int b = slot / s.L;
  const int64_t ri = (int64_t)b * Nv + lr[0];
  const float* xi = obj + ri * H;
  const int64_t vo = ((int64_t)b * Nv + lr[1]) * ldv + lr[2] * (int64_t)H;
  for (int l = lane; l < H; l += 64) {
    atomicAdd(&dobj[ri * H + l], g * V[vo + l]);
    atomicAdd(&dV[vo + l], g * xi[l]);
  }
}

// Scalar chain (:405-420). Valid entries of a sample must be a prefix of its slots (the
// collate fills rows from 0 and pads the tail, :445-449), so the reference's nonzero()
// order gives the c-th valid positive as slot (b, c - cum[b]): no compaction pass is
// needed. Outputs:
//   cum[b] = valid positives of samples < b; wsm[cum[b] + k] = softmax over all valid
//   positives (:420); st = (P, m1, Z1, m2, Z2, err, mr, Zr) with
//   mil_rel = (m1 + log Z1) - (m2 + log Z2)  the two clamped logsumexps (:405-406);
//   err = 1 (and mil_rel = NaN) if some sample's valid slots are not a prefix.
// Two launches over G workgroups, each owning a contiguous chunk of the index space
// [positives | negatives]:
//   rel_loss_part_kernel: per chunk, for each logsumexp its local max m_g and
//     z_g = sum exp(x - m_g), and per sample the valid count / last valid index + 1;
//   rel_loss_fold_kernel: every workgroup folds the G records (M = max m_g, then
//     Z = sum z_g exp(m_g - M) in a fixed tree), so all hold the same statistics bit for bit,
//     and writes the softmax of its own chunk's positives; workgroup 0 writes cum / st / mil_rel.
// The fold order depends on (B, Lp, Ln) only, never on scheduling. Workspace (caller's):
// G x 8 floats of records, then 2 x G x B ints of counts.
constexpr int REL_NT = 256;
constexpr int REL_CHUNK = 1024;  // slots per workgroup
constexpr int REL_MAXG = 1024;
constexpr int REL_MAXB = 64;

__device__ __forceinline__ float blk_max(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max(v);
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int k = 1; k < (int)(blockDim.x >> 6); ++k) r = fmaxf(r, red[k]);
  __syncthreads();
  return r;
}
__device__ __forceinline__ float blk_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) r += red[k];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(REL_NT) void rel_loss_part_kernel(
    RelSlots sp_s, const float* __restrict__ sp, RelSlots sn_s, const float* __restrict__ sn,
    float eps, int chunk, float* __restrict__ rec, int* __restrict__ cntp, int* __restrict__ kmxp) {
  __shared__ float red[REL_NT / 64];
  __shared__ int cnt[REL_MAXB], kmax[REL_MAXB];
  const int tid = threadIdx.x, g = blockIdx.x;
  const int B = sp_s.B, L = sp_s.L, S = B * L, Sn = sn_s.B * sn_s.L;
  const int lo = g * chunk, hi = min(lo + chunk, S + Sn);
  for (int b = tid; b < B; b += blockDim.x) cnt[b] = kmax[b] = 0;
  __syncthreads();
  float m1 = -INFINITY, mr = -INFINITY, m2 = -INFINITY;
  for (int t = lo + tid; t < hi; t += blockDim.x) {
    if (t < S) {
      if (slot_valid(sp_s, t)) {
        const int b = t / L;
        atomicAdd(&cnt[b], 1);
        atomicMax(&kmax[b], t - b * L + 1);
        const float v = sp[t];
        m1 = fmaxf(m1, fmaxf(v, eps));
        mr = fmaxf(mr, v);
      }
    } else if (slot_valid(sn_s, t - S)) {
      m2 = fmaxf(m2, fmaxf(sn[t - S], eps));
    }
  }
  m1 = blk_max(m1, red);  // (its barriers also publish cnt / kmax)
  mr = blk_max(mr, red);
  m2 = fmaxf(m1, blk_max(m2, red));
  float z1 = 0.f, z2 = 0.f, zr = 0.f;
  for (int t = lo + tid; t < hi; t += blockDim.x) {
    if (t < S) {
      if (slot_valid(sp_s, t)) {
        const float v = sp[t], vc = fmaxf(v, eps);
        z1 += expf(vc - m1);
        z2 += expf(vc - m2);
        zr += expf(v - mr);
      }
    } else if (slot_valid(sn_s, t - S)) {
      z2 += expf(fmaxf(sn[t - S], eps) - m2);
    }
  }
  z1 = blk_sum(z1, red);
  z2 = blk_sum(z2, red);
  zr = blk_sum(zr, red);
  if (tid == 0) {
    float* r = rec + (int64_t)g * 8;
    r[0] = m1, r[1] = z1, r[2] = mr, r[3] = zr, r[4] = m2, r[5] = z2;
  }
  for (int b = tid; b < B; b += blockDim.x) {
    cntp[(int64_t)g * B + b] = cnt[b];
    kmxp[(int64_t)g * B + b] = kmax[b];
  }
}

// (M, Z) of one logsumexp from the G records at offset k: chunks without entries (z_g = 0)
// are skipped, so an empty set folds to (-inf, 0)
__device__ __forceinline__ float2 fold_lse(const float* __restrict__ rec, int G, int k, float* red) {
  float m = -INFINITY;
  for (int g = threadIdx.x; g < G; g += blockDim.x) m = fmaxf(m, rec[(int64_t)g * 8 + k]);
  const float M = blk_max(m, red);
  float z = 0.f;
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    const float zg = rec[(int64_t)g * 8 + k + 1];
    if (zg > 0.f) z += zg * expf(rec[(int64_t)g * 8 + k] - M);
  }
  return make_float2(M, blk_sum(z, red));
}

__global__ __launch_bounds__(REL_NT) void rel_loss_fold_kernel(
    RelSlots sp_s, const float* __restrict__ sp, int chunk, int G, const float* __restrict__ rec,
    const int* __restrict__ cntp, const int* __restrict__ kmxp, int* __restrict__ cum,
    float* __restrict__ wsm, float* __restrict__ st, float* __restrict__ mil_rel) {
  __shared__ float red[REL_NT / 64];
  __shared__ int cn[REL_MAXB], bad[REL_MAXB], cs[REL_MAXB + 1], err;
  const int tid = threadIdx.x;
  const int B = sp_s.B, L = sp_s.L, S = B * L;
  const float2 f1 = fold_lse(rec, G, 0, red), fr = fold_lse(rec, G, 2, red),
               f2 = fold_lse(rec, G, 4, red);
  for (int b = tid; b < B; b += blockDim.x) {
    int c = 0, k = 0;
    for (int g = 0; g < G; ++g) {
      c += cntp[(int64_t)g * B + b];
      k = max(k, kmxp[(int64_t)g * B + b]);
    }
    cn[b] = c;
    bad[b] = k != c;
  }
  __syncthreads();
  if (tid == 0) {
    int c = 0, e = 0;
    for (int b = 0; b < B; ++b) {
      cs[b] = c;
      c += cn[b];
      e |= bad[b];
    }
    cs[B] = c;
    err = e;
  }
  __syncthreads();
  const int lo = blockIdx.x * chunk, hi = min(lo + chunk, S);
  for (int t = lo + tid; t < hi; t += blockDim.x) {
    if (slot_valid(sp_s, t)) {
      const int b = t / L;
      wsm[cs[b] + (t - b * L)] = expf(sp[t] - fr.x) / fr.y;
    }
  }
  if (blockIdx.x != 0) return;
  for (int b = tid; b <= B; b += blockDim.x) cum[b] = cs[b];
  if (tid == 0) {
    const int P = cs[B];
    st[0] = (float)P;
    st[1] = f1.x;
    st[2] = f1.y;
    st[3] = f2.x;
    st[4] = f2.y;
    st[5] = (float)err;
    st[6] = fr.x;
    st[7] = fr.y;
    *mil_rel = (P > 0 && err == 0) ? (f1.x + logf(f1.y)) - (f2.x + logf(f2.y)) : NAN;
  }
}

// Macro-node update (:418-436), one wave per run: the entries of one relation node
// (same sample, same macro_rel_loc) are consecutive slots (the loader appends a pair's
// entries together and each pair owns one relation node, :208-237), so the node's row
// is  0 + w[m4_1] f_1 + w[m4_2] f_2 + ...  accumulated in the reference's order in
// registers and written once (the zeroing of :418 is the accumulator's initial 0).
__global__ __launch_bounds__(256) void rel_macro_fwd_kernel(RelSlots s, const float* __restrict__ st,
                                                           const float* __restrict__ wsm,
                                                           const float* __restrict__ relf, int Ns,
                                                           int H, float* __restrict__ macro) {
  const int lane = threadIdx.x & 63;
  const int slot = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (slot >= s.B * s.L) return;
  const int b = slot / s.L, k0 = slot - b * s.L;
  const int64_t* lr = s.loc + (int64_t)slot * s.W;
  const int64_t r3 = lr[3];
  if (r3 < 0) return;
  if (k0 > 0 && s.loc[(int64_t)(slot - 1) * s.W + 3] == r3) return;  // not a run start
  const int P = (int)st[0];
  constexpr int HV = 16;  // columns per lane (H <= 1024)
  float acc[HV];
#pragma unroll
  for (int t = 0; t < HV; ++t) acc[t] = 0.f;
  for (int k = k0; k < s.L; ++k) {
    const int64_t* e = s.loc + ((int64_t)b * s.L + k) * s.W;
    if (e[3] != r3) break;
    const int64_t m4 = e[4];
    if (m4 >= P) continue;  // (the reference would index out of range)
    const float wv = wsm[m4];
    const float* src = relf + ((int64_t)b * s.L + m4) * H;
#pragma unroll
    for (int t = 0; t < HV; ++t) {
      const int h = lane + 64 * t;
      if (h < H) acc[t] += wv * src[h];
    }
  }
  float* row = macro + ((int64_t)b * Ns + r3) * H;
#pragma unroll
  for (int t = 0; t < HV; ++t) {
    const int h = lane + 64 * t;
    if (h < H) row[h] = acc[t];
  }
}

// Backward of the update, one wave per entry: dwsm[loc4] += dmacro[b,loc3] . relf[b,loc4],
// drelf[b,loc4] += wsm[loc4] * dmacro[b,loc3]. (The zeroing of the relation rows' previous
// contents is applied by rel_zero_rows_kernel after this kernel has read dmacro.)
__global__ __launch_bounds__(256) void rel_macro_bwd_kernel(RelSlots s, const float* __restrict__ st,
                                                           const float* __restrict__ wsm,
                                                           const float* __restrict__ relf, int Ns,
                                                           int H, const float* __restrict__ dmacro,
                                                           float* __restrict__ dwsm,
                                                           float* __restrict__ drelf) {
  const int lane = threadIdx.x & 63;
  const int slot = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (slot >= s.B * s.L) return;
  const int64_t* lr = s.loc + (int64_t)slot * s.W;
  if (lr[3] < 0 || lr[4] >= (int64_t)st[0]) return;
  const int b = slot / s.L;
  const float* drow = dmacro + ((int64_t)b * Ns + lr[3]) * H;
  const int64_t fr = ((int64_t)b * s.L + lr[4]) * H;
  const float wv = wsm[lr[4]];
  float dot = 0.f;
  for (int h = lane; h < H; h += 64) {
    dot += drow[h] * relf[fr + h];
    atomicAdd(&drelf[fr + h], wv * drow[h]);
  }
  dot = wave_sum(dot);
  if (lane == 0) atomicAdd(&dwsm[lr[4]], dot);
}

__global__ __launch_bounds__(256) void rel_zero_rows_kernel(RelSlots s, int Ns, int H,
                                                           float* __restrict__ dmacro) {
  const int lane = threadIdx.x & 63;
  const int slot = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (slot >= s.B * s.L) return;
  const int64_t* lr = s.loc + (int64_t)slot * s.W;
  if (lr[3] < 0) return;
  float* row = dmacro + ((int64_t)(slot / s.L) * Ns + lr[3]) * H;
  for (int h = lane; h < H; h += 64) row[h] = 0.f;
}

// per-chunk partials of sum_c wsm[c] dwsm[c] (the softmax-path adjoint), c < P = st[0]
__global__ __launch_bounds__(REL_NT) void rel_wdot_part_kernel(const float* __restrict__ wsm,
                                                              const float* __restrict__ dwsm,
                                                              const float* __restrict__ st,
                                                              int chunk, float* __restrict__ part) {
  __shared__ float red[REL_NT / 64];
  const int P = (int)st[0];
  const int lo = blockIdx.x * chunk, hi = min(lo + chunk, P);
  float t = 0.f;
  for (int c = lo + threadIdx.x; c < hi; c += blockDim.x) t += wsm[c] * dwsm[c];
  t = blk_sum(t, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// dsp / dsn per slot (parallel): d mil_rel through both clamped logsumexps (clamp passes
// gradient where x >= eps) + the softmax path wsm[c] (dwsm[c] - wd); every workgroup folds the
// Gw wdot partials in the same fixed order (wd, also left in st[8] by workgroup 0)
__global__ __launch_bounds__(256) void rel_loss_bwd_kernel(RelSlots sp_s, const float* __restrict__ sp,
                                                          RelSlots sn_s, const float* __restrict__ sn,
                                                          float eps, const int* __restrict__ cum,
                                                          const float* __restrict__ wsm,
                                                          const float* __restrict__ dwsm,
                                                          float* __restrict__ st,
                                                          const float* __restrict__ part, int Gw,
                                                          const float* __restrict__ dmil,
                                                          float* __restrict__ dsp,
                                                          float* __restrict__ dsn) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int S = sp_s.B * sp_s.L, Sn = sn_s.B * sn_s.L;
  __shared__ float red[256 / 64];
  float w = 0.f;
  for (int k = threadIdx.x; k < Gw; k += blockDim.x) w += part[k];
  const float wd = blk_sum(w, red);
  if (blockIdx.x == 0 && threadIdx.x == 0) st[8] = wd;
  const float m1 = st[1], z1 = st[2], m2 = st[3], z2 = st[4];
  const float g = dmil ? *dmil : 0.f;
  if (t < S) {
    const int slot = (int)t;
    float d = 0.f;
    if (slot_valid(sp_s, slot)) {
      const float v = sp[slot];
      if (v >= eps) d = g * (expf(v - m1) / z1 - expf(v - m2) / z2);
      const int b = slot / sp_s.L;
      const int c = cum[b] + (slot - b * sp_s.L);
      d += wsm[c] * (dwsm[c] - wd);
    }
    dsp[slot] = d;
  } else if (t < S + Sn) {
    const int slot = (int)(t - S);
    float d = 0.f;
    if (slot_valid(sn_s, slot) && sn[slot] >= eps) d = -g * expf(sn[slot] - m2) / z2;
    dsn[slot] = d;
  }
}

}  // namespace savqa

using namespace savqa;

static int rel_check(const RelSlots& s, const char* who) {
  if (!s.loc || s.B <= 0 || s.L < 0 || (s.W != 4 && s.W != 5))
    return fail(SAVQA_EINVAL, std::string(who) + ": bad loc table");
  return 0;
}

extern "C" int savqa_rel_entries_fwd(void* stream, const int64_t* loc, int32_t loc_w, int64_t B,
                                     int64_t L, const float* obj, int64_t Nv, int64_t H,
                                     const float* V, int64_t ldv, float* val) {
  RelSlots s{loc, loc_w, (int)B, (int)L};
  if (B * L == 0) return 0;
  if (int rc = rel_check(s, "savqa_rel_entries_fwd")) return rc;
  hipLaunchKernelGGL(rel_entries_fwd_kernel, dim3((unsigned)((B * L + 3) / 4)), dim3(256), 0,
                     as_stream(stream), s, obj, (int)Nv, (int)H, V, ldv, val);
  return check_launch("savqa_rel_entries_fwd");
}

extern "C" int savqa_rel_entries_bwd(void* stream, const int64_t* loc, int32_t loc_w, int64_t B,
                                     int64_t L, const float* obj, int64_t Nv, int64_t H,
                                     const float* V, int64_t ldv, const float* dval, float* dobj,
                                     float* dV) {
  RelSlots s{loc, loc_w, (int)B, (int)L};
  if (B * L == 0) return 0;
  if (int rc = rel_check(s, "savqa_rel_entries_bwd")) return rc;
  hipLaunchKernelGGL(rel_entries_bwd_kernel, dim3((unsigned)((B * L + 3) / 4)), dim3(256), 0,
                     as_stream(stream), s, obj, (int)Nv, (int)H, V, ldv, dval, dobj, dV);
  return check_launch("savqa_rel_entries_bwd");
}

// G workgroups of `chunk` slots over `total` slots (G <= REL_MAXG)
static void rel_fold_shape(int64_t total, int& G, int& chunk) {
  G = (int)std::min<int64_t>(REL_MAXG, std::max<int64_t>(1, (total + REL_CHUNK - 1) / REL_CHUNK));
  chunk = (int)std::max<int64_t>(1, (total + G - 1) / G);
}

extern "C" int64_t savqa_rel_loss_ws_bytes(int64_t B, int64_t Lp, int64_t Ln) {
  if (B <= 0 || Lp < 0 || Ln < 0) return 0;
  int G, chunk;
  rel_fold_shape(B * (Lp + Ln), G, chunk);
  return (int64_t)G * 8 * 4 + 2 * (int64_t)G * B * 4;
}

extern "C" int savqa_rel_loss_fwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp,
                                  const float* sp, const int64_t* neg_loc, int64_t Ln,
                                  const float* sn, float eps, int32_t* cum, float* wsm, float* st,
                                  float* mil_rel, void* ws, int64_t ws_bytes) {
  RelSlots a{pos_loc, 5, (int)B, (int)Lp}, n{neg_loc, 4, (int)B, (int)Ln};
  if (int rc = rel_check(a, "savqa_rel_loss_fwd")) return rc;
  if (int rc = rel_check(n, "savqa_rel_loss_fwd")) return rc;
  if (B > REL_MAXB) return fail(SAVQA_EUNSUP, "savqa_rel_loss_fwd: batch > 64");
  if (B * (Lp + Ln) > INT32_MAX) return fail(SAVQA_EUNSUP, "savqa_rel_loss_fwd: > 2^31 slots");
  if (!ws || ws_bytes < savqa_rel_loss_ws_bytes(B, Lp, Ln))
    return fail(SAVQA_EINVAL, "savqa_rel_loss_fwd: workspace smaller than savqa_rel_loss_ws_bytes");
  int G, chunk;
  rel_fold_shape(B * (Lp + Ln), G, chunk);
  float* rec = static_cast<float*>(ws);
  int* cntp = reinterpret_cast<int*>(rec + (int64_t)G * 8);
  int* kmxp = cntp + (int64_t)G * B;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(rel_loss_part_kernel, dim3(G), dim3(REL_NT), 0, s, a, sp, n, sn, eps, chunk,
                     rec, cntp, kmxp);
  if (int rc = check_launch("savqa_rel_loss_fwd(part)")) return rc;
  hipLaunchKernelGGL(rel_loss_fold_kernel, dim3(G), dim3(REL_NT), 0, s, a, sp, chunk, G, rec, cntp,
                     kmxp, cum, wsm, st, mil_rel);
  return check_launch("savqa_rel_loss_fwd(fold)");
}

extern "C" int savqa_rel_macro_fwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp,
                                   const float* st, const float* wsm, const float* relf, int64_t Ns,
                                   int64_t H, float* macro) {
  RelSlots a{pos_loc, 5, (int)B, (int)Lp};
  if (int rc = rel_check(a, "savqa_rel_macro_fwd")) return rc;
  if (H > 1024) return fail(SAVQA_EUNSUP, "savqa_rel_macro_fwd: H > 1024");
  const int64_t S = B * Lp;
  if (S == 0) return 0;
  hipLaunchKernelGGL(rel_macro_fwd_kernel, dim3((unsigned)((S + 3) / 4)), dim3(256), 0,
                     as_stream(stream), a, st, wsm, relf, (int)Ns, (int)H, macro);
  return check_launch("savqa_rel_macro_fwd");
}

extern "C" int savqa_rel_macro_bwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp,
                                   const float* st, const float* wsm, const float* relf, int64_t Ns,
                                   int64_t H, float* dmacro, float* dwsm, float* drelf) {
  RelSlots a{pos_loc, 5, (int)B, (int)Lp};
  if (int rc = rel_check(a, "savqa_rel_macro_bwd")) return rc;
  const int64_t S = B * Lp;
  if (S == 0) return 0;
  const dim3 g((unsigned)((S + 3) / 4));
  hipLaunchKernelGGL(rel_macro_bwd_kernel, g, dim3(256), 0, as_stream(stream), a, st, wsm, relf,
                     (int)Ns, (int)H, dmacro, dwsm, drelf);
  if (int rc = check_launch("savqa_rel_macro_bwd")) return rc;
  hipLaunchKernelGGL(rel_zero_rows_kernel, g, dim3(256), 0, as_stream(stream), a, (int)Ns, (int)H,
                     dmacro);
  return check_launch("savqa_rel_macro_bwd(zero)");
}

extern "C" int savqa_rel_loss_bwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp,
                                  const float* sp, const int64_t* neg_loc, int64_t Ln,
                                  const float* sn, float eps, const int32_t* cum, const float* wsm,
                                  const float* dwsm, float* st, const float* dmil, float* dsp,
                                  float* dsn, void* ws, int64_t ws_bytes) {
  RelSlots a{pos_loc, 5, (int)B, (int)Lp}, n{neg_loc, 4, (int)B, (int)Ln};
  if (int rc = rel_check(a, "savqa_rel_loss_bwd")) return rc;
  if (int rc = rel_check(n, "savqa_rel_loss_bwd")) return rc;
  if (!ws || ws_bytes < savqa_rel_loss_ws_bytes(B, Lp, Ln))
    return fail(SAVQA_EINVAL, "savqa_rel_loss_bwd: workspace smaller than savqa_rel_loss_ws_bytes");
  hipStream_t s = as_stream(stream);
  int Gw, chunk;
  rel_fold_shape(B * Lp, Gw, chunk);  // P <= B * Lp valid positives
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(rel_wdot_part_kernel, dim3(Gw), dim3(REL_NT), 0, s, wsm, dwsm, st, chunk, part);
  if (int rc = check_launch("savqa_rel_loss_bwd(wdot)")) return rc;
  const int64_t n_all = B * Lp + B * Ln;
  if (n_all == 0) return 0;
  hipLaunchKernelGGL(rel_loss_bwd_kernel, dim3((unsigned)((n_all + 255) / 256)), dim3(256), 0, s, a,
                     sp, n, sn, eps, cum, wsm, dwsm, st, part, Gw, dmil, dsp, dsn);
  return check_launch("savqa_rel_loss_bwd");
}
