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
  if (lr[3] < 0) return;
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

// Scalar chain, one workgroup. Writes: cidx[c] = slot of the c-th valid positive (the
// reference's nonzero() order: b-major, then k), wsm[c] = softmax over the valid positives
// (:420), st[0..5] = (P, m1, Z1, m2, Z2, mx/Zsm packed below), mil_rel.
//   mil_rel = LSE_c(max(sp_c, eps)) - LSE(max(sp, eps) ++ max(sn, eps))   (:405-406)
__global__ __launch_bounds__(256) void rel_loss_fwd_kernel(RelSlots sp_s, const float* __restrict__ sp,
                                                          RelSlots sn_s, const float* __restrict__ sn,
                                                          float eps, int* __restrict__ cidx,
                                                          float* __restrict__ wsm,
                                                          float* __restrict__ st,
                                                          float* __restrict__ mil_rel) {
  __shared__ float red[4];
  __shared__ int count;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int S = sp_s.B * sp_s.L, Sn = sn_s.B * sn_s.L;
  if (tid == 0) {  // ordered compaction (S is small: slots = B x max_rel_len)
    int c = 0;
    for (int slot = 0; slot < S; ++slot)
      if (slot_valid(sp_s, slot)) cidx[c++] = slot;
    count = c;
  }
  __syncthreads();
  const int P = count;
  auto block_max = [&](float v) {
    v = wave_max(v);
    if (lane == 0) red[w] = v;
    __syncthreads();
    const float r = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    return r;
  };
  auto block_sum = [&](float v) {
    v = wave_sum(v);
    if (lane == 0) red[w] = v;
    __syncthreads();
    const float r = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
    return r;
  };
  // LSE over clamped positives, and over clamped positives ++ clamped negatives
  float m1 = -INFINITY, mn = -INFINITY, mr = -INFINITY;
  for (int c = tid; c < P; c += blockDim.x) {
    m1 = fmaxf(m1, fmaxf(sp[cidx[c]], eps));
    mr = fmaxf(mr, sp[cidx[c]]);
  }
  for (int slot = tid; slot < Sn; slot += blockDim.x)
    if (slot_valid(sn_s, slot)) mn = fmaxf(mn, fmaxf(sn[slot], eps));
  m1 = block_max(m1);
  mr = block_max(mr);
  const float m2 = fmaxf(m1, block_max(mn));
  float z1 = 0.f, z2 = 0.f, zr = 0.f;
  for (int c = tid; c < P; c += blockDim.x) {
    const float v = fmaxf(sp[cidx[c]], eps);
    z1 += expf(v - m1);
    z2 += expf(v - m2);
    zr += expf(sp[cidx[c]] - mr);
  }
  for (int slot = tid; slot < Sn; slot += blockDim.x)
    if (slot_valid(sn_s, slot)) z2 += expf(fmaxf(sn[slot], eps) - m2);
  z1 = block_sum(z1);
  z2 = block_sum(z2);
  zr = block_sum(zr);
  for (int c = tid; c < P; c += blockDim.x) wsm[c] = expf(sp[cidx[c]] - mr) / zr;
  if (tid == 0) {
    st[0] = (float)P;
    st[1] = m1;
    st[2] = z1;
    st[3] = m2;
    st[4] = z2;
    *mil_rel = P > 0 ? (m1 + logf(z1)) - (m2 + logf(z2)) : NAN;
  }
}

// Ordered macro-node update (:418, :421-436): rows macro[b, loc3] of every valid positive
// are zeroed, then, entry by entry, macro[b, loc3] += wsm[loc4] * relf[b, loc4].
// One workgroup: threads over columns, entries in the reference's order.
__global__ __launch_bounds__(256) void rel_macro_fwd_kernel(RelSlots s, const int* __restrict__ cidx,
                                                           const float* __restrict__ st,
                                                           const float* __restrict__ wsm,
                                                           const float* __restrict__ relf, int Ns,
                                                           int H, float* __restrict__ macro) {
  const int P = (int)st[0];
  for (int c = 0; c < P; ++c) {
    const int slot = cidx[c];
    const int64_t* lr = s.loc + (int64_t)slot * s.W;
    float* row = macro + ((int64_t)(slot / s.L) * Ns + lr[3]) * H;
    for (int h = threadIdx.x; h < H; h += blockDim.x) row[h] = 0.f;
  }
  __syncthreads();
  for (int c = 0; c < P; ++c) {
    const int slot = cidx[c];
    const int64_t* lr = s.loc + (int64_t)slot * s.W;
    const int b = slot / s.L;
    float* row = macro + ((int64_t)b * Ns + lr[3]) * H;
    if (lr[4] >= P) continue;  // (the reference would index out of range)
    const float wv = wsm[lr[4]];
    const float* src = relf + ((int64_t)b * s.L + lr[4]) * H;
    for (int h = threadIdx.x; h < H; h += blockDim.x) row[h] += wv * src[h];
  }
}

// Backward of the update, one wave per entry: dwsm[loc4] += dmacro[b,loc3] . relf[b,loc4],
// drelf[b,loc4] += wsm[loc4] * dmacro[b,loc3]. (The zeroing of the relation rows' previous
// contents is applied by rel_zero_rows_kernel after this kernel has read dmacro.)
__global__ __launch_bounds__(256) void rel_macro_bwd_kernel(RelSlots s, const int* __restrict__ cidx,
                                                           const float* __restrict__ st,
                                                           const float* __restrict__ wsm,
                                                           const float* __restrict__ relf, int Ns,
                                                           int H, const float* __restrict__ dmacro,
                                                           float* __restrict__ dwsm,
                                                           float* __restrict__ drelf) {
  const int P = (int)st[0];
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (c >= P) return;
  const int slot = cidx[c];
  const int64_t* lr = s.loc + (int64_t)slot * s.W;
  const int b = slot / s.L;
  const float* drow = dmacro + ((int64_t)b * Ns + lr[3]) * H;
  if (lr[4] >= P) return;
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

__global__ __launch_bounds__(256) void rel_zero_rows_kernel(RelSlots s, const int* __restrict__ cidx,
                                                           const float* __restrict__ st, int Ns,
                                                           int H, float* __restrict__ dmacro) {
  const int P = (int)st[0];
  for (int c = blockIdx.x; c < P; c += gridDim.x) {
    const int slot = cidx[c];
    const int64_t* lr = s.loc + (int64_t)slot * s.W;
    float* row = dmacro + ((int64_t)(slot / s.L) * Ns + lr[3]) * H;
    for (int h = threadIdx.x; h < H; h += blockDim.x) row[h] = 0.f;
  }
}

// Scalar-chain backward (one workgroup): dsp / dsn per slot from
//   d mil_rel (through both clamped logsumexps; clamp passes gradient where x >= eps)
//   + the softmax path: dsp[cidx[c]] += wsm[c] (dwsm[c] - sum_c' wsm[c'] dwsm[c'])
__global__ __launch_bounds__(256) void rel_loss_bwd_kernel(RelSlots sp_s, const float* __restrict__ sp,
                                                          RelSlots sn_s, const float* __restrict__ sn,
                                                          float eps, const int* __restrict__ cidx,
                                                          const float* __restrict__ wsm,
                                                          const float* __restrict__ dwsm,
                                                          const float* __restrict__ st,
                                                          const float* __restrict__ dmil,
                                                          float* __restrict__ dsp,
                                                          float* __restrict__ dsn) {
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int P = (int)st[0];
  const float m1 = st[1], z1 = st[2], m2 = st[3], z2 = st[4];
  const float g = dmil ? *dmil : 0.f;
  const int S = sp_s.B * sp_s.L, Sn = sn_s.B * sn_s.L;
  for (int slot = tid; slot < S; slot += blockDim.x) dsp[slot] = 0.f;
  for (int slot = tid; slot < Sn; slot += blockDim.x) {
    float d = 0.f;
    if (slot_valid(sn_s, slot) && sn[slot] >= eps) d = -g * expf(sn[slot] - m2) / z2;
    dsn[slot] = d;
  }
  float t = 0.f;
  for (int c = tid; c < P; c += blockDim.x) t += wsm[c] * dwsm[c];
  t = wave_sum(t);
  if (lane == 0) red[w] = t;
  __syncthreads();
  const float wd = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();  // dsp zeroed before the scattered writes below
  for (int c = tid; c < P; c += blockDim.x) {
    const int slot = cidx[c];
    const float v = sp[slot];
    float d = 0.f;
    if (v >= eps) d = g * (expf(v - m1) / z1 - expf(v - m2) / z2);
    d += wsm[c] * (dwsm[c] - wd);
    dsp[slot] = d;
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

extern "C" int savqa_rel_loss_fwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp,
                                  const float* sp, const int64_t* neg_loc, int64_t Ln,
                                  const float* sn, float eps, int32_t* cidx, float* wsm, float* st,
                                  float* mil_rel) {
  RelSlots a{pos_loc, 5, (int)B, (int)Lp}, n{neg_loc, 4, (int)B, (int)Ln};
  if (int rc = rel_check(a, "savqa_rel_loss_fwd")) return rc;
  if (int rc = rel_check(n, "savqa_rel_loss_fwd")) return rc;
  hipLaunchKernelGGL(rel_loss_fwd_kernel, dim3(1), dim3(256), 0, as_stream(stream), a, sp, n, sn, eps,
                     cidx, wsm, st, mil_rel);
  return check_launch("savqa_rel_loss_fwd");
}

extern "C" int savqa_rel_macro_fwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp,
                                   const int32_t* cidx, const float* st, const float* wsm,
                                   const float* relf, int64_t Ns, int64_t H, float* macro) {
  RelSlots a{pos_loc, 5, (int)B, (int)Lp};
  if (int rc = rel_check(a, "savqa_rel_macro_fwd")) return rc;
  hipLaunchKernelGGL(rel_macro_fwd_kernel, dim3(1), dim3(256), 0, as_stream(stream), a, cidx, st, wsm,
                     relf, (int)Ns, (int)H, macro);
  return check_launch("savqa_rel_macro_fwd");
}

extern "C" int savqa_rel_macro_bwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp,
                                   const int32_t* cidx, const float* st, const float* wsm,
                                   const float* relf, int64_t Ns, int64_t H, float* dmacro,
                                   float* dwsm, float* drelf) {
  RelSlots a{pos_loc, 5, (int)B, (int)Lp};
  if (int rc = rel_check(a, "savqa_rel_macro_bwd")) return rc;
  const int64_t S = B * Lp;
  if (S == 0) return 0;
  hipLaunchKernelGGL(rel_macro_bwd_kernel, dim3((unsigned)((S + 3) / 4)), dim3(256), 0,
                     as_stream(stream), a, cidx, st, wsm, relf, (int)Ns, (int)H, dmacro, dwsm, drelf);
  if (int rc = check_launch("savqa_rel_macro_bwd")) return rc;
  hipLaunchKernelGGL(rel_zero_rows_kernel, dim3(64), dim3(256), 0, as_stream(stream), a, cidx, st,
                     (int)Ns, (int)H, dmacro);
  return check_launch("savqa_rel_macro_bwd(zero)");
}

extern "C" int savqa_rel_loss_bwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp,
                                  const float* sp, const int64_t* neg_loc, int64_t Ln,
                                  const float* sn, float eps, const int32_t* cidx, const float* wsm,
                                  const float* dwsm, const float* st, const float* dmil, float* dsp,
                                  float* dsn) {
  RelSlots a{pos_loc, 5, (int)B, (int)Lp}, n{neg_loc, 4, (int)B, (int)Ln};
  if (int rc = rel_check(a, "savqa_rel_loss_bwd")) return rc;
  if (int rc = rel_check(n, "savqa_rel_loss_bwd")) return rc;
  hipLaunchKernelGGL(rel_loss_bwd_kernel, dim3(1), dim3(256), 0, as_stream(stream), a, sp, n, sn, eps,
                     cidx, wsm, dwsm, st, dmil, dsp, dsn);
  return check_launch("savqa_rel_loss_bwd");
}
