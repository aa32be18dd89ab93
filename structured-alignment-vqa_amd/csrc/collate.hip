// Batch collation on the device.
//
// The reference's collate_fn (models/data_loader_itp_bbox_super_node_onlyobj.py:341-445;
// dataloader/data_loader_itp_bbox_super_node.py:366-497) pads every per-sample array to
// the batch maximum on the host and builds dense int32 (B,T,T) masks and graphs there,
// then the whole padded batch crosses PCIe. Here the host only packs the ragged arrays
// back to back (plus per-sample row offsets) into one staging buffer; this file expands
// them into the same dense tensors in HBM:
//   savqa_collate        one launch for every padded field of the batch: each workgroup
//                        writes a 4 KB chunk of one sample of one field (valid rows copied
//                        from the packed source, the rest filled; masks computed from the
//                        per-sample lengths); every store is a 16-B vector on the output's
//                        16-B grid (a sample's unaligned head/tail words aside), loads are
//                        16-B vectors where the packed source lines up too;
//   savqa_collate_edges  one thread per edge: graph[b][i][j] = 1 (after the zero fill).
// Pure HBM streaming: bytes written = the dense batch, bytes read = the packed batch.
#include "common.h"

namespace savqa {

constexpr int kColNT = 256;                 // threads per workgroup
constexpr int kColIter = 4;                 // 16-B groups per thread
constexpr int kColWords = kColNT * 4 * kColIter;  // 32-bit words per chunk (16 KB)

struct CollateArgs {
  savqa_collate_field f[SAVQA_COLLATE_MAX_FIELDS];
  int64_t first[SAVQA_COLLATE_MAX_FIELDS + 1];  // first workgroup of each field
  int64_t chunks[SAVQA_COLLATE_MAX_FIELDS];     // chunks per sample
  int32_t nfields;
};

__device__ __forceinline__ uint32_t fill_word(const savqa_collate_field& f, int64_t w) {
  // 8-byte elements start on even words of a sample (sample bases are element aligned)
  return (f.elem_bytes == 8 && (w & 1)) ? (uint32_t)(f.fill >> 32) : (uint32_t)f.fill;
}

// one 16-B group (words w0 .. w0+3 of sample b's dense output) of field f
__device__ __forceinline__ void collate_group(const savqa_collate_field& f, int64_t b,
                                              uint32_t* __restrict__ dst, int64_t wps,
                                              int64_t w0) {
  using u4 = uint32_t __attribute__((ext_vector_type(4)));
  const bool full = w0 >= 0 && w0 + 4 <= wps;  // whole aligned group inside the sample
  uint32_t v[4];
  if (f.kind == SAVQA_COLLATE_BOX) {
    // int32 mask value of word w = (t, c): t < n && (!square || c < n); one 32-bit
    // division per group (T * row_elems < 2^31 checked on the host)
    const int n = (int)(f.off[b + 1] - f.off[b]);
    const int C = (int)f.row_elems;
    const int ws = (int)(w0 < 0 ? 0 : w0);
    int t = ws / C, c = ws - t * C;
    const int qs = (int)(ws - w0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= qs) {
        v[q] = (t < n && (!f.square || c < n)) ? 1u : 0u;
        if (++c == C) { c = 0; ++t; }
      }
    }
  } else {
    int64_t valid = 0;  // words of this sample that come from the source
    const uint32_t* src = nullptr;
    if (f.kind == SAVQA_COLLATE_ROWS) {
      const int64_t r0 = f.off[b];
      const int64_t epw = f.row_elems * f.elem_bytes / 4;  // words per row
      valid = min((f.off[b + 1] - r0) * epw, wps);
      src = reinterpret_cast<const uint32_t*>(f.src) + r0 * epw;
    }
    if (full && w0 + 4 <= valid && ((reinterpret_cast<uintptr_t>(src + w0) & 15) == 0)) {
      const u4 x = *reinterpret_cast<const u4*>(src + w0);
      v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t w = w0 + q;
        if (w >= 0 && w < wps) v[q] = (w < valid) ? src[w] : fill_word(f, w);
      }
    }
  }
  if (full) {
    *reinterpret_cast<u4*>(dst + w0) = u4{v[0], v[1], v[2], v[3]};
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t w = w0 + q;
      if (w >= 0 && w < wps) dst[w] = v[q];
    }
  }
}

__global__ __launch_bounds__(kColNT) void collate_kernel(CollateArgs a) {
  const uint32_t bid = blockIdx.x;
  int fi = 0;
  while (fi + 1 < a.nfields && bid >= (uint32_t)a.first[fi + 1]) ++fi;
  const savqa_collate_field& f = a.f[fi];
  const uint32_t local = bid - (uint32_t)a.first[fi];
  const uint32_t cps = (uint32_t)a.chunks[fi];
  const int64_t b = local / cps;
  const int64_t chunk = local - (uint32_t)b * cps;
  const int64_t wps = f.T * f.row_elems * f.elem_bytes / 4;  // words per sample
  uint32_t* dst = reinterpret_cast<uint32_t*>(f.dst) + b * wps;
  // 4-word groups are laid on the 16-B grid of dst: the sample's first `head` words (its
  // base is only 4-B aligned in general) form a partial group -1 (host adds one group)
  const int head = (int)(((16u - (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u) >> 2);
  const int64_t base = chunk * kColWords + head - (head ? 4 : 0);
#pragma unroll
  for (int k = 0; k < kColIter; ++k) {  // group k*256 + tid: each store wave-contiguous
    const int64_t w0 = base + 4 * (int64_t)(k * kColNT + threadIdx.x);
    if (w0 < wps) collate_group(f, b, dst, wps, w0);
  }
}

// graph[b][e0][e1] = 1 for every edge of sample b (edge_off: per-sample edge offsets)
__global__ __launch_bounds__(256) void collate_edges_kernel(const int32_t* __restrict__ edges,
                                                            const int64_t* __restrict__ edge_off,
                                                            int64_t B, int64_t E, int64_t T,
                                                            int32_t* __restrict__ graph) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  int64_t lo = 0, hi = B;  // sample b with edge_off[b] <= e < edge_off[b+1]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (edge_off[mid] <= e) lo = mid; else hi = mid;
  }
  const int64_t i = edges[2 * e], j = edges[2 * e + 1];
  if (i < 0 || i >= T || j < 0 || j >= T) return;  // host validated; never write out of bounds
  graph[(lo * T + i) * T + j] = 1;
}

}  // namespace savqa

using namespace savqa;

extern "C" int savqa_collate(void* stream, const savqa_collate_field* fields, int32_t nfields,
                             int64_t B) {
  if (B <= 0 || nfields <= 0) return 0;
  if (nfields > SAVQA_COLLATE_MAX_FIELDS)
    return fail(SAVQA_EINVAL, "savqa_collate: too many fields");
  CollateArgs a{};
  a.nfields = nfields;
  int64_t total = 0;
  for (int i = 0; i < nfields; ++i) {
    const savqa_collate_field& f = fields[i];
    if (f.kind < SAVQA_COLLATE_ROWS || f.kind > SAVQA_COLLATE_FILL)
      return fail(SAVQA_EINVAL, "savqa_collate: bad field kind");
    if ((f.elem_bytes != 4 && f.elem_bytes != 8) || (f.kind == SAVQA_COLLATE_BOX && f.elem_bytes != 4))
      return fail(SAVQA_EINVAL, "savqa_collate: elem_bytes must be 4 or 8 (BOX: 4)");
    if (f.T < 0 || f.row_elems < 0 || !f.dst || (f.kind != SAVQA_COLLATE_FILL && !f.off) ||
        (f.kind == SAVQA_COLLATE_ROWS && !f.src))
      return fail(SAVQA_EINVAL, "savqa_collate: bad field");
    if (f.kind == SAVQA_COLLATE_BOX && f.square && f.row_elems != f.T)
      return fail(SAVQA_EINVAL, "savqa_collate: square mask needs row_elems == T");
    const int64_t words = f.T * f.row_elems * f.elem_bytes / 4;
    if (words >= ((int64_t)1 << 31)) return fail(SAVQA_EUNSUP, "savqa_collate: sample too large");
    a.f[i] = f;
    // + one group: a sample's 16-B grid may start up to 3 words in (see the kernel)
    a.chunks[i] = (words + 4 + kColWords - 1) / kColWords;
    a.first[i] = total;
    total += B * a.chunks[i];
  }
  a.first[nfields] = total;
  if (total >= (int64_t)1 << 31) return fail(SAVQA_EUNSUP, "savqa_collate: batch too large");
  hipLaunchKernelGGL(collate_kernel, dim3((unsigned)total), dim3(kColNT), 0, as_stream(stream), a);
  return check_launch("savqa_collate");
}

extern "C" int savqa_collate_edges(void* stream, const int32_t* edges, const int64_t* edge_off,
                                   int64_t B, int64_t E, int64_t T, int32_t* graph) {
  if (B <= 0 || E <= 0) return 0;
  if (T <= 0 || !edges || !edge_off || !graph)
    return fail(SAVQA_EINVAL, "savqa_collate_edges: bad arguments");
  hipLaunchKernelGGL(collate_edges_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0,
                     as_stream(stream), edges, edge_off, B, E, T, graph);
  return check_launch("savqa_collate_edges");
}
