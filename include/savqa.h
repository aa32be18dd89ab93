/*
 * savqa.h -- C ABI of libsavqa.so, the MI355X (gfx950) kernel library behind the
 * SA-VQA model_v=3 structured-alignment hot path.
 *
 * The reference (Peixixiong/Structured-Alignment-VQA) has no FFI: every op is a
 * PyTorch/ATen call from Python. Each entry point below replaces the ATen op
 * sequence of the reference function cited in its comment (file:line under
 * models/). The host side (structured-alignment-vqa_amd/, imported as savqa_amd)
 * binds these with ctypes.
 *
 * Conventions (all entry points):
 *  - every pointer is a device pointer owned by the caller; the library never
 *    allocates or frees device memory and keeps no state between calls;
 *  - all work is enqueued asynchronously on `stream` (a hipStream_t); no host
 *    synchronisation happens inside, so calls are capturable into hipGraphs;
 *  - tensors are fp32 unless stated; index tensors are int64 (as the reference's
 *    collate_fn produces them); mask/graph inputs are int32;
 *  - return 0 on success, a hipError_t (>0) or a negative SAVQA_E* code on
 *    failure; savqa_last_error() returns a thread-local message.
 */
#ifndef SAVQA_H
#define SAVQA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SAVQA_EINVAL (-1)   /* bad shape / argument */
#define SAVQA_EUNSUP (-2)   /* shape outside what the kernel supports */

int savqa_version(void);
const char* savqa_last_error(void);
/* sizeof of the descriptor structs, for bindings to check their layouts: out[0] =
 * savqa_gemm_desc, out[1] = savqa_gemm_lp_desc, out[2] = savqa_collate_field; n >= 3;
 * with n >= 4 also out[3] = savqa_x6_planes_job */
int savqa_struct_sizes(int64_t* out, int32_t n);

/* ------------------------------------------------------------------------
 * GEMM:  C[crow(m)][n] (op)= epilogue( sum_k A(m,k) * B(k,n) )
 * Replaces every nn.Linear of the path (modules.py:135-137, 227-229, 428-429;
 * AttModel_x3.py:42-44, 173-175, 316-335, 482-500) and their backward GEMMs.
 *   A(m,k) = a_trans ? A[ra(k)*lda + m] : A[ra(m)*lda + k]   ra(i) = a_rows ? a_rows[i] : i
 *   B(k,n) = b_trans ? B[rb(n)*ldb + k] : B[rb(k)*ldb + n]   rb(i) = b_rows ? b_rows[i] : i
 *            (b_trans=1: nn.Linear weight [N][K]; the *_rows gathers implement F.embedding)
 *   crow(m) = c_rows ? c_rows[m] : (m / c_group) * c_stride + (m % c_group) + c_offset
 *   v = acc*alpha + bias[n] + rowvec[(m % rowvec_period)*ldrv + n]
 *   v = relu ? max(v,0) : v ;  v *= rowscale[m] ;
 *   v = (mask && !(mask[mr*ldmask+n] > 0)) ? 0 : v   mr = mask_arows ? a_rows[m] : m
 *   v += resid[m*ldr + n]
 *   C = atomic ? C + v (atomicAdd) : v + beta*C
 * split_k > 1 splits K across workgroups and forces atomic accumulation; split_k < 0
 * (requires atomic=1) lets the library pick the split from the tile count and CU count.
 * Non-atomic launches with a linear epilogue (relu=0, beta=0, C not aliasing resid) may
 * split the last partial wave of tiles over K internally (zero-fill + atomics): results
 * then differ from a single-pass launch only in fp32 summation order.
 * prec 1: the skinny (M = B row) launches round both operands to bf16 and use one bf16 MFMA
 * per 16 k (gemm_skinny_bf_kernel; k-row gathers stay fp32), the 128x128 ones run as prec 6.
 * prec (128x128-tile launches; the skinny kernel stays fp32): 3 = each operand split into
 * bf16 hi + lo (lo = bf16(x - hi)) and a*b ~ ah*bh + ah*bl + al*bh on
 * v_mfma_f32_32x32x16_bf16: ~2^-16 relative per product (the "bf16x3" mode). The bf16
 * training mode (BASELINE cfg 3) uses savqa_gemm_lp on bf16-resident operands instead.
 * ------------------------------------------------------------------------ */
typedef struct savqa_gemm_desc {
    int64_t M, N, K;
    const float* A; int64_t lda; int32_t a_trans;
    int32_t prec;      /* products: 0 fp32 MFMA (exact), 1 bf16 on the skinny launches (x6
                          else), 3 3xbf16 split, 6 fp32 from exact three-term bf16 splits
                          (six bf16 MFMA products, gemm_x6.hip) */
    const int64_t* a_rows;
    const float* B; int64_t ldb; int32_t b_trans; int32_t _pad1;
    const int64_t* b_rows;
    float* C; int64_t ldc;
    int64_t c_group, c_stride, c_offset;
    const int64_t* c_rows;
    const float* bias;
    const float* rowvec; int64_t ldrv; int64_t rowvec_period;
    const float* resid; int64_t ldr;
    const float* mask; int64_t ldmask; int64_t mask_arows;
    const float* rowscale;
    float alpha, beta;
    int32_t relu, atomic, split_k, _pad2;
    float* colsum_a;   /* optional, a_trans=1 only: colsum_a[m] += sum_k A(m,k) (bias grad) */
    float* ws; int64_t ws_elems;  /* optional split-K / tail-split workspace (fp32 elements,
                          >= savqa_gemm_ws_elems(d)): the 128x128 fp32 / x6 kernels then store
                          each K slice's partial tile (and its column sums) with plain stores
                          and add the slices in a fixed order in a second pass -- results no
                          longer depend on the order atomics land in, i.e. run to run
                          deterministic (a c_rows scatter / row map keeps its atomics) */
    const void* b_planes;  /* optional, x6 (prec 5 / 6) launches with !a_trans only: B as the
                          x6 kernel's LDS images, pre-split by savqa_x6_weight_planes for
                          exactly this B (same N, K, layout); the kernel then DMAs B's three
                          bf16 planes instead of loading and splitting B (the weights of the
                          forward / dX GEMMs: split once per optimizer step, not per tile).
                          Results are bit-identical to the launch without it. NULL: off */
} savqa_gemm_desc;

/* The x6 kernel's bf16 plane images of a GEMM's B operand (the N x K operand of
 * savqa_gemm's formula; b_trans = 1: B(n, k) = Bp[n * ldb + k], else B(n, k) = Bp[k * ldb + n]):
 * for every 128-row n tile and 32-wide k tile, 3 planes x 128 x 32 bf16 (24 KB) at
 * out + (nt * ceil(K / 32) + kt) * 24576 bytes, each value split exactly into the three
 * truncated bf16 terms gemm_x6 makes, in its swizzled order; zeros past N and K.
 * out: savqa_x6_weight_planes_bytes(N, K) bytes, 16-B aligned. */
int64_t savqa_x6_weight_planes_bytes(int64_t N, int64_t K);
int savqa_x6_weight_planes(void* stream, const float* Bp, int64_t ldb, int32_t b_trans, int64_t N,
                           int64_t K, void* out);
/* Many operands' plane images at once (an optimizer step's weights: a few launches instead of
 * one per weight). jobs: HOST array of n entries, read before the call returns; each as
 * savqa_x6_weight_planes' arguments (entries with N or K <= 0 are skipped). */
typedef struct savqa_x6_planes_job {
    const float* B;
    int64_t ldb;
    int32_t b_trans, reserved;
    int64_t N, K;
    void* out;
} savqa_x6_planes_job;
int savqa_x6_weight_planes_batch(void* stream, const savqa_x6_planes_job* jobs, int32_t n);

int savqa_gemm(void* stream, const savqa_gemm_desc* d);
/* fp32 elements of workspace *d's launch would use for split-K / tail-split slabs (0: the plan
 * has no K split, or its epilogue cannot take slabs: c_rows scatter, row map, relu, beta) */
int64_t savqa_gemm_ws_elems(const savqa_gemm_desc* d);

/* The launch plan savqa_gemm would use for *d (no launch): out[0] = tile (16 / 32: skinny
 * kernels, 128), out[1] = split-K factor, out[2] = tail split factor (0: none),
 * out[3] = workgroups. */
int savqa_gemm_plan(const savqa_gemm_desc* d, int32_t* out);

/* ------------------------------------------------------------------------
 * Low-precision-operand GEMM (BASELINE cfg 3 bf16 training, cfg 5 fp8 region features):
 * the same operator as savqa_gemm, with bf16-RESIDENT operands (or fp8-e4m3 ones with
 * per-32-k block scales) read straight from HBM, fp32 accumulation, and an fp32 and/or
 * bf16 output.
 *   A(m,k) = a_trans ? A[k*lda + m] : A[ra(m)*lda + k]     ra(i) = a_rows ? a_rows[i] : i
 *   B(k,n) = b_trans ? B[n*ldb + k] : B[k*ldb + n]
 *   a_type / b_type: SAVQA_DT_BF16 or SAVQA_DT_FP8 (OCP e4m3fn). fp8 needs both operands
 *   fp8, a_trans = 0, b_trans = 1, K % 128 == 0, and e8m0 block scales a_scale[m][k/32]
 *   (row stride lds_a bytes, 4-byte aligned rows) / b_scale[n][k/32]: value = e4m3 * 2^(scale - 127)
 *   (v_mfma_scale_f32_16x16x128_f8f6f4). bf16 needs K % 8 == 0 (unless both operands are
 *   k-major: a_trans = 1, b_trans = 0), 16-B aligned operands with ld % 8 == 0, and M % 8 == 0
 *   (a_trans) / N % 8 == 0 (b_trans = 0).
 *   v = acc*alpha + bias[n] + rowvec[(m % rowvec_period)*ldrv + n]  (bias/rowvec/resid:
 *       first K slice only) ; v = relu ? max(v,0) : v ;
 *   v = (mask && !(mask[mr*ldmask+n] > 0)) ? 0 : v   mr = mask_arows ? a_rows[m] : m
 *       (mask_type SAVQA_DT_BF16 or SAVQA_DT_F32; SAVQA_DT_BITS: the gate is bit (n & 7) of
 *       byte ((uint8_t*)mask)[mr*ldmask + n/8], ldmask in bytes, bf16-only outputs Cb with
 *       N % 8 == 0 and no C / resid / rowvec / atomic) ; v += resid[m*ldr + n]
 *   crow(m) = (m / c_group)*c_stride + m % c_group + c_offset  (c_group <= 0: identity)
 *   C[crow*ldc + n] = v  (atomic: +=)      Cb[crow*ldcb + n] = bf16(v)  (not with atomic)
 * split_k > 1 / < 0 (auto) requires atomic = 1 and C. savqa_gemm_lp_supported() says
 * whether a descriptor meets these constraints (no launch).
 * ------------------------------------------------------------------------ */
#define SAVQA_DT_F32 0
#define SAVQA_DT_BF16 1
#define SAVQA_DT_FP8 2
#define SAVQA_DT_BITS 3  /* mask_type only: one bit per element (see savqa_gemm_lp_desc) */
typedef struct savqa_gemm_lp_desc {
    int64_t M, N, K;
    const void* A; int64_t lda; int32_t a_trans; int32_t a_type;
    const int64_t* a_rows;
    const uint8_t* a_scale; int64_t lds_a;
    const void* B; int64_t ldb; int32_t b_trans; int32_t b_type;
    const uint8_t* b_scale; int64_t lds_b;
    float* C; int64_t ldc;
    void* Cb; int64_t ldcb;
    int64_t c_group, c_stride, c_offset;
    const float* bias;
    const float* rowvec; int64_t ldrv; int64_t rowvec_period;
    const float* resid; int64_t ldr;
    const void* mask; int64_t ldmask; int32_t mask_arows; int32_t mask_type;
    float alpha;
    int32_t relu, atomic, split_k;
    int32_t tile_hint;  /* 0 = library's choice; 1..5 force a kernel variant (gemm_lp.hip) */
    const int64_t* c_rows;  /* atomic only: output row of m is c_rows[m] (scatter-add) */
    int64_t n_store;        /* atomic only, > 0: columns >= n_store are not stored (an operand
                               zero-padded to a multiple of 8 columns, C rows n_store wide) */
    float* ws; int64_t ws_elems;  /* optional split-K workspace (fp32 elements): a split-K
                               launch into fp32 C with a linear epilogue (no relu / mask / Cb /
                               c_rows / row map; n_store a multiple of 4) and ws_elems >=
                               slices*M*(N + (colsum_a != 0)) stores each K slice's partial tile
                               (and column sums) with plain stores and then adds the slices into
                               C (and colsum_a) in one pass in slice order (C += sum), instead
                               of fp32 atomics */
    float* colsum_a;        /* optional, a_trans = 1, bf16: colsum_a[m] += sum_k A(m, k) (the
                               bias gradient of dW = dY^T X), summed in fp32 from the staged A
                               tiles by the 128x128 kernel; other kernels add it in a separate
                               (atomic) column-sum pass */
    uint8_t* bits_out; int64_t ldbits;  /* optional, bf16-only outputs (Cb; N % 8 == 0; no C /
                               resid / rowvec / atomic): bit (n & 7) of byte bits_out[crow*ldbits
                               + n/8] = (Cb[crow*ldcb + n] > 0) -- the ReLU gate of this output
                               as a SAVQA_DT_BITS mask, 1/16 of the bf16 output's bytes */
} savqa_gemm_lp_desc;

int savqa_gemm_lp(void* stream, const savqa_gemm_lp_desc* d);
int savqa_gemm_lp_supported(const savqa_gemm_lp_desc* d);
/* The launch plan savqa_gemm_lp would use for *d (no launch): out[0] = kernel variant
 * (1: 128x128 tile, two workgroups per CU; 3: 256x256; 4: 256x128 -- one per CU),
 * out[1] = K slices, out[2] = workgroups, out[3] = epilogue operand prefetched under the
 * last k-tile (variant 1: 0 none, 1 the residual, 2 the bf16 mask). */
int savqa_gemm_lp_plan(const savqa_gemm_lp_desc* d, int32_t* out);
/* fp32 elements of d.ws that let the launch of *d store partial slabs instead of adding fp32
 * atomics: split-K weight gradients (slices x M x N) and the split-off last round of tiles of
 * long-K launches into fp32 C (tail slices x rows x N, then one ordered reduce that assigns
 * those rows: deterministic, no zero fill). 0 = no slab use. */
int64_t savqa_gemm_lp_ws_elems(const savqa_gemm_lp_desc* d);

/* Conversions feeding the low-precision operands (output row of input row r: ro(r) =
 * (r / group)*stride + r % group + offset, or r when group <= 0 -- e.g. the question rows
 * of a [B][T] concat buffer):
 *   savqa_cast_bf16: out[ro(r)*ldo + c] = bf16(in[r*ldi + c])  (round to nearest even)
 *   savqa_quant_fp8: per row r and 32-column block b: s = e8m0 scale making max|x| <= 448,
 *     q[ro(r)*ldq + c] = e4m3fn(x / 2^(s-127)) (round to nearest even), scale[ro(r)*lds + b]
 *     = s; cols % 32 == 0
 *   savqa_dequant_fp8_bf16: out = bf16(q * 2^(s-127))  (the backward's bf16 copy)
 *   savqa_gather_rows_bf16: out[r*ldo + c] = bf16(table[ids[r]*ldt + c]) for c < cols, 0 for
 *     cols <= c < ldo (GloVe rows of a token list, zero-padded to a multiple of 8 columns:
 *     the K = 300 embedding GEMMs of the low-precision modes) */
int savqa_cast_bf16(void* stream, const float* in, int64_t rows, int64_t cols, int64_t ldi,
                    void* out, int64_t ldo, int64_t group, int64_t stride, int64_t offset);
int savqa_quant_fp8(void* stream, const float* in, int64_t rows, int64_t cols, int64_t ldi,
                    void* q, int64_t ldq, uint8_t* scale, int64_t lds, int64_t group,
                    int64_t stride, int64_t offset);
int savqa_dequant_fp8_bf16(void* stream, const void* q, int64_t rows, int64_t cols, int64_t ldq,
                           const uint8_t* scale, int64_t lds, void* out, int64_t ldo);
/* out[r*ldo + c] = float(in[r*ldi + c]) over bf16 rows (exact): the fp32 Q/K/V the key-tiled
 * attention reads when a low-precision mode meets a sequence longer than 128 */
int savqa_widen_bf16(void* stream, const void* in, int64_t rows, int64_t cols, int64_t ldi,
                     float* out, int64_t ldo);
/* out[c] += sum_r X[r*ldx + c] over a bf16 X (bias gradients of the low-precision GEMMs) */
int savqa_colsum_bf16(void* stream, const void* X, int64_t rows, int64_t cols, int64_t ldx,
                      float* out);
int savqa_gather_rows_bf16(void* stream, const float* table, int64_t ldt, const int64_t* ids,
                           int64_t n, int64_t cols, void* out, int64_t ldo);

/* out[c] += sum_r X[r*ldx + c]  (bias gradients of every Linear above) */
int savqa_colsum_acc(void* stream, const float* X, int64_t rows, int64_t cols, int64_t ldx, float* out);

/* ------------------------------------------------------------------------
 * Residual + layer_normalization (modules.py:62-65: mean, UNBIASED std, eps on std),
 * fused with the residual add of modules.py:304 / :439:
 *   z = x*xscale[row] + r ;  y = gamma*(z-mean)/(std+eps) + beta   (xscale, r optional;
 *   xscale carries the decoder self-attention's query mask, modules.py:187-190)
 * Saves z (if z_out), mean, rden = 1/(std+eps), std; flag[row] = sign(|sum_c y|)
 * (the key/query mask of the next attention, modules.py:257/:289) if flag != NULL.
 * ------------------------------------------------------------------------ */
int savqa_ln_fwd(void* stream, const float* x, const float* xscale, const float* r,
                 int64_t rows, int64_t cols,
                 const float* gamma, const float* beta, float eps,
                 float* z_out, float* y, float* mean, float* rden, float* stdv, float* flag,
                 void* yb /* optional bf16 copy of y (the next low-precision GEMM's operand) */);

/* Backward of the above: dz = dLN/dz (+ dz_add), dgamma += ..., dbeta += ...
 * Per-workgroup column sums land in the caller's workspace `ws` first (ws_bytes >=
 * savqa_ln_bwd_workspace_bytes(cols), 16-B aligned, no initial contents needed);
 * a second tiny kernel on the same stream adds them into dgamma/dbeta in a fixed
 * order (bit-identical run to run), so one workspace serves every later call on the
 * same stream (calls on concurrently running streams need one workspace each). */
int64_t savqa_ln_bwd_workspace_bytes(int64_t cols);
int savqa_ln_bwd(void* stream, const float* dy, const float* z, const float* mean,
                 const float* rden, const float* stdv, const float* gamma,
                 int64_t rows, int64_t cols, const float* dz_add, float* dz,
                 float* dgamma, float* dbeta, float* ws, int64_t ws_bytes,
                 void* dzb /* optional bf16 copy of dz */);

/* flag[r] = sign(|sum_c X[r*ldx+c]|)  (modules.py:257 key mask / :289 query mask) */
int savqa_rowflag(void* stream, const float* X, int64_t rows, int64_t cols, int64_t ldx, float* flag);

/* ------------------------------------------------------------------------
 * Graph-guided attention core, new_multihead_attention.forward modules.py:246-301
 * (after the ReLU'd projections, before the residual):
 *   S = Q_h K_h^T / sqrt(dk);  S[:, j] = -4294967296 where kflag[b,j] == 0
 *   A = softmax_row(S);  Bm = A * G[b];  N = Bm / max(sum|Bm|, 1e-12);  P = N * qflag[b,i]
 *   O_h = P V_h
 * Q/K/V are strided views: row (b*Tq+i) of Q at q + (b*Tq+i)*ldq + h*dk, etc.
 * G is (B, Tq, Tk) fp32 (dense graph / dec_mask). att (optional) receives N in the
 * reference's head-major (h*B + b, Tq, Tk) layout (return_att, modules.py:286).
 * ------------------------------------------------------------------------ */
int savqa_gattn_fwd(void* stream, const float* q, int64_t ldq, const float* k, int64_t ldk,
                    const float* v, int64_t ldv, const float* G, const float* kflag,
                    const float* qflag, int64_t B, int64_t Tq, int64_t Tk, int64_t H, int64_t dk,
                    float* o, int64_t ldo, float* att);

/* Backward: given dO, recompute P and write dQ/dK/dV already multiplied by the
 * ReLU masks of the projections (Q>0 etc.), i.e. the pre-activation gradients. */
int savqa_gattn_bwd(void* stream, const float* q, int64_t ldq, const float* k, int64_t ldk,
                    const float* v, int64_t ldv, const float* G, const float* kflag,
                    const float* qflag, int64_t B, int64_t Tq, int64_t Tk, int64_t H, int64_t dk,
                    const float* dout, int64_t lddo, float* dq, int64_t lddq, float* dk_, int64_t lddk,
                    float* dv, int64_t lddv);

/* bf16-storage variants (BASELINE cfg 3 / cfg 5 bf16 attention core): K / V and dK / dV are
 * bf16 (rows 8-B aligned, ld % 4 == 0), Q / dQ are bf16 if q_bf16 else fp32 (the decoder's
 * single query; mixed types need T_q = 1); O, dO, G and the flags stay fp32 and the softmax /
 * graph / L1 chain runs in fp32. T_q > 1 (q_bf16 = 1): bf16 MFMA strip kernels -- S = QK^T and
 * dP = dO V^T on bf16 operands (dO rounded to bf16), PV / P^T dO / dS^T Q / dS K with P and dS
 * rounded to bf16, fp32 accumulation. T_q = 1: the single-query kernels, fp32 products on the
 * bf16 values. T_k <= 128. */
int savqa_gattn_fwd_bf16(void* stream, int32_t q_bf16, const void* q, int64_t ldq, const void* k,
                         int64_t ldk, const void* v, int64_t ldv, const float* G,
                         const float* kflag, const float* qflag, int64_t B, int64_t Tq,
                         int64_t Tk, int64_t H, int64_t dk, float* o, int64_t ldo, float* att);
int savqa_gattn_bwd_bf16(void* stream, int32_t q_bf16, const void* q, int64_t ldq, const void* k,
                         int64_t ldk, const void* v, int64_t ldv, const float* G,
                         const float* kflag, const float* qflag, int64_t B, int64_t Tq,
                         int64_t Tk, int64_t H, int64_t dk, const float* dout, int64_t lddo,
                         void* dq, int64_t lddq, void* dk_, int64_t lddk, void* dv, int64_t lddv);

/* Key-tiled variant of the same operator for long sequences (any Tq, Tk; used for
 * Tk > 128: cfg 4's 449-token stacks, super-node relation graphs up to T = 1600).
 * Keys stream through LDS in tiles of 64 with per-row online statistics; nothing of
 * size Tq x Tk is materialised. stats: caller-owned [B*H*Tq][4] fp32 (m, Z, W, delta),
 * written by the forward (m, Z, W) and the backward (delta = sum_j n_ij dN_ij); keep it
 * from the forward to the backward. att (return_att) is not available on this path. */
int savqa_gattn_fwd_flash(void* stream, const float* q, int64_t ldq, const float* k, int64_t ldk,
                          const float* v, int64_t ldv, const float* G, const float* kflag,
                          const float* qflag, int64_t B, int64_t Tq, int64_t Tk, int64_t H,
                          int64_t dk, float* o, int64_t ldo, float* stats);

/* Backward of savqa_gattn_fwd_flash: delta (workgroup per query tile, one key sweep; writes
 * stats' Z, W, delta and parks a per-row fp64 term in dq, which must therefore not alias any
 * input), dQ (second key sweep), then dK/dV (workgroup per key tile); ReLU-masked like
 * savqa_gattn_bwd. */
int savqa_gattn_bwd_flash(void* stream, const float* q, int64_t ldq, const float* k, int64_t ldk,
                          const float* v, int64_t ldv, const float* G, const float* kflag,
                          const float* qflag, int64_t B, int64_t Tq, int64_t Tk, int64_t H,
                          int64_t dk, const float* dout, int64_t lddo, float* stats, float* dq, int64_t lddq, float* dk_, int64_t lddk,
                          float* dv, int64_t lddv);

/* The same two entry points with a caller-owned workspace (16-B aligned, at least
 * savqa_gattn_flash_ws_bytes(B, Tq, Tk, H, backward) bytes; contents not preserved): the
 * library first splits Q, K, V (and dO) of every (sample, head) into the x6 kernels' bf16 plane
 * tiles there, so the attention kernels stage tiles by DMA instead of splitting them in every
 * workgroup. Same results as without (bit-identical: the same splits meet the same MFMAs).
 * ws = NULL: the kernels split in place, as savqa_gattn_{fwd,bwd}_flash. */
int64_t savqa_gattn_flash_ws_bytes(int64_t B, int64_t Tq, int64_t Tk, int64_t H, int32_t backward);
int savqa_gattn_fwd_flash_ws(void* stream, const float* q, int64_t ldq, const float* k,
                             int64_t ldk, const float* v, int64_t ldv, const float* G,
                             const float* kflag, const float* qflag, int64_t B, int64_t Tq,
                             int64_t Tk, int64_t H, int64_t dk, float* o, int64_t ldo,
                             float* stats, void* ws, int64_t ws_bytes);
int savqa_gattn_bwd_flash_ws(void* stream, const float* q, int64_t ldq, const float* k,
                             int64_t ldk, const float* v, int64_t ldv, const float* G,
                             const float* kflag, const float* qflag, int64_t B, int64_t Tq,
                             int64_t Tk, int64_t H, int64_t dk, const float* dout, int64_t lddo,
                             float* stats, float* dq, int64_t lddq, float* dk_, int64_t lddk,
                             float* dv, int64_t lddv, void* ws, int64_t ws_bytes);

/* Single-query graph attention over long key sequences (T_q = 1: the decoder cross-attention
 * at T_k > 128, AttModel_x3.py:279 -> modules.py:236-311), split over keys so every wave takes
 * 64 keys of one (sample, head): same operator, layouts and ReLU-masked gradients as
 * savqa_gattn_fwd / _bwd with T_q = 1 (q / o / dout / dq rows are samples; G is (B, 1, Tk)).
 * stats: caller-owned [B*H*4] floats (16-B aligned) written by the forward (row max, softmax
 * denominator, graph-weighted mass) and read by the backward; ws: scratch of at least
 * savqa_gattn_q1s_ws_bytes(B, H, Tk) bytes, 16-B aligned (per-split partials, summed in a
 * fixed order: deterministic). */
int64_t savqa_gattn_q1s_ws_bytes(int64_t B, int64_t H, int64_t Tk);
int savqa_gattn_fwd_q1s(void* stream, const float* q, int64_t ldq, const float* k, int64_t ldk,
                        const float* v, int64_t ldv, const float* G, const float* kflag,
                        const float* qflag, int64_t B, int64_t Tk, int64_t H, int64_t dk, float* o,
                        int64_t ldo, float* stats, void* ws, int64_t ws_bytes);
int savqa_gattn_bwd_q1s(void* stream, const float* q, int64_t ldq, const float* k, int64_t ldk,
                        const float* v, int64_t ldv, const float* G, const float* kflag,
                        const float* qflag, int64_t B, int64_t Tk, int64_t H, int64_t dk,
                        const float* dout, int64_t lddo, const float* stats, float* dq,
                        int64_t lddq, float* dk_, int64_t lddk, float* dv, int64_t lddv, void* ws,
                        int64_t ws_bytes);

/* ------------------------------------------------------------------------
 * Graph construction, AttModel_x3.py:103-122 (vis, node_graph == NULL) and
 * :229-247 (syb): graph_diag, graph (== graph_cross, aliased in the reference),
 * dec_mask. Inputs int32 (B,Nn,Nn), (B,Lq,Lq), (B,Lq,Lq), optional (B,Nn,Nn).
 * ------------------------------------------------------------------------ */
int savqa_graph_build(void* stream, const int32_t* node_mask, const int32_t* q_mask,
                      const int32_t* q_graph, const int32_t* node_graph, int64_t B, int64_t Nn,
                      int64_t Lq, int32_t dec_mask_on, float* graph_diag, float* graph,
                      float* dec_mask);

/* dec0[b,:] = D(emb[idx,:]*scale + pos[0,:])   (AttModel_x3.py:141-147, :267-274,
 * modules.py:40-43); D = dec_dropout with keep mask savqa_dropout(site) when p > 0
 * (element index b*d + c), identity when p == 0 (eval / dropout_rate 0). */
int savqa_dec_init(void* stream, const float* emb, int64_t idx, float scale, const float* pos,
                   int64_t B, int64_t d, uint64_t seed, int32_t site, float p, float* out);

/* backward of savqa_dec_init: with g' = D'(g): demb[idx,:] += scale*sum_b g'[b,:];
 * dpos[0,:] += sum_b g'[b,:] */
int savqa_dec_init_bwd(void* stream, const float* g, int64_t B, int64_t d, int64_t idx, float scale,
                       uint64_t seed, int32_t site, float p, float* demb, float* dpos);

/* ------------------------------------------------------------------------
 * MIL-NCE relation branch (only_obj = False), AttModel_x3.py:382-437. Slot tables are
 * the loader's loc tensors (int64 [B][L][5] positives: obj_i, obj_j, rel_category,
 * macro_rel_loc, micro_rel_loc; [B][L][4] negatives; macro_rel_loc < 0 = padding).
 * obj = new_obj_fea [B*Nv][H]; R = MIL_NCE.R [nrel][H][H]; relf = relu(syb_mlp(syb_emb
 * (micro_positive_rel))) [B*Lp][H]; macro = new_macro_ipt [B*Ns][H].
 * ------------------------------------------------------------------------ */
/* val[slot] = obj[b,i] . V[b*Nv + j][r*H : r*H + H] for every listed entry (0 on padding),
 * where V = obj Rmat^T is computed by savqa_gemm (Rmat = R as [nrel*H][H]): x_i^T R_r x_j */
int savqa_rel_entries_fwd(void* stream, const int64_t* loc, int32_t loc_w, int64_t B, int64_t L,
                          const float* obj, int64_t Nv, int64_t H, const float* V, int64_t ldv,
                          float* val);
/* dobj[b,i] += dval V[(b,j)][rH:]; dV[(b,j)][rH:] += dval obj[b,i]  (atomics) */
int savqa_rel_entries_bwd(void* stream, const int64_t* loc, int32_t loc_w, int64_t B, int64_t L,
                          const float* obj, int64_t Nv, int64_t H, const float* V, int64_t ldv,
                          const float* dval, float* dobj, float* dV);
/* mil_rel = LSE(max(sp,eps)) - LSE(max(sp,eps) ++ max(sn,eps)) over valid entries (:405-406);
 * valid entries must be a prefix of each sample's slots (collate pads the tail); cum[b] =
 * valid positives of samples < b (int32 [B+1]); wsm[cum[b]+k] = softmax over the batch's
 * valid positives (:420); st (16 floats) = (P, m1, Z1, m2, Z2, err, mr, Zr, ...) for the
 * backward; err = 1 and mil_rel = NaN if the prefix layout is violated. Multi-workgroup with a
 * fixed-order fold of per-chunk records (deterministic): ws holds savqa_rel_loss_ws_bytes. */
int64_t savqa_rel_loss_ws_bytes(int64_t B, int64_t Lp, int64_t Ln);
int savqa_rel_loss_fwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp, const float* sp,
                       const int64_t* neg_loc, int64_t Ln, const float* sn, float eps, int32_t* cum,
                       float* wsm, float* st, float* mil_rel, void* ws, int64_t ws_bytes);
/* macro[b, loc3] = sum over the node's (consecutive) entries, in order, of
 * wsm[loc4] * relf[b, loc4]  (:418-436: zero, then the reference's accumulation loop) */
int savqa_rel_macro_fwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp, const float* st,
                        const float* wsm, const float* relf, int64_t Ns, int64_t H, float* macro);
/* backward of the update: dwsm[loc4] += dmacro[b,loc3].relf[b,loc4], drelf[b,loc4] +=
 * wsm[loc4] dmacro[b,loc3] (both zero-initialised by the caller), then dmacro rows loc3 := 0 */
int savqa_rel_macro_bwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp, const float* st,
                        const float* wsm, const float* relf, int64_t Ns, int64_t H, float* dmacro,
                        float* dwsm, float* drelf);
/* dsp / dsn per slot from dmil (device scalar) through both logsumexps and the softmax path
 * (ws: savqa_rel_loss_ws_bytes, as for the forward) */
int savqa_rel_loss_bwd(void* stream, const int64_t* pos_loc, int64_t B, int64_t Lp, const float* sp,
                       const int64_t* neg_loc, int64_t Ln, const float* sn, float eps,
                       const int32_t* cum, const float* wsm, const float* dwsm, float* st,
                       const float* dmil, float* dsp, float* dsn, void* ws, int64_t ws_bytes);

/* out = a*x + b*y over n floats (combining the MIL-NCE terms of the loss) */
int savqa_axpby(void* stream, const float* x, const float* y, int64_t n, float a, float b,
                float* out);

/* ------------------------------------------------------------------------
 * Dropout (nn.Dropout(dropout_rate) sites of model_v=3: stack inputs
 * AttModel_x3.py:71-72/:102 (vis: position-table dropout, then enc_dropout) and :227
 * (syb enc_dropout); decoder inputs :147/:274 (savqa_dec_init); heads :482-500).
 * Keep bit of element idx at dropout site `site` (>= 0) under step seed `seed`:
 *   z = seed + site*0xD1B54A32D192ED03 + (idx+1)*0x9E3779B97F4A7C15   (mod 2^64)
 *   z = (z ^ z>>30)*0xBF58476D1CE4E5B9; z = (z ^ z>>27)*0x94D049BB133111EB; z ^= z>>31
 *   keep = (uint32)(z>>32) >= floor(p*2^32);  kept values are scaled by 1/(1-p).
 * (torch's Philox stream is not reproducible outside torch; the backward regenerates
 * masks from (seed, site, idx), so none are stored.) p == 1 drops everything.
 * ------------------------------------------------------------------------ */
/* out[i] = in[i]*keep(i)*scale (in == out allowed); forward and backward of nn.Dropout */
int savqa_dropout(void* stream, const float* in, int64_t n, uint64_t seed, int32_t site, float p,
                  float* out);

/* out[b,t,c] = Dx(z[b,t,c] + Dp(pos[t,c])), idx = (b*T+t)*d + c; Dp = identity if
 * site_pos < 0 (syb stack), else the vis stack's position-table dropout (:71-72). */
int savqa_posadd_dropout(void* stream, const float* z, const float* pos, int64_t B, int64_t T,
                         int64_t d, uint64_t seed, int32_t site_pos, int32_t site_x, float p,
                         float* out);

/* backward: dz = Dx'(g) (dz == g allowed); dpos[t,c] += sum_b Dp'(dz[b,t,c]) */
int savqa_posadd_dropout_bwd(void* stream, const float* g, int64_t B, int64_t T, int64_t d,
                             uint64_t seed, int32_t site_pos, int32_t site_x, float p, float* dz,
                             float* dpos);

/* out[t][c] += sum_b X[(b*T+t)*ldx + c]: gradient of the learned position tables
 * (syb_positional_encoding, AttModel_x3.py:100-101, :225-226; padding_idx=-1 row untouched
 * as long as T < maxlen, which the loader guarantees). */
int savqa_period_sum_acc(void* stream, const float* X, int64_t B, int64_t T, int64_t C, int64_t ldx,
                         float* out);

/* dst rows: dst[(r/group)*stride + r%group + offset][:cols] = src[r][:cols]  (torch.cat) */
int savqa_copy_rows(void* stream, const float* src, int64_t rows, int64_t cols, int64_t lds,
                    float* dst, int64_t ldd, int64_t group, int64_t stride, int64_t offset);

/* ------------------------------------------------------------------------
 * MIL-NCE only_obj core, AttModel_x3.py:361-374:
 *   s+ = Pf.v, s- = Nf.v (per (b,n,k)); w = softmax_k(s+); obj[b,n] = sum_k w Pf
 *   term[b,n] = LSE_k(eps) - LSE_k(max(mask*s-, eps));  mil = sum term / (2*B*Nv)
 * Pf, Nf: (B*Nv*K, H) post-ReLU; v: (B*Nv, H) post-ReLU; mask int32 (B,Nv,K).
 * mil_out: device scalar. ws: (B*Nv) floats of workspace.
 * ------------------------------------------------------------------------ */
int savqa_mil_fwd(void* stream, const float* Pf, const float* Nf, const float* v,
                  const int32_t* mask, int64_t BN, int64_t K, int64_t H, float eps,
                  float* obj, float* ws, float* mil_out);
/* Backward: dobj (BN,H) (may be NULL), dmil (device scalar) -> dPf, dNf, dv (pre-ReLU). */
int savqa_mil_bwd(void* stream, const float* Pf, const float* Nf, const float* v,
                  const int32_t* mask, int64_t BN, int64_t K, int64_t H, float eps,
                  const float* dobj, const float* dmil, float* dPf, float* dNf, float* dv);
/* The same with bf16 dPf / dNf (the operands of the low-precision modes' embedding GEMMs). */
int savqa_mil_bwd_bf16(void* stream, const float* Pf, const float* Nf, const float* v,
                       const int32_t* mask, int64_t BN, int64_t K, int64_t H, float eps,
                       const float* dobj, const float* dmil, void* dPf, void* dNf, float* dv);

/* macro[b*Ns + loc[b,n]][:] = obj[b*Nv+n][:] for 0 <= loc < Ns (AttModel_x3.py:377-380),
 * and its backward dobj[b*Nv+n] = dmacro[b*Ns+loc] (dobj rows with loc outside [0, Ns)
 * zeroed). The reference raises IndexError on loc >= Ns; here such a location is never
 * dereferenced (no write, zero gradient) -- collate.pack rejects it on the host. */
int savqa_index_put_rows(void* stream, const int64_t* loc, int64_t B, int64_t Nv, int64_t Ns,
                         int64_t H, const float* obj, float* macro);
int savqa_index_get_rows(void* stream, const int64_t* loc, int64_t B, int64_t Nv, int64_t Ns,
                         int64_t H, const float* dmacro, float* dobj);

/* Deterministic embedding-table gradient (the backward of nn.Embedding's row gather,
 * modules.py:32-46 / AttModel_x3.py:96-99, :352-360 -- torch accumulates it with index_add):
 * table[sid[j]][:cols] += sum of T[perm[k]][:cols] over the run of positions k with
 * sid[k] == sid[j], added in run order. sid: the R row ids sorted ascending, perm: the stable
 * sort's permutation (equal ids keep their row order), so the sum has ONE order whatever the
 * schedule: run-to-run bit-identical, unlike an atomic scatter. T: the dense rows dY W of
 * the GEMM that used to scatter. cols, ldt, ldtab multiples of 4; T, table 16-B aligned. */
int savqa_segment_add_rows(void* stream, const float* T, int64_t ldt, const int64_t* perm,
                           const int64_t* sid, int64_t R, int64_t cols, float* table,
                           int64_t ldtab);

/* ------------------------------------------------------------------------
 * Loss, main_itp_ddp_tar_super_node.py:335-361 + label_smoothing modules.py:461-463:
 *   lsm = (lsm(vis)+lsm(syb)+lsm(concat))/3; y = (1-eps)*onehot + eps/C
 *   loss = mean_b(-sum_c y*lsm) - (with_mil ? mil : 0)
 * Also writes dlogits (3,B,C) = d loss / d logits (order concat, vis, syb), and
 * lsm (B,C) if non-NULL. loss: device scalar. ws: B floats.
 * ------------------------------------------------------------------------ */
int savqa_loss_fwd(void* stream, const float* lc, const float* lv, const float* ls,
                   const int64_t* answer, int64_t B, int64_t C, float eps, const float* mil,
                   int32_t with_mil, float* loss, float* dlogits, float* lsm, float* ws);

/* out[r][c] = in[r][c] * rowscale[r] * (mask[r][c] > 0)   (either optional): ReLU backward of
 * the decoder self-attention value path, LN(qm * relu(V_proj(x)) + x) (modules.py:187-205) */
int savqa_rowscale_mask(void* stream, const float* in, const float* rowscale, const float* mask,
                        int64_t rows, int64_t cols, float* out);

/* out = a*in + b   (label_smoothing.forward, modules.py:461-463) */
int savqa_affine(void* stream, const float* in, int64_t n, float a, float b, float* out);

/* embedding.forward (modules.py:40-43): out[r] = table[idx[r]] * scale; and its backward
 * dtable[idx[r]] += g[r] * scale for idx[r] != padding_idx (pass -1 for none... the
 * reference's padding_idx=-1 means the LAST row: the caller passes vocab-1). */
int savqa_gather_rows(void* stream, const float* table, const int64_t* idx, int64_t rows,
                      int64_t cols, float scale, float* out);
int savqa_scatter_rows(void* stream, const float* g, const int64_t* idx, int64_t rows,
                       int64_t cols, float scale, int64_t padding_idx, float* dtable);

/* out[i] = in[i] * (*scale)  (chain rule with a device-side upstream gradient) */
int savqa_scale_by(void* stream, const float* in, const float* scale, int64_t n, float* out);

/* ------------------------------------------------------------------------
 * Adam (torch.optim.Adam semantics, main:206/:366) over one flat fp32 range:
 *   g' = g*grad_scale; m = b1 m + (1-b1) g'; v = b2 v + (1-b2) g'^2
 *   p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
 * ------------------------------------------------------------------------ */
int savqa_adam(void* stream, float* p, const float* g, float* m, float* v, int64_t n,
               float lr, float beta1, float beta2, float eps, float bc1, float bc2,
               float grad_scale);
/* The same update, also writing the updated p rounded to bf16 (round to nearest even) into
 * shadow[0, n) (8-B aligned): the bf16 weight image of the low-precision modes, refreshed in
 * the optimizer's pass instead of a cast that re-reads p. shadow may be NULL (= savqa_adam). */
int savqa_adam_shadow(void* stream, float* p, const float* g, float* m, float* v, int64_t n,
                      float lr, float beta1, float beta2, float eps, float bc1, float bc2,
                      float grad_scale, void* shadow);

/* Row-tracked tables (the three 407000 x 300 GloVe tables, AttModel_x3.py:36-41, :168-171,
 * :295): flags[r] bit 0 = row r has Adam state (touched at some step), bit 1 = row
 * r was touched since the last savqa_zero_rows (its gradient may be non-zero).
 *   savqa_mark_rows: flags[ids[i]] |= 2 (ids outside [0, nrows) ignored)
 *   savqa_zero_rows: g row r = 0 and bit 1 cleared, for every row with bit 1
 *   savqa_adam_rows: the savqa_adam update on every row with bit 0 or 1 (g read only with
 *     bit 1, else 0), then bit 0 set on rows with bit 1. Rows with neither bit are exactly
 *     what torch.optim.Adam would leave unchanged (m = v = 0, g = 0): skipping them is exact. */
int savqa_mark_rows(void* stream, const int64_t* ids, int64_t n, int64_t nrows, uint8_t* flags);
int savqa_zero_rows(void* stream, float* g, int64_t width, int64_t nrows, uint8_t* flags);
int savqa_adam_rows(void* stream, float* p, const float* g, float* m, float* v, int64_t width,
                    int64_t nrows, uint8_t* flags, float lr, float beta1, float beta2, float eps,
                    float bc1, float bc2, float grad_scale);

/* ------------------------------------------------------------------------
 * Batch collation. Replaces the host-side padding of
 * collate_fn (models/data_loader_itp_bbox_super_node_onlyobj.py:341-445;
 * dataloader/data_loader_itp_bbox_super_node.py:366-497): the host packs each
 * field's per-sample arrays back to back with per-sample row offsets off[B+1]
 * (n_b = off[b+1] - off[b]); one launch expands every field into its dense
 * [B][T][row_elems] tensor:
 *   ROWS : dst[b][t][:] = t < n_b ? src row (off[b] + t) : fill  (elem_bytes 4|8;
 *          fill = the element's bit pattern: PAD, LOC_PAD, 0)
 *   BOX  : int32 dst[b][t][c] = t < n_b && (!square || c < n_b)   (the masks)
 *   FILL : dst = fill                                              (graphs, before edges)
 * `fields` is a HOST array (copied into the kernel arguments); every pointer inside
 * it is a device pointer. savqa_collate_edges then sets graph[b][i][j] = 1 for
 * every (i, j) of sample b (edges int32 [E][2], already in [0, T); edge_off[B+1]).
 * ------------------------------------------------------------------------ */
#define SAVQA_COLLATE_MAX_FIELDS 24
#define SAVQA_COLLATE_ROWS 0
#define SAVQA_COLLATE_BOX 1
#define SAVQA_COLLATE_FILL 2
typedef struct savqa_collate_field {
  int32_t kind;
  int32_t elem_bytes;
  int32_t square;
  int32_t reserved;
  int64_t T;
  int64_t row_elems;
  uint64_t fill;
  const void* src;
  const int64_t* off;
  void* dst;
} savqa_collate_field;
int savqa_collate(void* stream, const savqa_collate_field* fields, int32_t nfields, int64_t B);
int savqa_collate_edges(void* stream, const int32_t* edges, const int64_t* edge_off, int64_t B,
                        int64_t E, int64_t T, int32_t* graph);

#ifdef __cplusplus
}
#endif
#endif /* SAVQA_H */
