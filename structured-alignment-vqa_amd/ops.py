"""Thin Python wrappers over the libsavqa C ABI (include/savqa.h).

Every function takes torch tensors that already live on the current HIP device and
enqueues work on torch's current stream. Nothing here computes with torch ops:
torch provides device memory and the stream only. There is no CPU fallback -- a
missing library or a CPU tensor raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import torch

from . import _lib
from ._lib import GemmDesc, call

Tensor = torch.Tensor


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: Optional[Tensor]):
    if t is None:
        return None
    if not t.is_cuda:
        raise _lib.SavqaError("savqa ops need device tensors (got a CPU tensor)")
    return t.data_ptr()


def _f32(t: Optional[Tensor], name: str):
    if t is not None and t.dtype != torch.float32:
        raise _lib.SavqaError(f"{name}: expected float32, got {t.dtype}")


# ------------------------------------------------------------------------------ GEMM
class GemmProbe:
    """Optional per-launch timing of savqa_gemm with HIP events on the launch stream
    (bench.py's roofline measurement). Off unless a probe is installed."""

    def __init__(self, detail: bool = False, keep: bool = False):
        self.records = []  # (variant, flops, start_event, end_event)
        self.detail = detail  # key launches by shape + fused options too (breakdowns)
        # keep: also a copy of every launch's descriptor, aligned with records, as
        # ("gemm" | "lp", desc) -- tools/gemm_replay.py re-issues them on their own buffers
        self.keep = keep
        self.descs = []

    @staticmethod
    def shape_key(d):
        lay = ("T" if d.a_trans else "N") + ("T" if d.b_trans else "N")
        opts = "".join(c for c, on in (("g", d.a_rows or d.b_rows), ("s", d.c_rows),
                                        ("b", d.bias), ("p", d.rowvec), ("r", d.resid),
                                        ("m", d.mask), ("R", d.relu), ("a", d.atomic),
                                        ("c", d.colsum_a)) if on)
        return f"{lay} {d.M}x{d.N}x{d.K} {opts}"

    @staticmethod
    def variant(d):
        plan = (C.c_int32 * 4)()
        call("savqa_gemm_plan", C.byref(d), C.cast(plan, C.c_void_p))
        lay = f"{str(bool(d.a_trans)).lower()},{str(bool(d.b_trans)).lower()}"
        if plan[0] == 32:
            kg = (d.a_trans and d.a_rows) or (not d.b_trans and d.b_rows)
            if d.prec == 1 and not kg:
                return f"gemm_skinny_bf_kernel<{lay}>"
            return f"gemm_skinny_kernel<{lay}>"
        if plan[0] == 16:
            return f"gemm_skinny16_kernel<{lay}>"
        if d.prec in (1, 5, 6):  # (savqa_gemm's fallback: operands that are not 16-B vectors)
            al = all(p % 16 == 0 and ld % 4 == 0 for p, ld in ((d.A, d.lda), (d.B, d.ldb)))
            if al:  # third argument: hi / lo accumulators (prec 5: the two-level form);
                # fourth: B from the pre-split weight planes (the conditions savqa_gemm applies)
                bp = bool(d.b_planes) and plan[0] == 128 and not d.a_trans and \
                    not d.b_rows and d.b_planes % 16 == 0
                return (f"gemm_x6_kernel<{lay},{str(d.prec != 5).lower()},"
                        f"{str(bp).lower()}>")
            return f"gemm_f32_kernel<{plan[0]},{plan[0]},{lay}>"
        if d.prec:
            return f"gemm_bf16_kernel<{lay},{d.prec}>"
        return f"gemm_f32_kernel<{plan[0]},{plan[0]},{lay}>"

    def summary(self):
        torch.cuda.synchronize()
        agg = {}
        for var, fl, e0, e1 in self.records:
            ms = e0.elapsed_time(e1)
            a = agg.setdefault(var, [0, 0.0, 0.0])
            a[0] += 1
            a[1] += fl
            a[2] += ms
        return agg


_probe = None

# Product precision of the fp32-storage 128x128-tile GEMMs (savqa_gemm_desc.prec): 0 = fp32
# MFMA (exact fp32, the ops-level default), 3 = 3xbf16 split products (~2^-16), 6 = fp32 from
# exact three-term bf16 splits, six products per pair (gemm_x6.hip; the engine's fp32 mode). Set per model (AttModel(...,
# gemm_precision="bf16x3")) via gemm_precision(); the bf16 / fp8 modes use gemm_lp instead.
# "bf16sk" (1): the low-precision modes' fp32-storage GEMMs -- bf16 products on the skinny
# (M = B row) launches (gemm_skinny_bf_kernel: operands rounded to bf16 as autocast rounds a
# Linear's), x6 on the 128x128 ones
PREC = {"fp32": 0, "fp32_native": 0, "bf16x3": 3, "fp32x6": 6, "bf16sk": 1}
# prec 5: x6 in its two-level form (gemm_x6.hip: VALU adds of each k-tile's partial, no hi / lo
# accumulators), for launches whose outputs feed a rounding-sensitive chain (x6_two_level)
X6_TWO_LEVEL = 5


def x6_two_level() -> int:
    """The precision to pass a launch that wants x6's two-level accumulation: 5 when the
    current mode is x6, the current mode otherwise."""
    return X6_TWO_LEVEL if _prec == 6 else _prec
# fp32 / x6 K splits (split-K weight gradients, tail splits) through partial slabs summed in a
# fixed order (savqa_gemm_desc.ws) instead of fp32 atomics: run-to-run deterministic
# ("dw": split-K weight gradients only, the tail splits keep their atomics)
GEMM_SLABS = {"0": False, "dw": "dw"}.get(os.environ.get("SAVQA_GEMM_SLABS", "1"), True)
_prec = 0
class gemm_precision:
    """Context manager: GEMMs launched inside use the given product precision."""

    def __init__(self, name: str):
        if name not in PREC:
            raise ValueError(f"gemm precision must be one of {sorted(PREC)}")
        self.p = PREC[name]

    def __enter__(self):
        global _prec
        self.old, _prec = _prec, self.p
        return self

    def __exit__(self, *exc):
        global _prec
        _prec = self.old
        return False


# Optional per-launch timing of the HBM-bound kernels (LayerNorm, Adam, graph attention) with
# HIP events on the launch stream, keyed by kernel family, with each launch's ALGORITHMIC bytes
# and FLOPs (bench.py's "hbm_kernels" report). Off unless a recorder list is installed.
_kprobe = None


def set_kernel_probe(probe):
    global _kprobe
    _kprobe = probe


def _kcall(tag: str, nbytes: float, flops: float, name: str, *args):
    if _kprobe is None:
        call(name, *args)
        return
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    call(name, *args)
    e1.record()
    _kprobe.append((tag, float(nbytes), float(flops), e0, e1))


def _attn_bytes(q, B, Tq, Tk, H, dk, n_in, n_out):
    """Algorithmic bytes of one graph-attention launch: n_in (Tq or Tk) x dk operands per
    (sample, head) read, n_out written, the fp32 (B, Tq, Tk) graph read ONCE per sample."""
    es = q.element_size()
    rows = B * H * dk * es
    return rows * (n_in + n_out) + B * Tq * Tk * 4


# Pre-split x6 planes of GEMM weights (savqa_x6_weight_planes): a weight's B operand split
# into the x6 kernel's three bf16 plane images once per optimizer step instead of by every
# 128x128 tile that reads it (savqa_gemm_desc.b_planes; bit-identical results). The engine
# points WP_CACHE at its own cache (the images die with the model) and sets WP_KEY to the
# parameter arena's state key at every forward, then refresh_weight_planes() rebuilds every
# image made under another key in one batched launch on the current stream; an image seen for
# the first time is built at its first use, on the stream of that use.
X6_PLANES = os.environ.get("SAVQA_X6_PLANES", "1") != "0"
WP_BATCH = os.environ.get("SAVQA_WP_BATCH", "1") != "0"   # 0: rebuild each image at its use
WP_KEY = None
WP_CACHE = {}   # (W ptr, b_trans, N, K, ldb, device) -> [image, key it was built under]


def weight_planes(W: Tensor, b_trans: bool, N: int, K: int, ldb: int) -> Tensor:
    key = (W.data_ptr(), bool(b_trans), int(N), int(K), int(ldb), W.device)
    e = WP_CACHE.get(key)
    if e is not None and e[1] == WP_KEY:
        return e[0]
    buf = e[0] if e is not None else torch.empty(
        int(_lib.load().savqa_x6_weight_planes_bytes(int(N), int(K))), dtype=torch.uint8,
        device=W.device)
    call("savqa_x6_weight_planes", _stream(), _p(W), int(ldb), int(bool(b_trans)), int(N),
         int(K), _p(buf))
    WP_CACHE[key] = [buf, WP_KEY]
    return buf


def refresh_weight_planes() -> int:
    """Rebuild every WP_CACHE image made under another WP_KEY (one savqa_x6_weight_planes_batch
    call on the current stream); returns the number rebuilt."""
    stale = [(k, e) for k, e in WP_CACHE.items() if e[1] != WP_KEY]
    if not stale:
        return 0
    jobs = (_lib.PlanesJob * len(stale))()
    for i, ((ptr, bt, N, K, ldb, _dev), e) in enumerate(stale):
        jobs[i].B, jobs[i].ldb, jobs[i].b_trans = ptr, ldb, int(bt)
        jobs[i].N, jobs[i].K, jobs[i].out = N, K, _p(e[0])
    call("savqa_x6_weight_planes_batch", _stream(), C.cast(jobs, C.c_void_p), len(stale))
    for _, e in stale:
        e[1] = WP_KEY
    return len(stale)


def set_gemm_probe(probe):
    global _probe
    _probe = probe


def gemm(A: Tensor, B: Tensor, Cm: Tensor, M: int, N: int, K: int, *, lda: int, ldb: int,
         ldc: int, a_trans=False, b_trans=False, a_rows=None, b_rows=None, c_rows=None,
         c_group=0, c_stride=0, c_offset=0, bias=None, rowvec=None, ldrv=0, rowvec_period=0,
         resid=None, ldr=0, mask=None, ldmask=0, mask_arows=False, rowscale=None, relu=False,
         alpha=1.0, beta=0.0, atomic=False, split_k=1, colsum_a=None, prec=None,
         plan_only=False, b_planes=False):
    """Generic MFMA GEMM with fused epilogue (see savqa_gemm in include/savqa.h).
    plan_only: no launch, return savqa_gemm_plan's [tile, split, tail slices, workgroups]."""
    d = GemmDesc()
    d.prec = _prec if prec is None else int(prec)
    d.M, d.N, d.K = int(M), int(N), int(K)
    d.A, d.lda, d.a_trans = _p(A), int(lda), int(bool(a_trans))
    d.a_rows = _p(a_rows)
    d.B, d.ldb, d.b_trans = _p(B), int(ldb), int(bool(b_trans))
    d.b_rows = _p(b_rows)
    d.C, d.ldc = _p(Cm), int(ldc)
    d.c_group, d.c_stride, d.c_offset = int(c_group), int(c_stride), int(c_offset)
    d.c_rows = _p(c_rows)
    d.bias = _p(bias)
    d.rowvec, d.ldrv, d.rowvec_period = _p(rowvec), int(ldrv), int(rowvec_period)
    d.resid, d.ldr = _p(resid), int(ldr)
    d.mask, d.ldmask, d.mask_arows = _p(mask), int(ldmask), int(bool(mask_arows))
    d.rowscale = _p(rowscale)
    d.alpha, d.beta = float(alpha), float(beta)
    d.relu, d.atomic, d.split_k = int(bool(relu)), int(bool(atomic)), int(split_k)
    d.colsum_a = _p(colsum_a)
    if b_planes and X6_PLANES and d.prec in (5, 6) and not a_trans and b_rows is None:
        d.b_planes = _p(weight_planes(B, b_trans, N, K, ldb))
    if plan_only:
        plan = (C.c_int32 * 4)()
        call("savqa_gemm_plan", C.byref(d), C.cast(plan, C.c_void_p))
        return list(plan)
    if GEMM_SLABS and d.prec != 3 and not (relu or beta != 0.0 or c_rows is not None) and \
            (atomic or GEMM_SLABS is True):
        need = int(_lib.load().savqa_gemm_ws_elems(C.byref(d)))
        if need > 0:
            ws = _workspace(need, Cm.device)
            d.ws, d.ws_elems = _p(ws), int(ws.numel())
    if _probe is None:
        call("savqa_gemm", _stream(), C.byref(d))
        return
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    call("savqa_gemm", _stream(), C.byref(d))
    e1.record()
    key = GemmProbe.variant(d)
    if _probe.detail:
        key += " | " + GemmProbe.shape_key(d)
    _probe.records.append((key, 2.0 * M * N * K, e0, e1))
    if _probe.keep:
        _probe.descs.append(("gemm", GemmDesc.from_buffer_copy(d)))


# ------------------------------------------------------------------------------ low precision
DT = {torch.float32: 0, torch.bfloat16: 1, torch.float8_e4m3fn: 2, torch.uint8: 3}  # uint8: bits


def lp_desc(A: Tensor, B: Tensor, M: int, N: int, K: int, *, lda: int, ldb: int, a_trans=False,
            b_trans=False, a_rows=None, a_scale=None, lds_a=0, b_scale=None, lds_b=0, C=None,
            ldc=0, Cb=None, ldcb=0, c_group=0, c_stride=0, c_offset=0, bias=None, rowvec=None,
            ldrv=0, rowvec_period=0, resid=None, ldr=0, mask=None, ldmask=0, mask_arows=False,
            alpha=1.0, relu=False, atomic=False, split_k=1, tile_hint=0, c_rows=None,
            n_store=0, ws=None, colsum_a=None, bits_out=None, ldbits=0):
    """savqa_gemm_lp_desc for bf16 / fp8 operands (include/savqa.h). ws: split-K partial-slab
    workspace (fp32 tensor), see lp_workspace."""
    d = _lib.GemmLpDesc()
    d.M, d.N, d.K = int(M), int(N), int(K)
    d.A, d.lda, d.a_trans, d.a_type = _p(A), int(lda), int(bool(a_trans)), DT[A.dtype]
    d.a_rows, d.a_scale, d.lds_a = _p(a_rows), _p(a_scale), int(lds_a)
    d.B, d.ldb, d.b_trans, d.b_type = _p(B), int(ldb), int(bool(b_trans)), DT[B.dtype]
    d.b_scale, d.lds_b = _p(b_scale), int(lds_b)
    d.C, d.ldc, d.Cb, d.ldcb = _p(C), int(ldc), _p(Cb), int(ldcb)
    d.c_group, d.c_stride, d.c_offset = int(c_group), int(c_stride), int(c_offset)
    d.bias, d.rowvec, d.ldrv, d.rowvec_period = _p(bias), _p(rowvec), int(ldrv), int(rowvec_period)
    d.resid, d.ldr = _p(resid), int(ldr)
    d.mask, d.ldmask, d.mask_arows = _p(mask), int(ldmask), int(bool(mask_arows))
    d.mask_type = DT[mask.dtype] if mask is not None else 0
    d.alpha = float(alpha)
    d.relu, d.atomic, d.split_k = int(bool(relu)), int(bool(atomic)), int(split_k)
    d.tile_hint = int(tile_hint)
    d.c_rows, d.n_store = _p(c_rows), int(n_store)
    if ws is not None:
        d.ws, d.ws_elems = _p(ws), int(ws.numel())
    d.colsum_a = _p(colsum_a)
    d.bits_out, d.ldbits = _p(bits_out), int(ldbits)
    return d


_ws = {}
LP_SLABS = os.environ.get("SAVQA_LP_SLABS", "1") != "0"  # cfg 3: 17.86k -> 18.32k QA-samples/s
LP_TAIL_SLABS = os.environ.get("SAVQA_LP_TAIL_SLABS", "1") != "0"


def _workspace(need: int, dev) -> Tensor:
    """The split-K slab workspace of the current (device, stream), grown to `need` fp32
    elements: GEMMs on one stream run in order, so one buffer serves all of them."""
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), _stream())
    ws = _ws.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.float32, device=dev)
        _ws[key] = ws
    return ws


def lp_workspace(d, dev) -> Optional[Tensor]:
    """The partial-slab workspace a savqa_gemm_lp launch of d can use (split-K: slices x M x N
    fp32; a split-off last round of tiles: tail slices x rows x N), None when it uses none."""
    need = int(_lib.load().savqa_gemm_lp_ws_elems(C.byref(d)))
    return _workspace(need, dev) if need > 0 else None


def lp_variant(d) -> str:
    """Kernel instantiation savqa_gemm_lp launches for d (the name rocprof reports, up to
    the template arguments that follow from the variant)."""
    plan = (C.c_int32 * 4)()
    call("savqa_gemm_lp_plan", C.byref(d), C.cast(plan, C.c_void_p))
    at, bt = str(bool(d.a_trans)).lower(), str(bool(d.b_trans)).lower()
    if plan[0] == 3:
        return f"gemm_lp2_kernel<256,256,2,64,2,{at},{bt}>"
    if plan[0] == 4:
        return f"gemm_lp2_kernel<256,128,4,64,3,{at},{bt}>"
    if plan[0] == 5:
        return f"gemm_lp3_kernel<{at},{bt}>"
    return f"gemm_lp_kernel<{at},{bt},{str(d.a_type == 2).lower()},{plan[3]}>"


def lp_supported(d) -> bool:
    return bool(_lib.load().savqa_gemm_lp_supported(C.byref(d)))


def gemm_lp(*args, slabs=False, **kw):
    """Low-precision-operand MFMA GEMM (savqa_gemm_lp): same arguments as lp_desc; slabs: give a
    split-K launch its partial-slab workspace (no fp32 atomics). A long-K launch into fp32 C
    whose last round of tiles is split over K gets its tail workspace unless
    SAVQA_LP_TAIL_SLABS=0 (those slices then add atomically into a zero-filled C)."""
    d = lp_desc(*args, **kw)
    if LP_SLABS and (slabs or (not d.atomic and LP_TAIL_SLABS)):
        ws = lp_workspace(d, args[0].device)
        if ws is not None:
            d.ws, d.ws_elems = _p(ws), int(ws.numel())
    if _probe is None:
        call("savqa_gemm_lp", _stream(), C.byref(d))
        return
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    call("savqa_gemm_lp", _stream(), C.byref(d))
    e1.record()
    key = lp_variant(d)
    if _probe.detail:
        plan = (C.c_int32 * 4)()
        call("savqa_gemm_lp_plan", C.byref(d), C.cast(plan, C.c_void_p))
        key += (f" | {'T' if d.a_trans else 'N'}{'T' if d.b_trans else 'N'} {d.M}x{d.N}x{d.K}"
                f" split{plan[1]} wg{plan[2]}")
    _probe.records.append((key, 2.0 * d.M * d.N * d.K, e0, e1))
    if _probe.keep:
        _probe.descs.append(("lp", _lib.GemmLpDesc.from_buffer_copy(d)))


def cast_bf16(x: Tensor, rows: int, cols: int, ldi: int, out: Tensor, ldo: int, group=0,
              stride=0, offset=0):
    call("savqa_cast_bf16", _stream(), _p(x), int(rows), int(cols), int(ldi), _p(out), int(ldo),
         int(group), int(stride), int(offset))


def widen_bf16(x: Tensor, rows: int, cols: int, ldi: int, out: Tensor, ldo: int):
    """out = float(x) over bf16 rows (savqa_widen_bf16)."""
    call("savqa_widen_bf16", _stream(), _p(x), int(rows), int(cols), int(ldi), _p(out), int(ldo))


def quant_fp8(x: Tensor, rows: int, cols: int, ldi: int, q: Tensor, ldq: int, scale: Tensor,
              lds: int, group=0, stride=0, offset=0):
    call("savqa_quant_fp8", _stream(), _p(x), int(rows), int(cols), int(ldi), _p(q), int(ldq),
         _p(scale), int(lds), int(group), int(stride), int(offset))


def dequant_fp8_bf16(q: Tensor, rows: int, cols: int, ldq: int, scale: Tensor, lds: int,
                     out: Tensor, ldo: int):
    call("savqa_dequant_fp8_bf16", _stream(), _p(q), int(rows), int(cols), int(ldq), _p(scale),
         int(lds), _p(out), int(ldo))


def gather_rows_bf16(table: Tensor, ids: Tensor, cols: int, out: Tensor):
    """out[r, :cols] = bf16(table[ids[r], :cols]); out[r, cols:] = 0 (savqa_gather_rows_bf16)."""
    n = ids.numel()
    call("savqa_gather_rows_bf16", _stream(), _p(table), int(table.stride(0)), _p(ids), int(n),
         int(cols), _p(out), int(out.stride(0)))


def colsum_bf16(X: Tensor, rows: int, cols: int, ldx: int, out: Tensor):
    call("savqa_colsum_bf16", _stream(), _p(X), int(rows), int(cols), int(ldx), _p(out))


def linear_lp(X: Tensor, W: Tensor, b: Optional[Tensor], out: Optional[Tensor] = None,
              outb: Optional[Tensor] = None, *, relu=False, rows: Optional[int] = None,
              a_rows=None, rowvec=None, rowvec_period=0, resid=None, c_group=0, c_stride=0,
              c_offset=0, ldo=None, x_scale=None, w_scale=None, bits_out=None):
    """nn.Linear forward on low-precision operands: X [M][K] and W [N][K] both bf16, or both
    fp8-e4m3 with e8m0 block scales x_scale [M][K/32] / w_scale [N][K/32]; fp32 `out` and/or
    bf16 `outb` (same row map). bits_out (uint8 [M][N/8], bf16-only output): the output's
    (> 0) bits, the ReLU gate a later linear_dx_lp reads as its mask."""
    N, K = W.shape
    M = rows if rows is not None else (a_rows.numel() if a_rows is not None else X.numel() // K)
    ld = ldo if ldo is not None else N
    gemm_lp(X, W, M, N, K, lda=K, ldb=K, b_trans=True, a_rows=a_rows, a_scale=x_scale,
            lds_a=K // 32, b_scale=w_scale, lds_b=K // 32, C=out, ldc=ld, Cb=outb, ldcb=ld,
            c_group=c_group, c_stride=c_stride, c_offset=c_offset, bias=b, rowvec=rowvec, ldrv=N,
            rowvec_period=rowvec_period, resid=resid, ldr=N, relu=relu, bits_out=bits_out,
            ldbits=(bits_out.shape[-1] if bits_out is not None else 0))


def linear_dx_lp(dY: Tensor, W: Tensor, dX: Optional[Tensor] = None,
                 dXb: Optional[Tensor] = None, *, rows: int, a_rows=None, mask=None, ldmask=0,
                 mask_arows=False, resid=None):
    """dX = dY W on bf16 operands (W the bf16 shadow [N][K]); mask: the ReLU gate, bf16 values
    or a uint8 bit image (linear_lp's bits_out; ldmask in bytes)."""
    N, K = W.shape
    gemm_lp(dY, W, rows, K, N, lda=N, ldb=K, a_rows=a_rows, C=dX, ldc=K, Cb=dXb, ldcb=K,
            mask=mask, ldmask=ldmask, mask_arows=mask_arows, resid=resid, ldr=K)


def linear_dw_lp(dY: Tensor, X: Tensor, dW: Tensor, db: Optional[Tensor], *, rows: int):
    """dW += dY^T X on bf16 operands (split-K through slabs); db += colsum(dY), summed in fp32
    from the bf16 dY tiles the GEMM stages (savqa_gemm_lp_desc.colsum_a) -- the bf16 operand,
    as autocast's bias gradient is."""
    N, K = dW.shape
    gemm_lp(dY, X, N, K, rows, lda=N, ldb=K, a_trans=True, C=dW, ldc=K, atomic=True, split_k=-1,
            slabs=True, colsum_a=db)


def linear(X: Tensor, W: Tensor, b: Optional[Tensor], out: Tensor, *, relu=False,
           rows: Optional[int] = None, a_rows=None, rowvec=None, rowvec_period=0, resid=None,
           c_group=0, c_stride=0, c_offset=0, ldx=None, ldo=None, rowscale=None, prec=None,
           wp=False):
    """out = act(X W^T + b [+ rowvec]) [+ resid]  -- nn.Linear forward (W is [out, in])."""
    N, K = W.shape
    M = rows if rows is not None else (a_rows.numel() if a_rows is not None else X.numel() // K)
    gemm(X, W, out, M, N, K, lda=ldx if ldx is not None else K, ldb=K,
         ldc=ldo if ldo is not None else N, b_trans=True, a_rows=a_rows, bias=b, rowvec=rowvec,
         ldrv=N, rowvec_period=rowvec_period, resid=resid, ldr=N, relu=relu, c_group=c_group,
         c_stride=c_stride, c_offset=c_offset, rowscale=rowscale, prec=prec, b_planes=wp)


def linear_dx(dY: Tensor, W: Tensor, dX: Tensor, *, rows: int, a_rows=None, mask=None,
              ldmask=0, mask_arows=False, resid=None, ldr=None, c_rows=None, atomic=False,
              beta=0.0, lddy=None, lddx=None, wp=False):
    """dX = dY W  (mask: ReLU-backward gate of the producer of X; c_rows: scatter-add;
    wp: W's pre-split x6 planes, see weight_planes)."""
    N, K = W.shape  # dY has N cols, dX has K cols
    # a pure scatter-add (the GloVe-table gradient: few output tiles, K = 2048) may split K
    # across workgroups: every slice adds its partial with the same atomics
    split = -1 if (atomic and mask is None and resid is None and beta == 0.0) else 1
    gemm(dY, W, dX, rows, K, N, lda=lddy if lddy is not None else N, ldb=K,
         ldc=lddx if lddx is not None else K, a_rows=a_rows, mask=mask, ldmask=ldmask,
         mask_arows=mask_arows, resid=resid, ldr=ldr if ldr is not None else K, c_rows=c_rows,
         atomic=atomic, beta=beta, split_k=split, b_planes=wp)


def linear_dw(dY: Tensor, X: Tensor, dW: Tensor, db: Optional[Tensor], *, rows: int,
              x_rows=None, lddy=None, ldx=None):
    """dW += dY^T X ; db += colsum(dY)   (accumulating into the grad arena; the bias
    gradient is summed by the same GEMM from its staged dY^T tiles)."""
    N, K = dW.shape
    gemm(dY, X, dW, N, K, rows, lda=lddy if lddy is not None else N,
         ldb=ldx if ldx is not None else K, ldc=K, a_trans=True, b_rows=x_rows, atomic=True,
         split_k=-1, colsum_a=db)  # library picks the split-K factor


def colsum_acc(X: Tensor, rows: int, cols: int, ldx: int, out: Tensor):
    call("savqa_colsum_acc", _stream(), _p(X), int(rows), int(cols), int(ldx), _p(out))


# ------------------------------------------------------------------------------ LN
def ln_fwd(x: Tensor, gamma: Tensor, beta: Tensor, y: Tensor, mean: Tensor, rden: Tensor,
           std: Tensor, *, r=None, z_out=None, flag=None, xscale=None, eps=1e-8, yb=None):
    """yb: optional bf16 copy of y (operand of the next low-precision GEMM)."""
    cols = gamma.numel()
    rows = x.numel() // cols
    nb = rows * cols * (4 * (2 + (r is not None) + (z_out is not None)) + 2 * (yb is not None)) \
        + rows * 12
    _kcall("ln_fwd", nb, 0, "savqa_ln_fwd", _stream(), _p(x), _p(xscale), _p(r), rows, cols,
           _p(gamma), _p(beta), float(eps), _p(z_out), _p(y), _p(mean), _p(rden), _p(std),
           _p(flag), _p(yb))


_ln_ws = {}


def ln_workspace(cols: int, dev) -> Tensor:
    """The caller-owned workspace of savqa_ln_bwd for the current stream: 512 x 2 x cols
    floats of per-block gamma / beta partial rows, written with plain stores and summed in
    block order by the library (no initial contents needed; one per (device, stream) is
    reused, the two stacks' streams run LN backwards concurrently and get one each)."""
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), _stream())
    nbytes = int(_lib.load().savqa_ln_bwd_workspace_bytes(int(cols)))
    ws = _ln_ws.get(key)
    if ws is None or ws.numel() * 4 < nbytes:
        ws = torch.zeros((nbytes + 3) // 4, dtype=torch.float32, device=dev)
        _ln_ws[key] = ws
    return ws


def ln_bwd(dy: Tensor, z: Tensor, mean: Tensor, rden: Tensor, std: Tensor, gamma: Tensor,
           dz: Tensor, dgamma: Tensor, dbeta: Tensor, *, dz_add=None, dzb=None):
    """dzb: optional bf16 copy of dz (operand of the next low-precision GEMMs)."""
    cols = gamma.numel()
    rows = z.numel() // cols
    ws = ln_workspace(cols, z.device)
    nb = rows * cols * (4 * (3 + (dz_add is not None)) + 2 * (dzb is not None)) + rows * 12
    _kcall("ln_bwd", nb, 0, "savqa_ln_bwd", _stream(), _p(dy), _p(z), _p(mean), _p(rden), _p(std),
           _p(gamma), rows, cols, _p(dz_add), _p(dz), _p(dgamma), _p(dbeta), _p(ws),
           ws.numel() * 4, _p(dzb))


def rowflag(X: Tensor, rows: int, cols: int, ldx: int, flag: Tensor):
    call("savqa_rowflag", _stream(), _p(X), int(rows), int(cols), int(ldx), _p(flag))


# ------------------------------------------------------------------------------ attention
def gattn_fwd(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H, o, ldo, att=None, dk=64):
    """Graph-attention forward; bf16 Q/K/V select the bf16-storage kernels (fp32 math)."""
    fl = 4.0 * B * H * Tq * Tk * dk
    if k.dtype == torch.bfloat16:
        nb = _attn_bytes(k, B, Tq, Tk, H, dk, Tq + 2 * Tk, 0) + B * H * Tq * dk * o.element_size()
        _kcall(f"gattn_fwd_bf16 T{Tq}x{Tk}", nb, fl, "savqa_gattn_fwd_bf16", _stream(),
               int(q.dtype == torch.bfloat16), _p(q), ldq, _p(k), ldk, _p(v), ldv, _p(G),
               _p(kflag), _p(qflag), B, Tq, Tk, H, dk, _p(o), ldo, _p(att))
        return
    _kcall(f"gattn_fwd T{Tq}x{Tk}", _attn_bytes(q, B, Tq, Tk, H, dk, Tq + 2 * Tk, Tq), fl,
           "savqa_gattn_fwd", _stream(), _p(q), ldq, _p(k), ldk, _p(v), ldv, _p(G), _p(kflag),
           _p(qflag), B, Tq, Tk, H, dk, _p(o), ldo, _p(att))


def gattn_bwd(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H, dout, lddo, dq, lddq, dk_,
              lddk, dv, lddv, dk=64):
    fl = 10.0 * B * H * Tq * Tk * dk
    nb = _attn_bytes(k, B, Tq, Tk, H, dk, 2 * Tq + 2 * Tk, Tq + 2 * Tk)
    if k.dtype == torch.bfloat16:
        _kcall(f"gattn_bwd_bf16 T{Tq}x{Tk}", nb, fl, "savqa_gattn_bwd_bf16", _stream(),
               int(q.dtype == torch.bfloat16), _p(q), ldq, _p(k), ldk, _p(v), ldv, _p(G),
               _p(kflag), _p(qflag), B, Tq, Tk, H, dk, _p(dout), lddo, _p(dq), lddq, _p(dk_),
               lddk, _p(dv), lddv)
        return
    _kcall(f"gattn_bwd T{Tq}x{Tk}", nb, fl, "savqa_gattn_bwd", _stream(), _p(q), ldq, _p(k), ldk,
           _p(v), ldv, _p(G), _p(kflag), _p(qflag), B, Tq, Tk, H, dk, _p(dout), lddo, _p(dq), lddq,
           _p(dk_), lddk, _p(dv), lddv)


# The key-tiled kernels' operands pre-split into bf16 plane tiles in a workspace
# (savqa_gattn_*_flash_ws) instead of by every workgroup. The split pass costs what the kernels
# save except where many query tiles re-split each key tile (profiles/r06_ab_flash_x6.txt): "bwd"
# (default) pre-splits the backward at T_q >= 1024 (571 -> 521 us at T = 1314); "auto" the
# forward there too (the DMA-pipelined kernel: 149 -> 142 us alone, but the relation workload's
# step measured 258.8 vs 249.3 QA-samples/s mean in favour of "bwd", 4 interleaved runs each);
# SAVQA_FLASH_PLANES=1 always, 0 never.
FLASH_PLANES = os.environ.get("SAVQA_FLASH_PLANES", "bwd")


def _flash_ws(B, Tq, Tk, H, bwd, dev):
    if FLASH_PLANES == "0" or (FLASH_PLANES != "1" and Tq < 1024) or \
            (FLASH_PLANES == "bwd" and not bwd):
        return None, 0
    nb = int(_lib.load().savqa_gattn_flash_ws_bytes(B, Tq, Tk, H, int(bwd)))
    ws = _workspace((nb + 3) // 4, dev)   # the stream's slab workspace: launches are ordered
    return ws, nb


def gattn_fwd_flash(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H, o, ldo, stats, dk=64):
    ws, nb = _flash_ws(B, Tq, Tk, H, False, q.device)
    _kcall(f"gattn_fwd_flash T{Tq}x{Tk}", _attn_bytes(q, B, Tq, Tk, H, dk, Tq + 2 * Tk, Tq),
           4.0 * B * H * Tq * Tk * dk, "savqa_gattn_fwd_flash_ws", _stream(), _p(q), ldq, _p(k),
           ldk, _p(v), ldv, _p(G), _p(kflag), _p(qflag), B, Tq, Tk, H, dk, _p(o), ldo, _p(stats),
           _p(ws), nb)


def gattn_bwd_flash(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H, dout, lddo,
                    stats, dq, lddq, dk_, lddk, dv, lddv, dk=64):
    ws, nb = _flash_ws(B, Tq, Tk, H, True, q.device)
    _kcall(f"gattn_bwd_flash T{Tq}x{Tk}",
           _attn_bytes(q, B, Tq, Tk, H, dk, 2 * Tq + 2 * Tk, Tq + 2 * Tk),
           10.0 * B * H * Tq * Tk * dk, "savqa_gattn_bwd_flash_ws", _stream(), _p(q), ldq, _p(k),
           ldk, _p(v), ldv, _p(G), _p(kflag), _p(qflag), B, Tq, Tk, H, dk, _p(dout), lddo,
           _p(stats), _p(dq), lddq, _p(dk_), lddk, _p(dv), lddv, _p(ws), nb)


def gattn_fwd_q1s(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tk, H, o, ldo, stats, dk=64):
    """Single-query attention split over keys (T_q = 1, long T_k: csrc/attn_q1s.hip);
    stats: [B*H*4] fp32 kept for gattn_bwd_q1s."""
    ws = _workspace((int(_lib.load().savqa_gattn_q1s_ws_bytes(B, H, Tk)) + 3) // 4, q.device)
    _kcall(f"gattn_fwd_q1s T1x{Tk}", _attn_bytes(q, B, 1, Tk, H, dk, 1 + 2 * Tk, 1),
           4.0 * B * H * Tk * dk, "savqa_gattn_fwd_q1s", _stream(), _p(q), ldq, _p(k), ldk, _p(v),
           ldv, _p(G), _p(kflag), _p(qflag), B, Tk, H, dk, _p(o), ldo, _p(stats), _p(ws),
           ws.numel() * 4)


def gattn_bwd_q1s(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tk, H, dout, lddo, stats, dq,
                  lddq, dk_, lddk, dv, lddv, dk=64):
    ws = _workspace((int(_lib.load().savqa_gattn_q1s_ws_bytes(B, H, Tk)) + 3) // 4, q.device)
    _kcall(f"gattn_bwd_q1s T1x{Tk}", _attn_bytes(q, B, 1, Tk, H, dk, 2 + 2 * Tk, 1 + 2 * Tk),
           10.0 * B * H * Tk * dk, "savqa_gattn_bwd_q1s", _stream(), _p(q), ldq, _p(k), ldk, _p(v),
           ldv, _p(G), _p(kflag), _p(qflag), B, Tk, H, dk, _p(dout), lddo, _p(stats), _p(dq),
           lddq, _p(dk_), lddk, _p(dv), lddv, _p(ws), ws.numel() * 4)


def use_q1s(Tk: int) -> bool:
    """The decoder's single-query cross-attention at T_k > 128 runs split over keys
    (attn_q1s.hip). SAVQA_ATTN_Q1S=0 keeps it on the key-tiled kernels (A/B), =force uses it at
    every T_k (parity tests on the golden shapes)."""
    mode = os.environ.get("SAVQA_ATTN_Q1S", "1")
    return mode == "force" or (mode != "0" and Tk > FULL_ROW_MAX_T)

FULL_ROW_MAX_T = 128  # attn.hip's full-row kernels; longer sequences use the key-tiled path


def use_flash(Tq: int, Tk: int) -> bool:
    """Key-tiled attention beyond the full-row kernels' limit (SAVQA_ATTN_FLASH=1 forces it)."""
    import os
    if os.environ.get("SAVQA_ATTN_FLASH", "0") == "1":
        return True
    return Tk > FULL_ROW_MAX_T or Tq > FULL_ROW_MAX_T


# ------------------------------------------------------------------------------ misc
def graph_build(node_mask, q_mask, q_graph, node_graph, B, Nn, Lq, dec_on, gdiag, graph, dec_mask):
    call("savqa_graph_build", _stream(), _p(node_mask), _p(q_mask), _p(q_graph), _p(node_graph),
         B, Nn, Lq, int(bool(dec_on)), _p(gdiag), _p(graph), _p(dec_mask))


def dec_init(emb, idx, scale, pos, B, d, out, drop=None, site=-1):
    seed, p = drop if drop is not None else (0, 0.0)
    call("savqa_dec_init", _stream(), _p(emb), int(idx), float(scale), _p(pos), B, d, int(seed),
         int(site), float(p), _p(out))


def dec_init_bwd(g, B, d, idx, scale, demb, dpos, drop=None, site=-1):
    seed, p = drop if drop is not None else (0, 0.0)
    call("savqa_dec_init_bwd", _stream(), _p(g), B, d, int(idx), float(scale), int(seed),
         int(site), float(p), _p(demb), _p(dpos))


# ------------------------------------------------------------------------------ dropout
def dropout(inp, n, drop, site, out):
    """out = nn.Dropout(p)(inp) with the library's counter-hash masks; drop = (seed, p)."""
    seed, p = drop
    call("savqa_dropout", _stream(), _p(inp), int(n), int(seed), int(site), float(p), _p(out))


def posadd_dropout(z, pos, B, T, d, drop, site_pos, site_x, out):
    seed, p = drop
    call("savqa_posadd_dropout", _stream(), _p(z), _p(pos), B, T, d, int(seed), int(site_pos),
         int(site_x), float(p), _p(out))


def posadd_dropout_bwd(g, B, T, d, drop, site_pos, site_x, dz, dpos):
    seed, p = drop
    call("savqa_posadd_dropout_bwd", _stream(), _p(g), B, T, d, int(seed), int(site_pos),
         int(site_x), float(p), _p(dz), _p(dpos))


def period_sum_acc(X, B, T, Cc, ldx, out):
    call("savqa_period_sum_acc", _stream(), _p(X), B, T, Cc, ldx, _p(out))


def copy_rows(src, rows, cols, lds, dst, ldd, group=0, stride=0, offset=0):
    call("savqa_copy_rows", _stream(), _p(src), rows, cols, lds, _p(dst), ldd, group, stride,
         offset)


def mil_fwd(Pf, Nf, v, mask, BN, K, H, eps, obj, ws, mil_out):
    call("savqa_mil_fwd", _stream(), _p(Pf), _p(Nf), _p(v), _p(mask), BN, K, H, float(eps),
         _p(obj), _p(ws), _p(mil_out))


def mil_bwd_bf16(Pf, Nf, v, mask, BN, K, H, eps, dobj, dmil, dPf, dNf, dv):
    """mil_bwd with bf16 dPf / dNf (savqa_mil_bwd_bf16)."""
    call("savqa_mil_bwd_bf16", _stream(), _p(Pf), _p(Nf), _p(v), _p(mask), BN, K, H, float(eps),
         _p(dobj), _p(dmil), _p(dPf), _p(dNf), _p(dv))


def mil_bwd(Pf, Nf, v, mask, BN, K, H, eps, dobj, dmil, dPf, dNf, dv):
    call("savqa_mil_bwd", _stream(), _p(Pf), _p(Nf), _p(v), _p(mask), BN, K, H, float(eps),
         _p(dobj), _p(dmil), _p(dPf), _p(dNf), _p(dv))


# Embedding-table gradients (the GloVe-row scatters dE[ids] += dY W) through a dense GEMM and
# savqa_segment_add_rows over the stably sorted ids (one order per row: run-to-run
# bit-identical) instead of the GEMM's atomic scatter epilogue (SAVQA_DET_SCATTER=0)
DET_SCATTER = os.environ.get("SAVQA_DET_SCATTER", "1") != "0"


def segment_add_rows(T: Tensor, ldt: int, ids: Tensor, cols: int, table: Tensor, ldtab: int):
    """table[ids[r]][:cols] += T[r][:cols] for every row r, summed per id in row order."""
    sid, perm = torch.sort(ids.reshape(-1), stable=True)
    call("savqa_segment_add_rows", _stream(), _p(T), int(ldt), _p(perm), _p(sid), int(sid.numel()),
         int(cols), _p(table), int(ldtab))


def index_put_rows(loc, B, Nv, Ns, H, obj, macro):
    call("savqa_index_put_rows", _stream(), _p(loc), B, Nv, Ns, H, _p(obj), _p(macro))


def index_get_rows(loc, B, Nv, Ns, H, dmacro, dobj):
    call("savqa_index_get_rows", _stream(), _p(loc), B, Nv, Ns, H, _p(dmacro), _p(dobj))


def loss_fwd(lc, lv, ls, answer, B, Cc, eps, mil, with_mil, loss, dlogits, lsm, ws):
    call("savqa_loss_fwd", _stream(), _p(lc), _p(lv), _p(ls), _p(answer), B, Cc, float(eps),
         _p(mil), int(bool(with_mil)), _p(loss), _p(dlogits), _p(lsm), _p(ws))


def scale_by(inp, scale, n, out):
    call("savqa_scale_by", _stream(), _p(inp), _p(scale), int(n), _p(out))


def rowscale_mask(inp, rowscale, mask, rows, cols, out):
    call("savqa_rowscale_mask", _stream(), _p(inp), _p(rowscale), _p(mask), int(rows), int(cols),
         _p(out))


def affine(inp, n, a, b, out):
    call("savqa_affine", _stream(), _p(inp), int(n), float(a), float(b), _p(out))


def gather_rows(table, idx, rows, cols, scale, out):
    call("savqa_gather_rows", _stream(), _p(table), _p(idx), int(rows), int(cols), float(scale),
         _p(out))


def scatter_rows(g, idx, rows, cols, scale, padding_idx, dtable):
    call("savqa_scatter_rows", _stream(), _p(g), _p(idx), int(rows), int(cols), float(scale),
         int(padding_idx), _p(dtable))


# ------------------------------------------------------------------------------ relations
def rel_entries_fwd(loc, B, L, obj, Nv, H, V, ldv, val):
    call("savqa_rel_entries_fwd", _stream(), _p(loc), int(loc.shape[-1]), B, L, _p(obj), Nv, H,
         _p(V), int(ldv), _p(val))


def rel_entries_bwd(loc, B, L, obj, Nv, H, V, ldv, dval, dobj, dV):
    call("savqa_rel_entries_bwd", _stream(), _p(loc), int(loc.shape[-1]), B, L, _p(obj), Nv, H,
         _p(V), int(ldv), _p(dval), _p(dobj), _p(dV))


def _rel_ws(B, Lp, Ln, dev):
    nb = int(_lib.load().savqa_rel_loss_ws_bytes(B, Lp, Ln))
    return _workspace((nb + 3) // 4, dev), nb


def rel_loss_fwd(pos_loc, B, Lp, sp, neg_loc, Ln, sn, eps, cum, wsm, st, mil_rel):
    ws, nb = _rel_ws(B, Lp, Ln, sp.device)
    call("savqa_rel_loss_fwd", _stream(), _p(pos_loc), B, Lp, _p(sp), _p(neg_loc), Ln, _p(sn),
         float(eps), _p(cum), _p(wsm), _p(st), _p(mil_rel), _p(ws), nb)


def rel_macro_fwd(pos_loc, B, Lp, st, wsm, relf, Ns, H, macro):
    call("savqa_rel_macro_fwd", _stream(), _p(pos_loc), B, Lp, _p(st), _p(wsm), _p(relf), Ns, H,
         _p(macro))


def rel_macro_bwd(pos_loc, B, Lp, st, wsm, relf, Ns, H, dmacro, dwsm, drelf):
    call("savqa_rel_macro_bwd", _stream(), _p(pos_loc), B, Lp, _p(st), _p(wsm), _p(relf), Ns, H,
         _p(dmacro), _p(dwsm), _p(drelf))


def rel_loss_bwd(pos_loc, B, Lp, sp, neg_loc, Ln, sn, eps, cum, wsm, dwsm, st, dmil, dsp, dsn):
    ws, nb = _rel_ws(B, Lp, Ln, sp.device)
    call("savqa_rel_loss_bwd", _stream(), _p(pos_loc), B, Lp, _p(sp), _p(neg_loc), Ln, _p(sn),
         float(eps), _p(cum), _p(wsm), _p(dwsm), _p(st), _p(dmil), _p(dsp), _p(dsn), _p(ws), nb)


def axpby(x, y, n, a, b, out):
    call("savqa_axpby", _stream(), _p(x), _p(y), int(n), float(a), float(b), _p(out))


def mark_rows(ids, nrows, flags):
    call("savqa_mark_rows", _stream(), _p(ids), int(ids.numel()), int(nrows), _p(flags))


def zero_rows(g, width, nrows, flags):
    call("savqa_zero_rows", _stream(), _p(g), int(width), int(nrows), _p(flags))


def adam_rows(p, g, m, v, width, nrows, flags, lr, beta1, beta2, eps, bc1, bc2, grad_scale=1.0):
    call("savqa_adam_rows", _stream(), _p(p), _p(g), _p(m), _p(v), int(width), int(nrows),
         _p(flags), float(lr), float(beta1), float(beta2), float(eps), float(bc1), float(bc2),
         float(grad_scale))


def adam(p, g, m, v, n, lr, beta1, beta2, eps, bc1, bc2, grad_scale=1.0, shadow=None):
    # 28 B per parameter: p, m, v read and written, g read (+2 B: the optional bf16 shadow)
    if shadow is None:
        _kcall("adam", 28 * int(n), 0, "savqa_adam", _stream(), _p(p), _p(g), _p(m), _p(v),
               int(n), float(lr), float(beta1), float(beta2), float(eps), float(bc1), float(bc2),
               float(grad_scale))
    else:
        _kcall("adam", 30 * int(n), 0, "savqa_adam_shadow", _stream(), _p(p), _p(g), _p(m),
               _p(v), int(n), float(lr), float(beta1), float(beta2), float(eps), float(bc1),
               float(bc2), float(grad_scale), _p(shadow))
