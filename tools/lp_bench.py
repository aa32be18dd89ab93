#!/usr/bin/env python
"""Micro-benchmark of savqa_gemm_lp (bf16 / fp8 operands) on the cfg-3 (B=512) and cfg-5
(B=1024) training-step GEMM shapes, with torch.mm on bf16 (hipBLASLt) as a yardstick.
HIP-event timed; random operands (cdna_hip_programming.md rule 25)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from savqa_amd import ops  # noqa: E402

dev = "cuda"
BF = torch.bfloat16


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def bf16_case(lay, m, n, k, out, hint=0):
    if lay == "NT":
        A, B = torch.randn(m, k, device=dev).to(BF), torch.randn(n, k, device=dev).to(BF)
        kw = dict(lda=k, ldb=k, b_trans=True)
        ref = lambda: torch.mm(A, B.t())
    elif lay == "NN":
        A, B = torch.randn(m, k, device=dev).to(BF), torch.randn(k, n, device=dev).to(BF)
        kw = dict(lda=k, ldb=n)
        ref = lambda: torch.mm(A, B)
    else:
        A, B = torch.randn(k, m, device=dev).to(BF), torch.randn(k, n, device=dev).to(BF)
        kw = dict(lda=m, ldb=n, a_trans=True)
        ref = lambda: torch.mm(A.t(), B)
    if out == "bf16mask":   # the ReLU-backward dX of the FFN: bf16 out, bf16 mask
        Cb = torch.empty(m, n, device=dev, dtype=BF)
        mk = torch.randn(m, n, device=dev).to(BF)
        f = lambda: ops.gemm_lp(A, B, m, n, k, Cb=Cb, ldcb=n, mask=mk, ldmask=n, tile_hint=hint,
                                **kw)
    elif out == "bf16bits":  # the same gate as a SAVQA_DT_BITS image (engine.LP_BITS)
        Cb = torch.empty(m, n, device=dev, dtype=BF)
        w = 2 ** torch.arange(8, device=dev, dtype=torch.int32)
        mk = ((torch.randn(m, n // 8, 8, device=dev) > 0).int() * w).sum(-1).to(torch.uint8)
        f = lambda: ops.gemm_lp(A, B, m, n, k, Cb=Cb, ldcb=n, mask=mk, ldmask=n // 8,
                                tile_hint=hint, **kw)
    elif out == "f32resid":  # FFN conv2 forward / dX with the residual: fp32 out + resid
        C = torch.empty(m, n, device=dev)
        R = torch.randn(m, n, device=dev)
        f = lambda: ops.gemm_lp(A, B, m, n, k, C=C, ldc=n, resid=R, ldr=n, tile_hint=hint, **kw)
    elif out == "bf16":
        Cb = torch.empty(m, n, device=dev, dtype=BF)
        f = lambda: ops.gemm_lp(A, B, m, n, k, Cb=Cb, ldcb=n, relu=True, tile_hint=hint, **kw)
    elif out.startswith("atomic"):  # "atomic" (library split) or "atomicS" (split_k = S)
        C = torch.zeros(m, n, device=dev)
        sk = int(out[6:]) if len(out) > 6 else -1
        slabs = os.environ.get("SAVQA_LP_SLABS", "1") != "0"  # split-K slabs (ops.linear_dw_lp)
        f = lambda: ops.gemm_lp(A, B, m, n, k, C=C, ldc=n, atomic=True, split_k=sk,
                                tile_hint=hint, slabs=slabs, **kw)
    else:
        C = torch.empty(m, n, device=dev)
        f = lambda: ops.gemm_lp(A, B, m, n, k, C=C, ldc=n, tile_hint=hint, **kw)
    return f, ref


def fp8_case(m, n, k):
    X = torch.randn(m, k, device=dev).clamp_min(0)
    W = torch.randn(n, k, device=dev) / k ** 0.5
    qx, sx = torch.empty(m, k, dtype=torch.uint8, device=dev), torch.empty(m, k // 32, dtype=torch.uint8, device=dev)
    qw, sw = torch.empty(n, k, dtype=torch.uint8, device=dev), torch.empty(n, k // 32, dtype=torch.uint8, device=dev)
    ops.quant_fp8(X, m, k, k, qx, k, sx, k // 32)
    ops.quant_fp8(W, n, k, k, qw, k, sw, k // 32)
    C = torch.empty(m, n, device=dev)
    f = lambda: ops.gemm_lp(qx.view(torch.float8_e4m3fn), qw.view(torch.float8_e4m3fn), m, n, k,
                            lda=k, ldb=k, b_trans=True, a_scale=sx, lds_a=k // 32, b_scale=sw,
                            lds_b=k // 32, C=C, ldc=n)
    A16, W16 = X.to(BF), W.to(BF)
    return f, lambda: torch.mm(A16, W16.t())


def main():
    Ms = 37376  # cfg 3 semantic stack rows: 512 x 73
    cases = [("fwd qkv", "NT", Ms, 1536, 512, "bf16"), ("fwd ffn1", "NT", Ms, 2048, 512, "bf16"),
             ("fwd ffn2", "NT", Ms, 512, 2048, "f32"), ("fwd kv_all", "NT", Ms, 6144, 512, "bf16"),
             ("fwd in", "NT", Ms, 512, 2048, "f32"),
             ("dx ffn2", "NN", Ms, 2048, 512, "bf16"), ("dx ffn1", "NN", Ms, 512, 2048, "f32"),
             ("dx qkv", "NN", Ms, 512, 1536, "f32"), ("dx kv", "NN", Ms, 512, 6144, "f32"),
             ("dw qkv", "TN", 1536, 512, Ms, "atomic"), ("dw ffn1", "TN", 2048, 512, Ms, "atomic"),
             ("dw ffn2", "TN", 512, 2048, Ms, "atomic"), ("dw kv", "TN", 6144, 512, Ms, "atomic"),
             ("dx ffn2 m", "NN", Ms, 2048, 512, "bf16mask"), ("dx ffn2 b", "NN", Ms, 2048, 512, "bf16bits"),
             ("fwd ffn2 r", "NT", Ms, 512, 2048, "f32resid"),
             ("dx ffn1 r", "NN", Ms, 512, 2048, "f32resid")]
    hints = [0] + ([1, 3, 4, 5] if "--variants" in sys.argv else [])
    if "--square" in sys.argv:  # structure check at 8192^3 / 4096^3 (cdna guide's reference shapes)
        hints = [1, 3, 5]
        cases = [(f"sq{n}", lay, n, n, n, "bf16") for n in (4096, 8192) for lay in ("NT", "NN", "TN")]
    if "--msweep" in sys.argv:  # wave quantisation: the same shapes at whole-round row counts
        hints = [1, 3, 4, 5]
        cases = [(f"m{m}", lay, m, n, k, out) for m in (32768, 37376, 40960)
                 for lay, n, k, out in (("NT", 512, 2048, "f32"), ("NN", 512, 2048, "f32"),
                                        ("NT", 2048, 512, "bf16"), ("NN", 2048, 512, "bf16"))]
    if "--dbg1" in sys.argv:  # 128x128 kernel as is / no MFMAs / no DMAs / no epilogue (needs a
        # diagnostic build: the tile_hint >> 8 bits tested in gemm_lp_kernel as in gemm_lp3_kernel)
        hints = [1, 1 + 256, 1 + 512, 1 + 1024, 1 + 256 + 1024, 1 + 256 + 512]
        cases = [cases[i] for i in (1, 2, 5, 10, 13)]
    elif "--dbg" in sys.argv:  # v5 as is / without MFMAs / without k-loop DMAs / no epilogue
        hints = [5, 5 + 256, 5 + 512, 5 + 1024, 5 + 256 + 1024]
        cases = cases[1:4] + cases[6:7] + cases[10:11]
    if "--fp8" in sys.argv:  # only the cfg-5 fp8 region-feature GEMMs
        cases = []
    custom = [a for a in sys.argv[1:] if a.count(":") == 4]  # LAYOUT:M:N:K:OUT
    if custom:
        cases = [(a, a.split(":")[0], int(a.split(":")[1]), int(a.split(":")[2]),
                  int(a.split(":")[3]), a.split(":")[4]) for a in custom]
    if "--dwvar" in sys.argv:  # the weight-gradient shapes on every kernel variant
        hints = [1, 3, 4, 5]
        cases = [c for c in cases if c[0].startswith("dw")]
    if "--splits" in sys.argv:  # split-K factor sweep of the weight-gradient shapes
        cases = [(f"{nm} s{sk}", "TN", m, n, k, "atomic" + (str(sk) if sk > 0 else ""))
                 for nm, m, n, k in (("dw ffn1", 2048, 512, Ms), ("dw qkv", 1536, 512, Ms),
                                     ("dw ffn2", 512, 2048, Ms))
                 for sk in (-1, 2, 3, 4, 6, 8, 12)]
    tot_f = 0.0
    tot_t = {h: 0.0 for h in hints}
    for name, lay, m, n, k, out in cases:
        fl = 2.0 * m * n * k
        tot_f += fl
        fs = {h: bf16_case(lay, m, n, k, out, h) for h in hints}
        t2 = timeit(fs[hints[0]][1])
        ts = {h: [] for h in hints}
        for _ in range(3):  # interleaved rounds (rule 24), min
            for h in hints:
                ts[h].append(timeit(fs[h][0]))
        line = f"{name:10s} {lay} {m:6d}x{n:5d}x{k:6d} {out:8s}"
        for h in hints:
            t1 = min(ts[h])
            tot_t[h] += t1
            line += f" v{h} {t1*1e6:7.1f}us {fl/t1/1e12:6.1f}TF"
        print(line + f" | torch bf16 {t2*1e6:7.1f}us {fl/t2/1e12:6.1f}TF", flush=True)
    for h in (hints if cases else []):
        print(f"bf16 total v{h}: {tot_f/tot_t[h]/1e12:.1f} TF over the cfg-3 encoder shapes",
              flush=True)
    for name, m, n, k in (() if "--square" in sys.argv else
                          (("fp8 vis in", 1024 * 50, 512, 2048), ("fp8 vis_mlp", 1024 * 36, 1024, 2048))):
        f, g = fp8_case(m, n, k)
        fl = 2.0 * m * n * k
        t1, t2 = timeit(f), timeit(g)
        print(f"{name:10s} NT {m:6d}x{n:5d}x{k:6d} fp8    savqa_lp {t1*1e6:8.1f}us "
              f"{fl/t1/1e12:7.1f} TF   torch bf16 {t2*1e6:8.1f}us {fl/t2/1e12:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
