#!/usr/bin/env python
"""Micro-benchmark of savqa_gemm on the training step's GEMM shapes (cfg 2, B=256)
against torch.mm (hipBLASLt/rocBLAS) as a yardstick. HIP-event timed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from savqa_amd import ops  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
dev = "cuda"


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    prec = ops.PREC[os.environ.get("SAVQA_BENCH_PREC", "fp32")]
    M = 18688
    cases = [("fwd qkv", "NT", M, 1536, 512), ("fwd ffn1", "NT", M, 2048, 512),
             ("fwd ffn2", "NT", M, 512, 2048), ("fwd kv_all", "NT", M, 6144, 512),
             ("dx ffn2", "NN", M, 2048, 512), ("dx ffn1", "NN", M, 512, 2048),
             ("dx qkv", "NN", M, 512, 1536), ("dx kv", "NN", M, 512, 6144),
             ("dw qkv", "TN", 1536, 512, M), ("dw ffn1", "TN", 2048, 512, M),
             ("dw ffn2", "TN", 512, 2048, M), ("dw kv", "TN", 6144, 512, M)]
    if len(sys.argv) > 1:  # custom shapes: LAYOUT:M:N:K ...
        cases = []
        for a in sys.argv[1:]:
            lay, m, n, k = a.split(":")
            cases.append((a, lay, int(m), int(n), int(k)))
    for name, lay, m, n, k in cases:
        fl = 2.0 * m * n * k
        if lay == "NT":
            A = torch.randn(m, k, device=dev)
            W = torch.randn(n, k, device=dev)
            C = torch.empty(m, n, device=dev)
            f = lambda: ops.gemm(A, W, C, m, n, k, lda=k, ldb=k, ldc=n, b_trans=True, prec=prec)
            g = lambda: torch.mm(A, W.t(), out=C)
        elif lay == "NN":
            A = torch.randn(m, k, device=dev)
            W = torch.randn(k, n, device=dev)
            C = torch.empty(m, n, device=dev)
            f = lambda: ops.gemm(A, W, C, m, n, k, lda=k, ldb=n, ldc=n, prec=prec)
            g = lambda: torch.mm(A, W, out=C)
        else:
            A = torch.randn(k, m, device=dev)
            X = torch.randn(k, n, device=dev)
            C = torch.zeros(m, n, device=dev)
            sk = int(os.environ.get("SAVQA_BENCH_SPLIT", "-1"))  # forced split-K (A/B)
            f = lambda: ops.gemm(A, X, C, m, n, k, lda=m, ldb=n, ldc=n, a_trans=True, atomic=True,
                                 split_k=sk, prec=prec)
            g = lambda: torch.mm(A.t(), X, out=C)
        C.zero_()
        f()
        if lay == "NT":
            ref = A.double() @ W.double().t()
        elif lay == "NN":
            ref = A.double() @ W.double()
        else:
            ref = A.double().t() @ X.double()
        err = float((C.double() - ref).abs().max() / ref.abs().max())
        t1 = timeit(f)
        if prec == 3:  # yardstick: torch's bf16 GEMM on bf16 copies
            A16 = A.bfloat16()
            B16 = (W if lay != "TN" else X).bfloat16()
            C16 = C.bfloat16()
            if lay == "NT":
                g = lambda: torch.mm(A16, B16.t(), out=C16)
            elif lay == "NN":
                g = lambda: torch.mm(A16, B16, out=C16)
            else:
                g = lambda: torch.mm(A16.t(), B16, out=C16)
        t2 = timeit(g)
        print(f"{name:10s} {lay} {m:6d}x{n:5d}x{k:6d}  savqa {t1*1e6:8.1f}us {fl/t1/1e12:6.1f} TF   "
              f"torch {t2*1e6:8.1f}us {fl/t2/1e12:6.1f} TF  err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
