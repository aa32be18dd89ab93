#!/usr/bin/env python
"""Run one savqa_gemm shape repeatedly (for rocprofv3 PMC passes).
Usage: python tools/gemm_one.py LAYOUT M N K PREC [ITERS]   (PREC: fp32 | fp32x6 | bf16x3)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from savqa_amd import ops  # noqa: E402

lay, m, n, k, prec = sys.argv[1], *map(int, sys.argv[2:5]), ops.PREC[sys.argv[5]]
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
dev = "cuda"
if lay == "NT":
    A, B = torch.randn(m, k, device=dev), torch.randn(n, k, device=dev)
    kw = dict(lda=k, ldb=k, ldc=n, b_trans=True)
elif lay == "NN":
    A, B = torch.randn(m, k, device=dev), torch.randn(k, n, device=dev)
    kw = dict(lda=k, ldb=n, ldc=n)
else:
    A, B = torch.randn(k, m, device=dev), torch.randn(k, n, device=dev)
    kw = dict(lda=m, ldb=n, ldc=n, a_trans=True, atomic=True, split_k=-1)
C = torch.zeros(m, n, device=dev)
for _ in range(iters):
    ops.gemm(A, B, C, m, n, k, prec=prec, **kw)
torch.cuda.synchronize()
