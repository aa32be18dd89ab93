#!/usr/bin/env python
"""Run one savqa_gemm_lp shape repeatedly (for rocprofv3 PMC passes).
Usage: python tools/lp_one.py LAYOUT M N K OUT HINT [ITERS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lp_bench import bf16_case  # noqa: E402

lay, m, n, k, out, hint = sys.argv[1], *map(int, sys.argv[2:5]), sys.argv[5], int(sys.argv[6])
iters = int(sys.argv[7]) if len(sys.argv) > 7 else 20
f, _ = bf16_case(lay, m, n, k, out, hint)
for _ in range(iters):
    f()
torch.cuda.synchronize()
