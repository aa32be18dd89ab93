#!/usr/bin/env python
"""Determinism of single GEMM launches at the shapes the race probe flagged: the MIL-NCE
macro projection relu(E[ids] Wm^T + b) (gathered rows, K = 300) and friends. Prints
where two launches on identical inputs differ."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import savqa_amd  # noqa: E402,F401
from savqa_amd import ops  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
for (M, N, K, gather) in [(480, 128, 300, True), (2880, 128, 300, True), (576, 128, 2048, False),
                          (480, 1024, 300, True), (704, 256, 2048, False)]:
    E = torch.randn(5000 if gather else M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
    b = torch.randn(N, device=dev, generator=g)
    ids = torch.randint(0, 5000, (M,), device=dev, generator=g) if gather else None
    outs = []
    for r in range(4):
        o = torch.full((M, N), float("nan"), device=dev)
        ops.linear(E, W, b, o, relu=True, a_rows=ids)
        torch.cuda.synchronize()
        outs.append(o.clone())
    ref = torch.relu((E[ids] if gather else E).double() @ W.double().t() + b.double())
    for r, o in enumerate(outs):
        bad = ~torch.isclose(o.double(), ref, rtol=1e-4, atol=1e-4)
        nb = int(bad.sum())
        msg = f"M={M} N={N} K={K} gather={gather} launch {r}: {nb} bad of {M * N}"
        if nb:
            rr, cc = bad.nonzero(as_tuple=True)
            msg += f", rows {int(rr.min())}..{int(rr.max())} cols {int(cc.min())}..{int(cc.max())}," \
                   f" nan {int(torch.isnan(o).sum())}"
        print(msg, flush=True)
