#!/usr/bin/env python
"""HIP-event timing of savqa_ln_fwd / savqa_ln_bwd at the step's row counts vs a copy of the
same bytes (torch), to price the LayerNorm kernels against HBM."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from savqa_amd import ops  # noqa: E402


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


for rows, d in ((18688, 512), (12800, 512), (256, 512), (37376, 512), (14368, 1024)):
    x, r = torch.randn(rows, d, device="cuda"), torch.randn(rows, d, device="cuda")
    g, b = torch.rand(d, device="cuda") + 0.5, torch.randn(d, device="cuda")
    y, z = torch.empty_like(x), torch.empty_like(x)
    st = [torch.empty(rows, device="cuda") for _ in range(3)]
    fl = torch.empty(rows, device="cuda")
    f = lambda: ops.ln_fwd(x, g, b, y, *st, r=r, z_out=z, flag=fl)
    t_f = timeit(f)
    f()
    dy, dz = torch.randn_like(x), torch.empty_like(x)
    dg, db = torch.zeros(d, device="cuda"), torch.zeros(d, device="cuda")
    fb = lambda: ops.ln_bwd(dy, z, *st, g, dz, dg, db)
    t_b = timeit(fb)
    big = torch.empty(rows * d * 3, device="cuda")
    t_c = timeit(lambda: big.copy_(torch.empty_like(big)))  # 3 reads+3 writes worth
    nb = rows * d * 4
    print(f"rows={rows:6d} d={d}: ln_fwd {t_f*1e6:7.1f}us ({4*nb/t_f/1e9:6.0f} GB/s)  "
          f"ln_bwd {t_b*1e6:7.1f}us ({3*nb/t_b/1e9:6.0f} GB/s)  copy6 {t_c*1e6:7.1f}us "
          f"({6*nb/t_c/1e9:6.0f} GB/s)", flush=True)
