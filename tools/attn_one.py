#!/usr/bin/env python
"""Run one graph-attention launch shape repeatedly (for rocprofv3 PMC passes).
Usage: python tools/attn_one.py fwd|bwd fp32|bf16 B T [ITERS]   (H = 8, dk = 64, QKV interleaved
as the engine lays it out; T > 128 runs the key-tiled kernels)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from savqa_amd import ops  # noqa: E402

which, prec, B, T = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
H, dk = 8, 64
d = H * dk
dev = "cuda"
dt = torch.bfloat16 if prec == "bf16" else torch.float32
qkv = torch.randn(B * T, 3 * d, device=dev).relu_().to(dt)
G = (torch.rand(B, T, T, device=dev) < 0.3).float()
flag = torch.ones(B * T, device=dev)
o = torch.empty(B * T, d, device=dev)
dout = torch.randn(B * T, d, device=dev)
dqkv = torch.zeros(B * T, 3 * d, device=dev, dtype=dt)
q, k, v = qkv, qkv[:, d:], qkv[:, 2 * d:]
if T > 128:
    st = torch.empty(B * H * T, 4, device=dev)
    ops.gattn_fwd_flash(q, 3 * d, k, 3 * d, v, 3 * d, G, flag, flag, B, T, T, H, o, d, st)
    f = (lambda: ops.gattn_fwd_flash(q, 3 * d, k, 3 * d, v, 3 * d, G, flag, flag, B, T, T, H, o, d, st)) \
        if which == "fwd" else \
        (lambda: ops.gattn_bwd_flash(q, 3 * d, k, 3 * d, v, 3 * d, G, flag, flag, B, T, T, H, dout, d,
                                     st, dqkv, 3 * d, dqkv[:, d:], 3 * d, dqkv[:, 2 * d:], 3 * d))
else:
    f = (lambda: ops.gattn_fwd(q, 3 * d, k, 3 * d, v, 3 * d, G, flag, flag, B, T, T, H, o, d)) \
        if which == "fwd" else \
        (lambda: ops.gattn_bwd(q, 3 * d, k, 3 * d, v, 3 * d, G, flag, flag, B, T, T, H, dout, d,
                               dqkv, 3 * d, dqkv[:, d:], 3 * d, dqkv[:, 2 * d:], 3 * d))
for _ in range(iters):
    f()
torch.cuda.synchronize()
