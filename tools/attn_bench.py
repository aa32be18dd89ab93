"""Time the graph-attention kernels on the step shapes (B=256, H=8, dk=64).

SAVQA_ATTN_PATH=rows|mfma selects the kernel family (read once per process).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import savqa_amd.ops as O  # noqa: E402

dev = torch.device("cuda")
B, H, D = 256, 8, 512
for Tq, Tk in [(73, 73), (1, 73), (50, 50), (1, 50)]:
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.rand(B * Tq, D, device=dev, generator=g) - 0.3
    kv = torch.rand(B * Tk, 2 * D, device=dev, generator=g) - 0.3
    G = (torch.rand(B, Tq, Tk, device=dev, generator=g) < 0.4).float()
    kf = torch.ones(B, Tk, device=dev)
    qf = torch.ones(B, Tq, device=dev)
    o = torch.empty(B * Tq, D, device=dev)
    dO = torch.randn(B * Tq, D, device=dev, generator=g)
    dq = torch.empty_like(q)
    dkv = torch.empty_like(kv)
    K, V = kv[:, :D], kv[:, D:]

    def fwd():
        O.gattn_fwd(q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, Tq, Tk, H, o, D)

    def bwd():
        O.gattn_bwd(q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, Tq, Tk, H, dO, D, dq, D, dkv, 2 * D,
                    dkv[:, D:], 2 * D)
    res = []
    for fn in (fwd, bwd):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / n * 1e3)
    fl = 2 * B * H * Tq * Tk * 64
    print(f"{os.environ.get('SAVQA_ATTN_PATH', 'default'):7s} Tq={Tq:3d} Tk={Tk:3d}  fwd {res[0]:8.1f} us "
          f"({2 * fl / res[0] / 1e6:6.1f} TF)  bwd {res[1]:8.1f} us ({5 * fl / res[1] / 1e6:6.1f} TF)",
          flush=True)
