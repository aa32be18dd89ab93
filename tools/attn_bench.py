#!/usr/bin/env python
"""Graph-attention core in isolation at the cfg-2 step shapes (QKV interleaved as the
engine lays it out: one [B*T, 3*d] buffer), HIP-event timed; bytes = Q,K,V + graph +
flags read and O (fwd) / dQ,dK,dV (bwd) written, per launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from savqa_amd import ops  # noqa: E402

dev = "cuda"


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


def main():
    H, dk = 8, 64
    d = H * dk
    for B, T in ((256, 73), (256, 50)):
        qkv = torch.randn(B * T, 3 * d, device=dev).relu_()
        G = (torch.rand(B, T, T, device=dev) < 0.3).float()
        flag = torch.ones(B * T, device=dev)
        o = torch.empty(B * T, d, device=dev)
        dout = torch.randn(B * T, d, device=dev)
        dqkv = torch.zeros(B * T, 3 * d, device=dev)
        f = lambda: ops.gattn_fwd(qkv, 3 * d, qkv[:, d:], 3 * d, qkv[:, 2 * d:], 3 * d, G, flag,
                                  flag, B, T, T, H, o, d)
        g = lambda: ops.gattn_bwd(qkv, 3 * d, qkv[:, d:], 3 * d, qkv[:, 2 * d:], 3 * d, G, flag,
                                  flag, B, T, T, H, dout, d, dqkv, 3 * d, dqkv[:, d:], 3 * d,
                                  dqkv[:, 2 * d:], 3 * d)
        tf, tb = timeit(f), timeit(g)
        fb = B * T * 3 * d * 4 + B * T * T * 4 + B * T * d * 4
        bb = B * T * 4 * d * 4 + B * T * T * 4 + B * T * 3 * d * 4
        ffl = B * H * 4 * T * T * dk
        bfl = B * H * 10 * T * T * dk
        print(f"B={B} T={T}: fwd {tf*1e6:7.1f} us {fb/tf/1e9:6.0f} GB/s {ffl/tf/1e12:5.1f} TF | "
              f"bwd {tb*1e6:7.1f} us {bb/tb/1e9:6.0f} GB/s {bfl/tb/1e12:5.1f} TF", flush=True)


if __name__ == "__main__":
    main()
