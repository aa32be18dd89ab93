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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--bf16", action="store_true", help="bf16 Q/K/V storage (cfg-3 mode)")
    ap.add_argument("--B", type=int, nargs="*", default=[256])
    ap.add_argument("--T", type=int, nargs="*", default=[73, 50])
    ap.add_argument("--q1", action="store_true",
                    help="decoder cross-attention: one fp32 query per sample, K/V of T rows")
    ap.add_argument("--flash", action="store_true",
                    help="key-tiled kernels (T > 128: cfg 4, super-node relation graphs), fp32")
    ap.add_argument("--q1s", action="store_true",
                    help="decoder cross-attention at T_k > 128: split-key single-query kernels "
                         "against the key-tiled ones with T_q = 1 (K/V rows of the 6-layer "
                         "[B*T, 12 d] decoder buffer)")
    args = ap.parse_args()
    if args.q1s:
        return q1s_main(args)
    if args.q1:
        return q1_main(args)
    if args.flash:
        return flash_main(args)
    H, dk = 8, 64
    d = H * dk
    dt = torch.bfloat16 if args.bf16 else torch.float32
    for B, T in ((args.B[0], t) for t in args.T):
        qkv = torch.randn(B * T, 3 * d, device=dev).relu_().to(dt)
        G = (torch.rand(B, T, T, device=dev) < 0.3).float()
        flag = torch.ones(B * T, device=dev)
        o = torch.empty(B * T, d, device=dev)
        dout = torch.randn(B * T, d, device=dev)
        dqkv = torch.zeros(B * T, 3 * d, device=dev, dtype=dt)
        f = lambda: ops.gattn_fwd(qkv, 3 * d, qkv[:, d:], 3 * d, qkv[:, 2 * d:], 3 * d, G, flag,
                                  flag, B, T, T, H, o, d)
        g = lambda: ops.gattn_bwd(qkv, 3 * d, qkv[:, d:], 3 * d, qkv[:, 2 * d:], 3 * d, G, flag,
                                  flag, B, T, T, H, dout, d, dqkv, 3 * d, dqkv[:, d:], 3 * d,
                                  dqkv[:, 2 * d:], 3 * d)
        tf, tb = timeit(f), timeit(g)
        es = 2 if args.bf16 else 4  # Q/K/V/dQ/dK/dV element size; O, dO, graph fp32
        fb = B * T * 3 * d * es + B * T * T * 4 + B * T * d * 4
        bb = B * T * 3 * d * es + B * T * d * 4 + B * T * T * 4 + B * T * 3 * d * es
        ffl = B * H * 4 * T * T * dk
        bfl = B * H * 10 * T * T * dk
        print(f"{dt} B={B} T={T}: fwd {tf*1e6:7.1f} us {fb/tf/1e9:6.0f} GB/s {ffl/tf/1e12:5.1f} TF | "
              f"bwd {tb*1e6:7.1f} us {bb/tb/1e9:6.0f} GB/s {bfl/tb/1e12:5.1f} TF", flush=True)


def flash_main(args):
    """gattn_{fwd,bwd}_flash at B x T (e.g. --B 4 --T 1314: the relation workload's stack);
    the backward is reported as its two launches together (dQ, then dK / dV)."""
    H, dk = 8, 64
    d = H * dk
    pairs = zip(args.B, args.T) if len(args.B) == len(args.T) else ((args.B[0], t) for t in args.T)
    for B, T in pairs:
        qkv = torch.randn(B * T, 3 * d, device=dev).relu_()
        G = (torch.rand(B, T, T, device=dev) < 0.3).float()
        flag = torch.ones(B * T, device=dev)
        o = torch.empty(B * T, d, device=dev)
        st = torch.empty(B * H * T, 4, device=dev)
        dout = torch.randn(B * T, d, device=dev)
        dqkv = torch.zeros(B * T, 3 * d, device=dev)
        f = lambda: ops.gattn_fwd_flash(qkv, 3 * d, qkv[:, d:], 3 * d, qkv[:, 2 * d:], 3 * d, G,
                                        flag, flag, B, T, T, H, o, d, st)
        g = lambda: ops.gattn_bwd_flash(qkv, 3 * d, qkv[:, d:], 3 * d, qkv[:, 2 * d:], 3 * d, G,
                                        flag, flag, B, T, T, H, dout, d, st, dqkv, 3 * d,
                                        dqkv[:, d:], 3 * d, dqkv[:, 2 * d:], 3 * d)
        tf = timeit(f)
        tb = timeit(g)
        ffl = B * H * 4 * T * T * dk
        bfl = B * H * 14 * T * T * dk  # dQ: S, dN twice + dS K; dK/dV: S, dN, dV, dK
        print(f"flash B={B} T={T}: fwd {tf*1e6:7.1f} us {ffl/tf/1e12:5.1f} TF | "
              f"bwd {tb*1e6:7.1f} us {bfl/tb/1e12:5.1f} TF", flush=True)


def q1_main(args):
    """T_q = 1 kernels (gattn_{fwd,bwd}_q1): bytes = K, V read + dK, dV written (+ q, o)."""
    H, dk = 8, 64
    d = H * dk
    dt = torch.bfloat16 if args.bf16 else torch.float32
    es = 2 if args.bf16 else 4
    for B, T in ((args.B[0], t) for t in args.T):
        q = torch.randn(B, d, device=dev).relu_()
        # the model's layout: the 6 decoder layers' K / V side by side in one [B T, 12 d] buffer
        kv = torch.randn(B * T, 12 * d, device=dev).relu_().to(dt)
        G = (torch.rand(B, 1, T, device=dev) < 0.3).float()
        kf, qf = torch.ones(B * T, device=dev), torch.ones(B, device=dev)
        o, dout = torch.empty(B, d, device=dev), torch.randn(B, d, device=dev)
        dq = torch.empty(B, d, device=dev)
        dkv = torch.empty(B * T, 12 * d, device=dev, dtype=dt)
        f = lambda: ops.gattn_fwd(q, d, kv, 12 * d, kv[:, d:], 12 * d, G, kf, qf, B, 1, T, H, o, d)
        g = lambda: ops.gattn_bwd(q, d, kv, 12 * d, kv[:, d:], 12 * d, G, kf, qf, B, 1, T, H, dout,
                                  d, dq, d, dkv, 12 * d, dkv[:, d:], 12 * d)
        tf, tb = timeit(f), timeit(g)
        fb = B * T * 2 * d * es
        bb = 2 * B * T * 2 * d * es
        print(f"q1 {dt} B={B} Tk={T}: fwd {tf*1e6:7.1f} us {fb/tf/1e9:6.0f} GB/s | "
              f"bwd {tb*1e6:7.1f} us {bb/tb/1e9:6.0f} GB/s", flush=True)


def q1s_main(args):
    H, dk = 8, 64
    d = H * dk
    ld = 12 * d
    for B, T in ((args.B[0], t) for t in args.T):
        q = torch.randn(B, d, device=dev).relu_()
        kv = torch.randn(B * T, ld, device=dev).relu_()
        G = (torch.rand(B, 1, T, device=dev) < 0.3).float()
        kf, qf = torch.ones(B * T, device=dev), torch.ones(B, device=dev)
        o, dout = torch.empty(B, d, device=dev), torch.randn(B, d, device=dev)
        dq = torch.empty(B, d, device=dev)
        dkv = torch.empty(B * T, ld, device=dev)
        st = torch.empty(B * H * 4, device=dev)
        res = {}
        for name, fw, bw in (
                ("q1s", lambda: ops.gattn_fwd_q1s(q, d, kv, ld, kv[:, d:], ld, G, kf, qf, B, T, H,
                                                  o, d, st),
                 lambda: ops.gattn_bwd_q1s(q, d, kv, ld, kv[:, d:], ld, G, kf, qf, B, T, H, dout,
                                           d, st, dq, d, dkv, ld, dkv[:, d:], ld)),
                ("q1", lambda: ops.gattn_fwd(q, d, kv, ld, kv[:, d:], ld, G, kf, qf, B, 1, T, H, o, d),
                 lambda: ops.gattn_bwd(q, d, kv, ld, kv[:, d:], ld, G, kf, qf, B, 1, T, H, dout, d,
                                       dq, d, dkv, ld, dkv[:, d:], ld)),
                ("flash", lambda: ops.gattn_fwd_flash(q, d, kv, ld, kv[:, d:], ld, G, kf, qf, B, 1,
                                                      T, H, o, d, st),
                 lambda: ops.gattn_bwd_flash(q, d, kv, ld, kv[:, d:], ld, G, kf, qf, B, 1, T, H,
                                             dout, d, st, dq, d, dkv, ld, dkv[:, d:], ld))):
            fw()
            res[name] = (timeit(fw), timeit(bw))
        fb = B * T * 2 * d * 4
        print(f"T_q=1 B={B} Tk={T}: " + " | ".join(
            f"{n} fwd {tf*1e6:6.1f} us ({fb/tf/1e9:5.0f} GB/s) bwd {tb*1e6:6.1f} us "
            f"({3*fb/tb/1e9:5.0f} GB/s)" for n, (tf, tb) in res.items()), flush=True)


if __name__ == "__main__":
    main()
