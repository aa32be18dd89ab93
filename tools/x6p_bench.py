#!/usr/bin/env python
"""x6 from pre-split planes (gemm_x6p_kernel) against the register-split x6 kernel on the cfg-2
step shapes: HIP-event time of each, of the savqa_split3 passes, and the max error of both
against fp64. usage: python tools/x6p_bench.py [LAYOUT:M:N:K ...]"""
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
    M = 18688
    cases = [("NT", M, 1536, 512), ("NT", M, 2048, 512), ("NT", M, 512, 2048),
             ("NT", M, 6144, 512), ("NN", M, 2048, 512), ("NN", M, 512, 2048),
             ("NN", M, 512, 1536), ("NN", M, 512, 6144), ("TN", 1536, 512, M),
             ("TN", 2048, 512, M), ("TN", 512, 2048, M), ("TN", 6144, 512, M)]
    if len(sys.argv) > 1:
        cases = [(a.split(":")[0],) + tuple(int(x) for x in a.split(":")[1:]) for a in sys.argv[1:]]
    tot = {"x6": 0.0, "x6p": 0.0, "split": 0.0, "fl": 0.0}
    for lay, m, n, k in cases:
        fl = 2.0 * m * n * k
        g = torch.Generator(device=dev).manual_seed(m + n + k)
        if lay == "NT":
            A = torch.randn(m, k, device=dev, generator=g)
            B = torch.randn(n, k, device=dev, generator=g)
            kw = dict(lda=k, ldb=k, ldc=n, b_trans=True)
            ref = A.double() @ B.double().t()
            sa = lambda: ops.split3(A, m, k, k)
            sb = lambda: ops.split3(B, n, k, k)
        elif lay == "NN":
            A = torch.randn(m, k, device=dev, generator=g)
            B = torch.randn(k, n, device=dev, generator=g)
            kw = dict(lda=k, ldb=n, ldc=n)
            ref = A.double() @ B.double()
            sa = lambda: ops.split3(A, m, k, k)
            sb = lambda: ops.split3(B, k, n, n)
        else:
            A = torch.randn(k, m, device=dev, generator=g)
            B = torch.randn(k, n, device=dev, generator=g)
            kw = dict(lda=m, ldb=n, ldc=n, a_trans=True, atomic=True, split_k=-1)
            ref = A.double().t() @ B.double()
            sa = lambda: ops.split3(A, k, m, m)
            sb = lambda: ops.split3(B, k, n, n)
        ap, bp = sa(), sb()
        C = torch.zeros(m, n, device=dev)
        errs = {}
        for name, extra in (("x6", {}), ("x6p", dict(ap=ap, bp=bp))):
            C.zero_()
            ops.gemm(A, B, C, m, n, k, prec=6, **kw, **extra)
            torch.cuda.synchronize()
            errs[name] = float((C.double() - ref).abs().max() / ref.abs().max())
        t6 = timeit(lambda: ops.gemm(A, B, C, m, n, k, prec=6, **kw))
        tp = timeit(lambda: ops.gemm(A, B, C, m, n, k, prec=6, ap=ap, bp=bp, **kw))
        ts = timeit(lambda: (ops.split3(A, *( (m, k, k) if lay != "TN" else (k, m, m)), out=ap)))
        plan = ops.gemm(A, B, C, m, n, k, prec=6, ap=ap, bp=bp, plan_only=True, **kw)
        tot["x6"] += t6
        tot["x6p"] += tp
        tot["split"] += ts
        tot["fl"] += fl
        print(f"{lay} {m:6d}x{n:5d}x{k:6d}  x6 {t6 * 1e6:7.1f}us {fl / t6 / 1e12:6.1f}TF  "
              f"x6p {tp * 1e6:7.1f}us {fl / tp / 1e12:6.1f}TF (plan {plan})  splitA "
              f"{ts * 1e6:6.1f}us  err x6 {errs['x6']:.2e} x6p {errs['x6p']:.2e}", flush=True)
    print(f"total: x6 {tot['fl'] / tot['x6'] / 1e12:.1f} TF, x6p {tot['fl'] / tot['x6p'] / 1e12:.1f} TF "
          f"(+ A splits {tot['split'] * 1e6:.0f} us over {tot['x6p'] * 1e6:.0f} us)")


if __name__ == "__main__":
    main()
