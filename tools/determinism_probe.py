#!/usr/bin/env python
"""Run-to-run determinism of one training step: the same weights and batch through
forward + loss + backward twice (fresh gradient arena each time); prints every live
parameter whose gradient differs bit-wise between the two runs, with the max relative
difference. usage: python tools/determinism_probe.py [fp32|fp32_native|bf16] [B]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    import savqa_amd  # noqa: F401
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.utils import init_params_
    m = AttModel(None, 512, 1024, 914, 40, 450, 49, 6, 8, 0.0, 0.1, 311, True, device="cuda",
                 init=False, gemm_precision=prec)
    init_params_(m, seed=5)
    m.train()
    b = synthetic_batch(B, seed=77)
    a = m._arena
    grads = []
    for _ in range(2):
        lc, lv, ls, mil, _ = m(*model_args(b), decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, b["answer"], mil)
        m.zero_grad(set_to_none=False)
        loss.backward()
        torch.cuda.synchronize()
        grads.append(a.grad[:a.n_live].clone())
    g0, g1 = grads
    print(f"{prec} B={B}: whole live gradient equal: {torch.equal(g0, g1)}")
    for n in a.live_names:
        o, shp = a.offsets[n]
        x, y = g0[o:o + shp.numel()], g1[o:o + shp.numel()]
        if not torch.equal(x, y):
            d = float((x - y).abs().max() / y.abs().max().clamp_min(1e-30))
            nd = int((x != y).sum())
            print(f"  differs: {n:60s} {nd:9d} elements  max rel {d:.2e}")


if __name__ == "__main__":
    main()
