#!/usr/bin/env python
"""Per-shape GEMM time of one training step of a bench.py workload (streams serialised, HIP
events per launch): which GEMMs of the real step run below the standalone rates. Usage:
python tools/gemm_breakdown.py [workload (cfg2|cfg3|cfg5|cfg4)] [batch]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from savqa_amd import ops  # noqa: E402
from savqa_amd.AttModel_x3 import AttModel  # noqa: E402
from savqa_amd.data import model_args, synthetic_batch  # noqa: E402
from savqa_amd.loss import smoothed_loss  # noqa: E402
from savqa_amd.optim import Adam  # noqa: E402
from savqa_amd.utils import init_params_  # noqa: E402


def main():
    from bench import WORKLOADS
    wl = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    W = WORKLOADS[wl]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else W["batch"]
    dev = torch.device("cuda", 0)
    model = AttModel(None, W["d"], 1024, 914, 40, 450, 49, 6, W["H"], 0.5, 0.1, 311, True,
                     device=dev, init=False, gemm_precision=W.get("prec", "fp32"))
    init_params_(model, seed=0)
    model.train()
    model._engine.concurrent = False
    opt = Adam(model, lr=1e-4)
    batch = synthetic_batch(B, Nv=W["Nv"], Ns=W["Ns"], seed=1234, device=dev)
    margs = model_args(batch)

    def step():
        lc, lv, ls, mil, mil_rel = model(*margs, decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil, with_milnce=True)
        opt.zero_grad()
        loss.backward()
        opt.step()

    for _ in range(2):
        step()
    probe = ops.GemmProbe(detail=True)
    ops.set_gemm_probe(probe)
    step()
    ops.set_gemm_probe(None)
    agg = probe.summary()
    tot = sum(v[2] for v in agg.values())
    print(f"{wl} B={B}: total GEMM {tot:.2f} ms/step, {sum(v[1] for v in agg.values()) / tot / 1e9:.1f} TF")
    for k, (n, fl, ms) in sorted(agg.items(), key=lambda kv: -kv[1][2]):
        print(f"{ms:8.3f} ms {100 * ms / tot:5.1f}%  n={n:3d}  {fl / ms / 1e9:7.1f} TF  {k}")


if __name__ == "__main__":
    main()
