#!/usr/bin/env python
"""Root cause of the cfg-2 deep-gradient spread (x6 seed 3, cls_vis.0.weight 3e-3
from fp64 while native lands 5e-7): count the ReLU units whose decision differs between the
HIP fp32 forward and the fp64 oracle's own forward, per site, and compare the HIP gradients
with fp64 both unaligned (the oracle's own ReLUs) and branch-aligned (the oracle under the HIP
path's masks, tests/branch_masks.py). Test infrastructure (imports the oracle).
usage: SEEDS=0,3,7 python tools/relu_flips.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import branch_masks  # noqa: E402
from oracle import savqa_oracle as O  # noqa: E402
from savqa_amd import engine  # noqa: E402

NAMES = ["cls.0.weight", "cls_vis.0.weight", "att_vis_grid.enc_self_attention_0.Q_proj.0.weight",
         "att_syb.syb_mlp.0.weight", "att_vis_grid.syb_mlp2.weight",
         "att_syb.enc_feed_forward_0.conv1.0.weight", "MIL_NCE.vis_mlp.0.weight",
         "MIL_NCE.ipt_mlp.0.weight"]


def frob(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def main():
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.utils import init_params_
    model = AttModel(None, 512, 1024, 914, 40, 450, 49, 6, 8, 0.0, 0.1, 311, True, device="cuda",
                     init=False)
    params = dict(model.named_parameters())
    for seed in [int(x) for x in os.environ.get("SEEDS", "0,3").split(",")]:
        init_params_(model, seed=11 + seed)
        g = torch.Generator(device="cuda").manual_seed(12 + seed)
        with torch.no_grad():
            for n, p in model.named_parameters():
                if n.endswith(".gamma"):
                    p.normal_(1.0, 0.2, generator=g)
                elif n.endswith(".beta"):
                    p.normal_(0.0, 0.2, generator=g)
        b = synthetic_batch(256, Nv=36, Ns=59, seed=2024 + seed, device="cuda")
        model.train()
        print(f"== seed {seed}")
        for kernel in ("x6", "native"):
            engine.FP32_GEMM = kernel
            box = branch_masks.capture(model)
            lc, lv, ls, mil, _ = model(*model_args(b), decMask=True, mcb=False)
            masks = branch_masks.hip_masks(box[0])
            loss, _ = smoothed_loss(lc, lv, ls, b["answer"], mil)
            model.zero_grad(set_to_none=False)
            loss.backward()
            torch.cuda.synchronize()
            mine = {n: params[n].grad.detach().clone() for n in NAMES}
            own = {"_record": True}
            r64, _ = branch_masks.oracle_grads(O, params, b, own, torch.float64, "cuda", NAMES)
            a64, _ = branch_masks.oracle_grads(O, params, b, masks, torch.float64, "cuda", NAMES)
            flips = {}
            for k in masks:
                if k not in own:
                    continue
                a, o = masks[k].to(own[k].device).reshape(own[k].shape), own[k]
                if ".enc_self_attention_0." in k[0] or ".enc_self_attention_1." in k[0]:
                    if k[0].endswith(("Q_proj.0", "V_proj.0")):  # node rows not computed
                        nn = 36 if k[0].startswith("att_vis") else 59
                        a, o = a[:, nn:], o[:, nn:]
                flips[k] = int((a != o).sum())
            nz = {f"{k[0]}#{k[1]}": v for k, v in flips.items() if v}
            print(f"  {kernel}: ReLU units decided differently from the fp64 forward: "
                  f"{sum(flips.values())} of {sum(m.numel() for m in masks.values())} {nz}")
            for n in NAMES:
                print(f"    {n:52s} unaligned {frob(mine[n], r64[n]):.2e}  "
                      f"branch-aligned {frob(mine[n], a64[n]):.2e}")
        engine.FP32_GEMM = "x6"


if __name__ == "__main__":
    main()
