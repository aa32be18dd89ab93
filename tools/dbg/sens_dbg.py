"""Sensitivity of the half-batch loss to parameter perturbations of rounding size (debug aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import tests.test_ddp_gpu as T
from savqa_amd.data import model_args
from savqa_amd.loss import smoothed_loss
from savqa_amd.optim import Adam


def loss_at(m, flat, batch):
    with torch.no_grad():
        m._arena.flat.copy_(flat)
    lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
    loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
    return float(loss), lc.detach().clone(), lv.detach().clone(), ls.detach().clone(), float(mil)


def main():
    full = T._equiv_batch()
    half = {k: v[:4] for k, v in full.items()}
    m = T._equiv_model()
    p0 = m._arena.flat.clone()
    opt = Adam(m, lr=1e-4)
    lc, lv, ls, mil, _ = m(*model_args(full), decMask=True, mcb=False)
    loss, _ = smoothed_loss(lc, lv, ls, full["answer"], mil)
    opt.zero_grad()
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    p1 = m._arena.flat.clone()
    a = m._arena
    g = torch.Generator(device="cuda").manual_seed(0)
    for tag, p in (("p0", p0), ("p1", p1)):
        L0, c0, v0, s0, mil0 = loss_at(m, p, half)
        print(tag, "base", L0, "mil", mil0)
        for name_filter in ("all", "att_vis_grid", "att_syb", "MIL_NCE", "cls"):
            q = p.clone()
            for n in a.live_names:
                if name_filter != "all" and not n.startswith(name_filter):
                    continue
                o, shp = a.offsets[n]
                v = q[o:o + shp.numel()]
                v.add_(v * 1e-6 * (torch.rand(v.shape, generator=g, device="cuda") - 0.5))
            L, c, vv, ss, mil1 = loss_at(m, q, half)
            print(f"  perturb {name_filter}: dloss {L - L0:.3e} dmil {mil1 - mil0:.3e} "
                  f"dlc {float((c - c0).abs().max()):.3e} dlv {float((vv - v0).abs().max()):.3e} "
                  f"dls {float((ss - s0).abs().max()):.3e}", flush=True)


if __name__ == "__main__":
    main()
