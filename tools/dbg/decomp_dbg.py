"""Is the loss gradient batch-decomposable (full-batch grad == mean of the two half-batch
grads) at the init parameters and after one Adam step? (debug aid)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import tests.test_ddp_gpu as T
from savqa_amd.data import model_args
from savqa_amd.loss import smoothed_loss
from savqa_amd.optim import Adam


def grad_at(flat, batch):
    m = T._equiv_model()
    a = m._arena
    with torch.no_grad():
        a.flat.copy_(flat)
    lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
    loss, parts = smoothed_loss(lc, lv, ls, batch["answer"], mil)
    a.ensure_grads()
    loss.backward()
    torch.cuda.synchronize()
    return m, a.grad[:a.n_live].clone(), float(loss), parts


def main():
    full = T._equiv_batch()
    halves = [{k: v[i * 4:(i + 1) * 4] for k, v in full.items()} for i in range(2)]
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
    for tag, p in (("p0", p0), ("p1", p1)):
        mm, gf, lf, pf = grad_at(p, full)
        _, ga, la, pa = grad_at(p, halves[0])
        _, gb, lb, pb = grad_at(p, halves[1])
        print(tag, "loss full", lf, "halves", la, lb, "mean", (la + lb) / 2)
        a = mm._arena
        worst = []
        for n in a.live_names:
            o, shp = a.offsets[n]
            x, y = (ga[o:o + shp.numel()] + gb[o:o + shp.numel()]).double() / 2, gf[o:o + shp.numel()].double()
            if float(y.norm()) == 0:
                continue
            worst.append((float((x - y).norm() / y.norm()), n))
        worst.sort(reverse=True)
        print("  ", worst[:5], flush=True)


if __name__ == "__main__":
    main()
