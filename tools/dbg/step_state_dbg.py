"""Does a training step depend on state carried from the previous step? Step 1's gradient of a
2-step run vs the gradient of a fresh model loaded with the parameters after step 0, with no
reducer and with a forced 1-rank GradReducer (debug aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.distributed as dist

import tests.test_ddp_gpu as T
from savqa_amd.data import model_args
from savqa_amd.ddp import GradReducer
from savqa_amd.loss import smoothed_loss
from savqa_amd.optim import Adam


def run(steps, red_mode, flat0=None):
    m = T._equiv_model()
    a = m._arena
    if flat0 is not None:
        with torch.no_grad():
            a.flat.copy_(flat0)
    batch = T._equiv_batch()
    if os.environ.get("HALF"):
        batch = {k: v[4 * int(os.environ["HALF"]) - 4:4 * int(os.environ["HALF"])] for k, v in batch.items()}
    red = None
    if red_mode:
        red = GradReducer(a, bucket_mb=1.0, force=True)
        m.attach_reducer(red)
    opt = Adam(m, lr=1e-4)
    flats, grads = [], []
    for _ in range(steps):
        if red:
            red.begin()
        lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
        opt.zero_grad()
        loss.backward()
        torch.cuda.synchronize()
        grads.append(a.grad[:a.n_live].clone())
        opt.step(reducer=red)
        torch.cuda.synchronize()
        flats.append(a.flat.clone())
    return m, flats, grads


def report(tag, m, g, gref):
    a = m._arena
    worst = []
    for n in a.live_names:
        o, shp = a.offsets[n]
        x, y = g[o:o + shp.numel()].double(), gref[o:o + shp.numel()].double()
        if float(y.norm()) == 0:
            continue
        worst.append((float((x - y).norm() / y.norm()), n))
    worst.sort(reverse=True)
    print(tag, worst[:4], flush=True)


def main():
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = "29533"
    dist.init_process_group("gloo", rank=0, world_size=1)
    for red_mode in (False, True):
        m, flats, grads = run(2, red_mode)
        _, _, g1 = run(1, red_mode, flats[0])
        report(f"reducer={red_mode} step1 vs fresh", m, grads[1], g1[0])
        if red_mode:
            report("reducer vs none step0", m, grads[0], ref_g[0])
            report("reducer vs none step1", m, grads[1], ref_g[1])
        else:
            ref_g = grads
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
