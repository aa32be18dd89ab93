"""Where a row-tracked Adam step differs from the dense replay (debug aid)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import savqa_amd  # noqa
from savqa_amd import ops
from savqa_amd.AttModel_x3 import AttModel
from savqa_amd.data import model_args, synthetic_batch
from savqa_amd.loss import smoothed_loss
from savqa_amd.optim import Adam
from savqa_amd.utils import init_params_
m = AttModel(None, 256, 64, 12, 16, 60, 10, 2, 4, 0.0, 0.0, 2, True, device="cuda", init=False)
init_params_(m, seed=5); m.train()
a = m._arena
opt = Adam(m, lr=1e-3)
for step in range(3):
    batch = synthetic_batch(4, Nv=6, Lq=5, Ns=8, topN=5, num_classes=12, seed=100 + step, device="cuda")
    lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
    loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
    opt.zero_grad(); loss.backward(); torch.cuda.synchronize()
    if opt.m is None:
        opt.m = torch.zeros(a.n_live, device="cuda"); opt.v = torch.zeros(a.n_live, device="cuda")
    n = a.n_live
    p0, g0, m0, v0 = a.flat[:n].clone(), a.grad[:n].clone(), opt.m.clone(), opt.v.clone()
    fl = {k: f.clone() for k, f in a.row_flags.items()}
    opt.step(); torch.cuda.synchronize()
    t = opt.step_count
    ops.adam(p0, g0, m0, v0, n, 1e-3, 0.9, 0.999, 1e-8, 1 - 0.9 ** t, 1 - 0.999 ** t, 1.0)
    torch.cuda.synchronize()
    bad = (a.flat[:n] != p0) | (opt.m != m0) | (opt.v != v0)
    print("step", step, "mismatches", int(bad.sum()))
    idx = bad.nonzero().reshape(-1)[:20].tolist()
    for i in idx[:10]:
        name = next(nm for nm in a.live_names if a.offsets[nm][0] <= i < a.offsets[nm][0] + a.offsets[nm][1].numel())
        o, shp = a.offsets[name]
        info = ""
        if name in fl:
            r = (i - o) // shp[1]; info = f"row {r} flag {int(fl[name][r])} g {float(g0[i])}"
        print("  ", i, name, info, float(a.flat[i]), float(p0[i]))
