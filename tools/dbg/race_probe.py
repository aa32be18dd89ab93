#!/usr/bin/env python
"""Find the first kernel whose output differs between two identical training steps (same
state, same inputs): wraps the ops entry points, clones every output on its launch stream
(stream-ordered, no host sync), compares call by call. Usage:
python tools/dbg/race_probe.py [serial]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import savqa_amd  # noqa: E402,F401
from savqa_amd import ops  # noqa: E402
from savqa_amd.AttModel_x3 import AttModel  # noqa: E402
from savqa_amd.data import model_args, synthetic_batch  # noqa: E402
from savqa_amd.loss import smoothed_loss  # noqa: E402
from savqa_amd.optim import Adam  # noqa: E402
from savqa_amd.utils import init_params_  # noqa: E402

# op name -> names of the output arguments (positional index or keyword)
OUTS = {"linear": [3], "linear_dx": [2], "linear_dw": [2, 3], "ln_bwd": [6, 7, 8],
        "ln_fwd": [3], "gattn_bwd": [15, 17, 19], "gattn_fwd": [13], "rowscale_mask": [5],
        "gemm": [2]}
REC = []


def wrap(name, outs):
    fn = getattr(ops, name)

    def w(*a, **k):
        r = fn(*a, **k)
        ts = []
        for o in outs:
            t = a[o] if isinstance(o, int) and o < len(a) else k.get(o) if isinstance(o, str) else None
            if isinstance(t, torch.Tensor):
                ts.append(t.detach().clone())
        for key in ("dz", "dX", "dq", "dkv", "out", "o"):
            if isinstance(k.get(key), torch.Tensor):
                ts.append(k[key].detach().clone())
        REC.append((name, torch.cuda.current_stream().cuda_stream, ts))
        return r
    setattr(ops, name, w)


def main():
    serial = len(sys.argv) > 1 and sys.argv[1] == "serial"
    for n, o in OUTS.items():
        if hasattr(ops, n):
            wrap(n, o)
    m = AttModel(None, 256, 128, 40, 16, 80, 40, 2, 4, 0.0, 0.0, 2, True, device="cuda",
                 init=False)
    init_params_(m, seed=5)
    m.train()
    if serial:
        m._engine.concurrent = False
    batch = synthetic_batch(16, Nv=36, Lq=14, Ns=40, topN=5, num_classes=40, seed=9, device="cuda")
    args = model_args(batch)
    opt = Adam(m, lr=1e-3)
    a = m._arena

    def step():
        lc, lv, ls, mil, _ = m(*args, decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
        opt.zero_grad()
        loss.backward()
        opt.step()

    step()
    torch.cuda.synchronize()
    st = (a.flat.clone(), opt.m.clone(), opt.v.clone(), opt.step_count)
    runs = []
    for _ in range(3):
        a.flat.copy_(st[0]); opt.m.copy_(st[1]); opt.v.copy_(st[2]); opt.step_count = st[3]
        torch.cuda.synchronize()
        REC.clear()
        step()
        torch.cuda.synchronize()
        runs.append((list(REC), a.grad.clone()))
    for r in (1, 2):
        g0, g1 = runs[0][1], runs[r][1]
        print(f"run {r}: grad max rel diff {float((g1 - g0).abs().max() / g0.abs().max()):.3e}")
        shown = 0
        for i, ((n0, s0, t0), (n1, s1, t1)) in enumerate(zip(runs[0][0], runs[r][0])):
            assert n0 == n1
            for j, (x, y) in enumerate(zip(t0, t1)):
                if not torch.equal(x, y):
                    e = float((x - y).abs().max() / x.abs().max().clamp_min(1e-30))
                    print(f"  call {i} {n0} out{j} shape {tuple(x.shape)} stream {s0:#x} rel {e:.3e}")
                    shown += 1
            if shown >= 12:
                break
        print(f"  ({len(runs[0][0])} calls recorded)")


if __name__ == "__main__":
    main()
