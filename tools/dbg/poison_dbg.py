"""Uninitialised-read hunt: fill torch's caching allocator with NaN before building and running
the model, then report the first library calls whose tensor arguments gain NaNs (debug aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import tests.test_ddp_gpu as T
from savqa_amd import ops
from savqa_amd.data import model_args
from savqa_amd.loss import smoothed_loss

REPORT = []


def poison():
    big = torch.empty(1 << 30, device="cuda").fill_(float("nan"))
    small = [torch.empty(1 << 16, device="cuda").fill_(float("nan")) for _ in range(2000)]
    tiny = [torch.empty(1 << 10, device="cuda").fill_(float("nan")) for _ in range(4000)]
    torch.cuda.synchronize()
    del big, small, tiny


def nan_counts(args):
    out = []
    for i, x in enumerate(args):
        if isinstance(x, torch.Tensor) and x.is_floating_point() and x.is_cuda:
            out.append((i, int(torch.isnan(x).sum())))
    return out


def wrap(name, fn):
    def w(*args, **kw):
        allv = list(args) + list(kw.values())
        torch.cuda.synchronize()
        before = nan_counts(allv)
        r = fn(*args, **kw)
        torch.cuda.synchronize()
        after = nan_counts(allv)
        grew = [(i, nb, na) for (i, nb), (_, na) in zip(before, after) if na > nb]
        if grew and len(REPORT) < 12:
            REPORT.append((name, grew, before))
        return r
    return w


def main():
    for n in dir(ops):
        f = getattr(ops, n)
        if callable(f) and not n.startswith("_") and getattr(f, "__module__", "") == ops.__name__ \
                and n not in ("use_flash", "lp_desc", "lp_variant", "lp_supported", "set_gemm_probe",
                              "ln_workspace"):
            setattr(ops, n, wrap(n, f))
    mode = os.environ.get("POISON", "1")
    if mode == "1":
        poison()
    m = T._equiv_model()
    full = T._equiv_batch()
    half = {k: v[:4] for k, v in full.items()}
    lc, lv, ls, mil, _ = m(*model_args(half), decMask=True, mcb=False)
    loss, _ = smoothed_loss(lc, lv, ls, half["answer"], mil)
    m._arena.ensure_grads()
    loss.backward()
    torch.cuda.synchronize()
    print("poison", mode, "loss", float(loss), "lc nan", int(torch.isnan(lc).sum()),
          "grad nan", int(torch.isnan(m._arena.grad).sum()))
    for r in REPORT:
        print("  ", r)


if __name__ == "__main__":
    main()
