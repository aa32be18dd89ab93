#!/usr/bin/env python
"""Conditioning of the cfg-2 parity case (tests/test_fullsize_gpu.py::test_cfg2_against_cpu_oracle):
the same B=256 batch and weights through the HIP path with both fp32 GEMM kernels (x6 and
native), the CPU oracle in fp32 (the reference's arithmetic) and the CPU oracle in fp64.
Prints, per compared gradient, the Frobenius-relative distance of each fp32 computation to the
fp64 one: how far any fp32 summation order lands from the exact gradient at this size.
Test infrastructure (imports the oracle). usage: python tools/cfg2_fp64_check.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_fullsize_gpu as T  # noqa: E402
from oracle import savqa_oracle as O  # noqa: E402
from savqa_amd import engine  # noqa: E402
from savqa_amd.data import model_args  # noqa: E402
from savqa_amd.loss import smoothed_loss  # noqa: E402

NAMES = ["cls.0.weight", "cls_vis.0.weight", "att_vis_grid.enc_self_attention_0.Q_proj.0.weight",
         "att_syb.syb_mlp.0.weight", "att_vis_grid.syb_mlp2.weight",
         "att_syb.enc_feed_forward_0.conv1.0.weight", "MIL_NCE.vis_mlp.0.weight",
         "MIL_NCE.ipt_mlp.0.weight"]


def gpu_grads(model, b, kernel):
    engine.FP32_GEMM = kernel
    params = dict(model.named_parameters())
    lc, lv, ls, mil, _ = model(*model_args(b), decMask=True, mcb=False)
    loss, _ = smoothed_loss(lc, lv, ls, b["answer"], mil)
    model.zero_grad(set_to_none=False)
    loss.backward()
    torch.cuda.synchronize()
    return {n: params[n].grad.detach().cpu().double().clone() for n in NAMES}, lc.detach().cpu()


def cpu_grads(model, b, dtype):
    torch.set_default_dtype(dtype)
    try:
        params = dict(model.named_parameters())
        P = {n: p.detach().cpu().to(dtype).clone().requires_grad_(n in NAMES)
             for n, p in params.items()}
        inp = {k: (v.cpu().to(dtype) if v.is_floating_point() else v.cpu()) for k, v in b.items()}
        t0 = time.perf_counter()
        rc, rv, rs, rmil, _ = O.attmodel_forward(P, inp, decMask=True)
        rloss, _ = O.train_loss(rc, rv, rs, inp["answer"], rmil)
        rloss.backward()
        print(f"  oracle {dtype}: {time.perf_counter() - t0:.1f} s", flush=True)
        return {n: P[n].grad.double() for n in NAMES}, rc.detach()
    finally:
        torch.set_default_dtype(torch.float32)


def install_filter(pred):
    """Run the x6-eligible launches matching pred on the native kernel (diagnostics)."""
    from savqa_amd import ops
    orig = ops.gemm if not hasattr(ops.gemm, "_orig") else ops.gemm._orig

    def gemm(*a, **kw):
        prec = ops._prec if kw.get("prec") is None else kw["prec"]
        if prec == 6 and pred(a, kw):
            kw["prec"] = 0
        return orig(*a, **kw)
    gemm._orig = orig
    ops.gemm = gemm


def lay(a, kw):
    return ("T" if kw.get("a_trans") else "N") + ("T" if kw.get("b_trans") else "N")


FILTERS = {
    "NT": lambda a, kw: lay(a, kw) == "NT",
    "NN": lambda a, kw: lay(a, kw) == "NN",
    "TN": lambda a, kw: lay(a, kw) == "TN",
    "gather": lambda a, kw: kw.get("a_rows") is not None or kw.get("b_rows") is not None,
    "cgroup": lambda a, kw: bool(kw.get("c_group")),
    "mask": lambda a, kw: kw.get("mask") is not None,
    "resid": lambda a, kw: kw.get("resid") is not None,
}


def main():
    torch.set_num_threads(min(32, os.cpu_count() or 1))
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.utils import init_params_
    model = AttModel(None, 512, 1024, 914, 40, 450, 49, 6, 8, 0.0, 0.1, 311, True, device="cuda",
                     init=False)  # the test's model fixture
    seed = int(os.environ.get("SEED", "0"))
    init_params_(model, seed=11 + seed)
    g = torch.Generator(device="cuda").manual_seed(12 + seed)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if n.endswith(".gamma"):
                p.normal_(1.0, 0.2, generator=g)
            elif n.endswith(".beta"):
                p.normal_(0.0, 0.2, generator=g)
    from savqa_amd.data import synthetic_batch
    b = synthetic_batch(256, Nv=36, Ns=59, seed=2024 + seed, device="cuda")  # T._batch() at 0
    model.train()
    runs, logits = {}, {}
    for k in ("x6", "native"):
        runs["gpu_" + k], logits["gpu_" + k] = gpu_grads(model, b, k)
    for f in sys.argv[1:]:  # x6 with the launches of filter f on the native kernel
        install_filter(FILTERS[f])
        runs["no_" + f], logits["no_" + f] = gpu_grads(model, b, "x6")
        install_filter(lambda a, kw: False)
    if os.environ.get("PERTURB"):  # native fp32 on region features moved by <= 1 ulp
        gen = torch.Generator(device="cuda").manual_seed(99)
        bp = dict(b)
        u = torch.randint(-1, 2, b["vis_fea"].shape, generator=gen, device="cuda").float()
        bp["vis_fea"] = b["vis_fea"] * (1 + u * 2.0 ** -24)
        runs["native_1ulp"], logits["native_1ulp"] = gpu_grads(model, bp, "native")
    if os.environ.get("WPERTURB"):  # both kernels on every weight moved by <= 1 ulp
        params = dict(model.named_parameters())
        saved = {n: p.detach().clone() for n, p in params.items()}
        gen = torch.Generator(device="cuda").manual_seed(98)
        with torch.no_grad():
            for n, p in params.items():
                u = torch.randint(-1, 2, p.shape, generator=gen, device="cuda").float()
                p.mul_(1 + u * 2.0 ** -24)
        for k in ("native", "x6"):
            runs[k + "_w1ulp"], logits[k + "_w1ulp"] = gpu_grads(model, b, k)
        with torch.no_grad():
            for n, p in params.items():
                p.copy_(saved[n])
    if not os.environ.get("NO_CPU32"):
        runs["cpu_fp32"], logits["cpu_fp32"] = cpu_grads(model, b, torch.float32)
    ref, lref = cpu_grads(model, b, torch.float64)
    print("logits max-rel vs fp64:", {k: f"{T._rel(v, lref):.2e}" for k, v in logits.items()})
    print(f"{'gradient':52s} " + " ".join(f"{k:>10s}" for k in runs))
    for n in NAMES:
        errs = [T._frob(runs[k][n], ref[n]) for k in runs]
        print(f"{n:52s} " + " ".join(f"{e:10.2e}" for e in errs))


if __name__ == "__main__":
    main()
