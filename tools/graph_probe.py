#!/usr/bin/env python
"""Experiment: one bench workload's training step eager vs captured into a hipGraph and
replayed (torch.cuda.graph), same process, N = 1. Measures whether the host's launches limit
the step (if replay is faster, they do). Not a training loop: the replay repeats Adam's bias
correction and the dropout seed of the captured step.  usage: python tools/graph_probe.py WL"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "rel"
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    from savqa_amd.utils import init_params_
    W = bench.WORKLOADS[wl]
    B = W["batch"]
    dev = "cuda"
    model = AttModel(None, W["d"], W.get("hm", 1024), 914, 40, W.get("maxlen", 450), 49, 6,
                     W["H"], 0.0, 0.1, 311, not W.get("rel", False), device=dev, init=False,
                     gemm_precision=W.get("prec", "fp32"))
    init_params_(model, seed=0)
    model.train()
    # the relation branch's per-step bounds check reads a device flag on the host, which a
    # capture cannot contain; the probe's inputs are valid, so it is skipped here
    model._check_relation_locs = lambda *a, **k: None
    opt = Adam(model, lr=1e-4)
    if W.get("rel"):
        from savqa_amd.data import model_args_rel, synthetic_relation_batch
        batch = synthetic_relation_batch(B, Nv=W["Nv"], seed=1234, device=dev)
        margs = model_args_rel(batch)
    else:
        batch = synthetic_batch(B, Nv=W["Nv"], Ns=W["Ns"], seed=1234, device=dev)
        margs = model_args(batch)

    def step():
        lc, lv, ls, mil, mil_rel = model(*margs, decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil, with_milnce=True,
                                mil_nce_rel=mil_rel)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()

    def timed(fn, n=10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n

    te = timed(step)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    tg = timed(g.replay)
    te2 = timed(step)
    print(f"{wl}: eager {te * 1e3:.2f} / {te2 * 1e3:.2f} ms/step, graph replay {tg * 1e3:.2f} "
          f"ms/step ({B / tg:.1f} vs {B / te:.1f} samples/s)", flush=True)


if __name__ == "__main__":
    main()
