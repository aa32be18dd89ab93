"""When does each backward phase finish? (cfg-2 train step on one GPU.)

Attaches a recording stand-in for ddp.GradReducer: every range declaration records a HIP
event on the stream that declared it, so the probe reports, relative to the start of
the backward, when the heads / visual stack / semantic stack / MIL-NCE gradients were
final and when the whole backward ended. At N > 1 the all-reduce of a phase's last
bucket can only start at its finish time, so (backward end - MIL-NCE finish) is the
window in which the MIL-NCE table's all-reduce is hidden behind the visual stack.
usage: SAVQA_BWD_ORDER=concurrent|dec|encN|syb_first python tools/tail_probe.py [--steps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    import savqa_amd  # noqa: F401
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    from savqa_amd.utils import init_params_
    dev = torch.device("cuda", 0)
    model = AttModel(None, 512, 1024, 914, 40, 450, 49, 6, 8, 0.5, 0.1, 311, True, device=dev,
                     init=False)
    init_params_(model, seed=0)
    model.train()
    opt = Adam(model, lr=1e-4)
    batch = synthetic_batch(args.batch, Nv=36, Ns=59, seed=1234, device=dev)
    margs = model_args(batch)
    b_heads, b_vis, b_syb = model._engine.region_bounds()
    n_live = model._arena.n_live

    class Probe:
        world = 1

        def __init__(self):
            self.ev = {}

        def set_rows(self, ids):
            pass

        def prepare_rows(self):
            pass

        def reduce_range(self, lo, hi, flush=False):
            if flush:
                e = torch.cuda.Event(enable_timing=True)
                e.record(torch.cuda.current_stream())
                self.ev[hi] = e

    names = {b_heads: "heads", b_vis: "vis_stack", b_syb: "syb_stack", n_live: "mil_nce"}
    rows = []
    for it in range(args.steps + 2):
        probe = Probe()
        object.__setattr__(model, "_reducer", probe)
        lc, lv, ls, mil, _ = model(*margs, decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil, with_milnce=True)
        opt.zero_grad()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        loss.backward()
        t1.record()
        opt.step()
        torch.cuda.synchronize()
        if it >= 2:
            r = {names.get(k, str(k)): round(t0.elapsed_time(e), 3) for k, e in probe.ev.items()}
            r["backward_end"] = round(t0.elapsed_time(t1), 3)
            rows.append(r)
    keys = rows[0].keys()
    mean = {k: round(sum(r[k] for r in rows) / len(rows), 3) for k in keys}
    mean["hidden_window_ms"] = round(mean["backward_end"] - mean["mil_nce"], 3)
    mean["bwd_order"] = model._engine.bwd_order
    print(json.dumps(mean))


if __name__ == "__main__":
    main()
