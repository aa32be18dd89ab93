#!/usr/bin/env python
"""Conditioning of a relation golden case: the oracle run in fp64 on the golden's inputs,
compared with the reference's fp32 outputs stored in the golden (tests/golden/<case>.npz).
Per trained gradient: max |fp64 - ref32| / scale over the sampled elements, with the scale of
tests/test_relation_gpu.py. Writes tests/golden/<case>_fp64dev.json, the per-parameter fp32
rounding floor the GPU parity test allows beside its 1e-3 bar. CPU only (test
infrastructure: imports the oracle).  usage: python tools/rel_fp64_check.py full_rel_big"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import hashfill  # noqa: E402
from oracle import savqa_oracle as O  # noqa: E402

INPUTS = ("vis_fea", "vis_mask", "q_ipt", "q_mask", "q_graph", "macro_ipt", "macro_mask",
          "macro_graph", "macro_obj_loc", "micro_positive_obj", "micro_negative_obj",
          "micro_obj_mask", "micro_positive_rel", "micro_negative_rel",
          "micro_positive_rel_loc", "micro_negative_rel_loc", "answer")


class HashParams64(hashfill.HashParams):
    def __missing__(self, name):
        shape = self.shapes[name]
        t = torch.from_numpy(hashfill.param_value(name, shape).astype(np.float64))
        t.requires_grad_(self.requires_grad)
        self[name] = t
        return t


def main(case):
    torch.set_default_dtype(torch.float64)
    g = np.load(os.path.join(ROOT, "tests", "golden", f"{case}.npz"))
    geo = {k: int(g[k]) for k in ("hidden_mil", "maxlen") if k in g}
    P = HashParams64(requires_grad=True, num_relations=int(g["num_relations"]), **geo)
    inp = {}
    for k in INPUTS:
        a = torch.from_numpy(g[k])
        inp[k] = a.double() if a.is_floating_point() else a
    lc, lv, ls, mil, mil_rel = O.attmodel_forward(P, inp, decMask=True, only_obj=False)
    loss, _ = O.train_loss(lc, lv, ls, inp["answer"], mil, mil_nce_rel=mil_rel)
    loss.backward()
    out = {}
    for n in [str(x) for x in g["grad_names"]]:
        flat = P[n].grad.reshape(-1).detach().numpy()
        ref = g[f"g:{n}:val"].astype(np.float64)
        idx = g[f"g:{n}:idx"]
        scale = max(np.abs(ref).max(), float(g[f"g:{n}:abssum"]) / flat.size, 1e-20)
        out[n] = float(np.abs(flat[idx] - ref).max() / scale)
    worst = sorted(out.items(), key=lambda kv: -kv[1])[:8]
    for n, e in worst:
        print(f"{e:.3e}  {n}")
    path = os.path.join(ROOT, "tests", "golden", f"{case}_fp64dev.json")
    with open(path, "w") as f:
        json.dump({"case": case, "note": "max |oracle fp64 - reference fp32| / scale per gradient "
                   "(tools/rel_fp64_check.py)", "dev": out}, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "full_rel_big")
