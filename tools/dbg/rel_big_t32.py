"""GPU: the oracle (plain torch fp32, hipBLASLt GEMMs) on a relation golden case, scored with
tests/test_relation_gpu.py's per-gradient metric against the reference's CPU fp32 outputs --
how far a second fp32 summation order lands from the reference at this size."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import hashfill  # noqa: E402
from oracle import savqa_oracle as O  # noqa: E402
from test_relation_gpu import INPUTS  # noqa: E402

case = sys.argv[1]
torch.backends.cuda.matmul.allow_tf32 = False
torch.set_default_device("cuda")
g = np.load(os.path.join(ROOT, "tests", "golden", f"{case}.npz"))


class PG(hashfill.HashParams):
    def __missing__(self, name):
        v = torch.from_numpy(hashfill.param_value(name, self.shapes[name])).cuda().requires_grad_(True)
        self[name] = v
        return v


geo = {k: int(g[k]) for k in ("hidden_mil", "maxlen") if k in g}
P = PG(requires_grad=True, num_relations=int(g["num_relations"]), **geo)
inp = {k: torch.from_numpy(g[k]).cuda() for k in INPUTS + ("answer",)}
r = O.attmodel_forward(P, inp, decMask=True, only_obj=False)
loss, _ = O.train_loss(r[0], r[1], r[2], inp["answer"], r[3], mil_nce_rel=r[4])
loss.backward()
worst = []
for n in [str(x) for x in g["grad_names"]]:
    flat = P[n].grad.reshape(-1).double().cpu().numpy()
    ref = g[f"g:{n}:val"].astype(np.float64)
    idx = g[f"g:{n}:idx"]
    scale = max(np.abs(ref).max(), float(g[f"g:{n}:abssum"]) / flat.size, 1e-20)
    worst.append((float(np.abs(flat[idx] - ref).max() / scale), n))
worst.sort(reverse=True)
for w in worst[:8]:
    print(case, "torch-gpu-fp32 %.3e %s" % w)
