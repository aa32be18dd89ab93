"""GPU debug: every trained gradient of the HIP model against the oracle run in fp64 on the
same device, for a relation golden case (inputs from tests/golden/<case>.npz).
usage: python tools/dbg/rel_big_cmp.py CASE"""
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
from savqa_amd.AttModel_x3 import AttModel  # noqa: E402
from savqa_amd.loss import smoothed_loss  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", f"{case}.npz"))
hm = int(g["hidden_mil"]) if "hidden_mil" in g else 1024
maxlen = int(g["maxlen"]) if "maxlen" in g else 450
m = AttModel(None, 512, hm, 914, 40, maxlen, 49, int(g["num_blocks"]), 8, 0.0, 0.0,
             int(g["num_relations"]), False, device="cuda", init=False)
with torch.no_grad():
    for n, p in m.named_parameters():
        p.copy_(torch.from_numpy(hashfill.param_value(n, tuple(p.shape))))
m.train()
t = {k: torch.from_numpy(g[k]).cuda() for k in INPUTS + ("answer",)}
lc, lv, ls, mil, mil_rel = m(*[t[k] for k in INPUTS], decMask=True, mcb=False)
loss, _ = smoothed_loss(lc, lv, ls, t["answer"], mil, mil_nce_rel=mil_rel)
m.zero_grad(set_to_none=False)
loss.backward()
gpu = {n: p.grad.detach().double() for n, p in m.named_parameters() if p.grad is not None}


class P64(hashfill.HashParams):
    def __missing__(self, name):
        v = torch.from_numpy(hashfill.param_value(name, self.shapes[name]).astype(np.float64))
        v = v.cuda().requires_grad_(True)
        self[name] = v
        return v


torch.set_default_device("cuda")
torch.set_default_dtype(torch.float64)
geo = {k: int(g[k]) for k in ("hidden_mil", "maxlen") if k in g}
P = P64(requires_grad=True, num_relations=int(g["num_relations"]), **geo)
inp = {}
for k in INPUTS + ("answer",):
    a = torch.from_numpy(g[k]).cuda()
    inp[k] = a.double() if a.is_floating_point() else a
r = O.attmodel_forward(P, inp, decMask=True, only_obj=False)
l64, _ = O.train_loss(r[0], r[1], r[2], inp["answer"], r[3], mil_nce_rel=r[4])
l64.backward()
print(case, "loss gpu", float(loss), "fp64", float(l64))
rows = []
for n, gg in gpu.items():
    if n not in P or P[n].grad is None:
        continue
    ref = P[n].grad.detach()
    d = (gg - ref)
    sc = ref.abs().max().clamp_min(1e-30)
    fro = float(d.norm() / ref.norm().clamp_min(1e-30))
    mx = float(d.abs().max() / sc)
    if ref.dim() == 2:
        rr = d.norm(dim=1) / ref.norm(dim=1).clamp_min(1e-30 + 1e-6 * float(ref.norm(dim=1).max()))
        wr = int(rr.argmax())
        rows.append((fro, mx, float(rr.max()), wr, n))
    else:
        rows.append((fro, mx, 0.0, -1, n))
rows.sort(reverse=True)
for x in rows[:40]:
    print(case, "fro %.2e max %.2e rowrel %.2e row %d %s" % x)
