"""GPU debug: the relation branch's updated macro features (engine s.macro after
rel_macro_fwd) against the oracle's mil_nce_forward in fp64, per node row."""
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
from savqa_amd import ops  # noqa: E402
from savqa_amd.AttModel_x3 import AttModel  # noqa: E402

cap = {}
orig = ops.rel_macro_fwd


def rel_macro_fwd(*args):
    orig(*args)
    cap["macro"] = args[-1].detach().clone()
    cap["args"] = args


ops.rel_macro_fwd = rel_macro_fwd
g = np.load(os.path.join(ROOT, "tests", "golden", f"{case}.npz"))
hm = int(g["hidden_mil"]) if "hidden_mil" in g else 1024
maxlen = int(g["maxlen"]) if "maxlen" in g else 450
m = AttModel(None, 512, hm, 914, 40, maxlen, 49, int(g["num_blocks"]), 8, 0.0, 0.0,
             int(g["num_relations"]), False, device="cuda", init=False)
with torch.no_grad():
    for n, p in m.named_parameters():
        p.copy_(torch.from_numpy(hashfill.param_value(n, tuple(p.shape))))
t = {k: torch.from_numpy(g[k]).cuda() for k in INPUTS + ("answer",)}
with torch.no_grad():
    m(*[t[k] for k in INPUTS], decMask=True, mcb=False)
torch.cuda.synchronize()
gm = cap["macro"].double()


class P64(hashfill.HashParams):
    def __missing__(self, name):
        v = torch.from_numpy(hashfill.param_value(name, self.shapes[name]).astype(np.float64)).cuda()
        self[name] = v
        return v


torch.set_default_device("cuda")
torch.set_default_dtype(torch.float64)
geo = {k: int(g[k]) for k in ("hidden_mil", "maxlen") if k in g}
P = P64(num_relations=int(g["num_relations"]), **geo)
inp = {k: (torch.from_numpy(g[k]).cuda().double() if g[k].dtype.kind == "f" else torch.from_numpy(g[k]).cuda())
       for k in INPUTS}
rel = (inp["micro_positive_rel"], inp["micro_negative_rel"], inp["micro_positive_rel_loc"],
       inp["micro_negative_rel_loc"])
with torch.no_grad():
    new_macro, mil_obj, mil_rel = O.mil_nce_forward(
        P, inp["vis_fea"], inp["macro_ipt"], inp["macro_obj_loc"], inp["micro_positive_obj"],
        inp["micro_negative_obj"], inp["micro_obj_mask"], rel=rel)
B, Ns, H = new_macro.shape
ref = new_macro.reshape(B * Ns, H)
gm = torch.relu(gm @ P["MIL_NCE.ipt_mlp.0.weight"].t() + P["MIL_NCE.ipt_mlp.0.bias"])
d = (gm - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-30)
print(case, "macro rows", B * Ns, "max row rel", float(d.max()), "median", float(d.median()))
top = torch.argsort(d, descending=True)[:12]
for i in top.tolist():
    print(case, "row", i, "b", i // Ns, "node", i % Ns, "rel %.3e" % float(d[i]), "norm %.3e" % float(ref[i].norm()))
