"""GPU debug: the graphs the engine hands to every key-tiled attention call against the
oracle's build_graphs (AttModel_x3.py:229-247) on a relation golden case."""
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
from savqa_amd import ops  # noqa: E402
from savqa_amd.AttModel_x3 import AttModel  # noqa: E402

calls = []
orig = ops.gattn_fwd_flash


def fwd(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H, o, ldo, stats, dk=64):
    orig(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H, o, ldo, stats, dk)
    calls.append((G.reshape(-1)[:B * Tq * Tk].reshape(B, Tq, Tk).detach().cpu().clone(),
                  kflag.reshape(-1)[:B * Tk].detach().cpu().clone(),
                  qflag.reshape(-1)[:B * Tq].detach().cpu().clone(), Tq, Tk))


ops.gattn_fwd_flash = fwd
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
gi = {k: torch.from_numpy(g[k]) for k in INPUTS}
gd, gg, dm = O.build_graphs(gi["macro_mask"], gi["q_mask"], gi["q_graph"], gi["macro_graph"], True)
print(case, "flash fwd calls", len(calls))
for n, (G, kf, qf, Tq, Tk) in enumerate(calls):
    if Tq == 1:
        ref = dm
    else:
        ref = gd if n < 2 else gg
    diff = (G != ref.float())
    line = f"call {n} Tq={Tq} Tk={Tk}: G mismatches {int(diff.sum())}"
    if diff.any():
        idx = diff.nonzero()[:5].tolist()
        line += f" first {idx}"
    line += f" kflag zeros {int((kf == 0).sum())} qflag zeros {int((qf == 0).sum())}"
    print(case, line)
