"""GPU debug: do the decoder cross-attention gradients (dK / dV written by the key-tiled
backward) reach the K/V projection's backward GEMM unchanged? Clones every flash backward's
outputs right after the call and compares them with the same memory at each later GEMM."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import hashfill  # noqa: E402
from test_relation_gpu import INPUTS  # noqa: E402

case = sys.argv[1]
torch.backends.cuda.matmul.allow_tf32 = False
from savqa_amd import ops  # noqa: E402
from savqa_amd.AttModel_x3 import AttModel  # noqa: E402
from savqa_amd.loss import smoothed_loss  # noqa: E402

saved = []
ob, og = ops.gattn_bwd_flash, ops.gemm
events = []


def bwd(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H, dout, lddo, stats, dq, lddq,
        dk_, lddk, dv, lddv, dk=64):
    ob(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H, dout, lddo, stats, dq, lddq,
       dk_, lddk, dv, lddv, dk)
    torch.cuda.synchronize()
    D = H * dk
    for nm, t, ld, rows in (("dk", dk_, lddk, B * Tk), ("dv", dv, lddv, B * Tk), ("dq", dq, lddq, B * Tq)):
        vw = torch.as_strided(t, (rows, D), (ld, 1))
        saved.append((f"call{len(saved)//3} Tq={Tq} {nm}", vw, vw.clone()))


def check(tag):
    torch.cuda.synchronize()
    for nm, vw, cl in saved:
        d = (vw != cl)
        if d.any():
            idx = d.nonzero()[:4].tolist()
            events.append(f"{tag}: {nm} changed at {int(d.sum())} elements, first {idx}")


def gemm(A, B, Cm, M, N, K, **kw):
    check(f"before gemm {M}x{N}x{K} at={kw.get('a_trans')}")
    og(A, B, Cm, M, N, K, **kw)
    check(f"after gemm {M}x{N}x{K} at={kw.get('a_trans')}")


ops.gattn_bwd_flash = bwd
ops.gemm = gemm
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
check("end")
print(case, "flash bwd outputs tracked", len(saved))
seen = set()
for e in events:
    key = e.split(": ", 1)[1]
    if key in seen:
        continue
    seen.add(key)
    print(case, e)
