"""GPU debug: every key-tiled attention call of the model on a relation golden case, checked
in place against fp64 and fp32 torch restatements of the same call (tests/test_kernels_gpu
_attn_ref) -- which call, if any, is less accurate than torch-fp32.
usage: python tools/dbg/rel_big_attn.py CASE"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import hashfill  # noqa: E402
from test_relation_gpu import INPUTS  # noqa: E402
from tests.test_kernels_gpu import _attn_ref  # noqa: E402

case = sys.argv[1]
torch.backends.cuda.matmul.allow_tf32 = False
from savqa_amd import ops  # noqa: E402
from savqa_amd.AttModel_x3 import AttModel  # noqa: E402
from savqa_amd.loss import smoothed_loss  # noqa: E402

orig_bwd = ops.gattn_bwd_flash
calls = []


def fro(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-300))


def view(t, rows, ld, cols):
    return torch.as_strided(t, (rows, cols), (ld, 1))


def bwd(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H, dout, lddo, stats, dq, lddq,
        dk_, lddk, dv, lddv, dk=64):
    orig_bwd(q, ldq, k, ldk, v, ldv, G, kflag, qflag, B, Tq, Tk, H, dout, lddo, stats, dq, lddq,
             dk_, lddk, dv, lddv, dk)
    torch.cuda.synchronize()
    D = H * dk
    Q = view(q, B * Tq, ldq, D).reshape(B, Tq, D)
    K = view(k, B * Tk, ldk, D).reshape(B, Tk, D)
    V = view(v, B * Tk, ldv, D).reshape(B, Tk, D)
    dO = view(dout, B * Tq, lddo, D).reshape(B, Tq, D)
    Gm = G.reshape(B, Tq, Tk)
    res = {}
    for nm, dt in (("f64", torch.float64), ("f32", torch.float32)):
      with torch.enable_grad():
        Qr = Q.detach().to(dt).clone().requires_grad_(True)
        Kr = K.detach().to(dt).clone().requires_grad_(True)
        Vr = V.detach().to(dt).clone().requires_grad_(True)
        o, _ = _attn_ref(Qr, Kr, Vr, Gm.to(dt), kflag.reshape(B, Tk).to(dt),
                         qflag.reshape(B, Tq).to(dt), h=H)
        gq, gk, gv = torch.autograd.grad((o * dO.detach().to(dt)).sum(), (Qr, Kr, Vr))
        res[nm] = (gq * (Qr > 0), gk * (Kr > 0), gv * (Vr > 0))
    ours = (view(dq, B * Tq, lddq, D).reshape(B, Tq, D), view(dk_, B * Tk, lddk, D).reshape(B, Tk, D),
            view(dv, B * Tk, lddv, D).reshape(B, Tk, D))
    line = f"bwd Tq={Tq} Tk={Tk} H={H}:"
    for i, nm in enumerate(("dQ", "dK", "dV")):
        line += f" {nm} ours {fro(ours[i], res['f64'][i]):.1e} t32 {fro(res['f32'][i], res['f64'][i]):.1e}"
    calls.append(line)


ops.gattn_bwd_flash = bwd

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
torch.cuda.synchronize()
for c in calls:
    print(case, c)
