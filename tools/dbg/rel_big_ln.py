"""GPU debug: every LayerNorm forward / backward call of one step on a relation golden case,
checked in place against fp64 (modules.py:62-65: unbiased std, eps on std)."""
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

of, ob = ops.ln_fwd, ops.ln_bwd
out = []


def ln64(z, g, b, eps=1e-8):
    mu = z.mean(-1, keepdim=True)
    sd = z.std(-1, keepdim=True)
    return g * (z - mu) / (sd + eps) + b


def ln_fwd(x, gamma, beta, y, mean, rden, std, *, r=None, z_out=None, flag=None, xscale=None,
           eps=1e-8, yb=None):
    of(x, gamma, beta, y, mean, rden, std, r=r, z_out=z_out, flag=flag, xscale=xscale, eps=eps, yb=yb)
    torch.cuda.synchronize()
    cols = gamma.numel()
    rows = x.numel() // cols
    z = x.reshape(rows, cols).double()
    if xscale is not None:
        z = z * xscale[:rows].double().unsqueeze(1)
    if r is not None:
        z = z + r.reshape(rows, cols).double()
    ref = ln64(z, gamma.double(), beta.double(), eps)
    got = y.reshape(rows, cols).double()
    e = float((got - ref).norm() / ref.norm())
    rowe = ((got - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-300))
    out.append(f"fwd rows={rows} err {e:.1e} worst row {int(rowe.argmax())} {float(rowe.max()):.1e}")


def ln_bwd(dy, z, mean, rden, std, gamma, dz, dgamma, dbeta, *, dz_add=None, dzb=None):
    torch.cuda.synchronize()
    g0, b0 = dgamma.double().clone(), dbeta.double().clone()
    ob(dy, z, mean, rden, std, gamma, dz, dgamma, dbeta, dz_add=dz_add, dzb=dzb)
    torch.cuda.synchronize()
    cols = gamma.numel()
    rows = z.numel() // cols
    with torch.enable_grad():
        zz = z.reshape(rows, cols).double().clone().requires_grad_(True)
        gg = gamma.double().clone().requires_grad_(True)
        bb = torch.zeros_like(gg).requires_grad_(True)
        yv = ln64(zz, gg, bb)
        dzr, dgr, dbr = torch.autograd.grad((yv * dy.reshape(rows, cols).double()).sum(), (zz, gg, bb))
    if dz_add is not None:
        dzr = dzr + dz_add.reshape(rows, cols).double()
    got = dz.reshape(rows, cols).double()
    e = float((got - dzr).norm() / dzr.norm().clamp_min(1e-300))
    rowe = ((got - dzr).norm(dim=1) / dzr.norm(dim=1).clamp_min(1e-300))
    eg = float((dgamma.double() - g0 - dgr).norm() / dgr.norm().clamp_min(1e-300))
    eb = float((dbeta.double() - b0 - dbr).norm() / dbr.norm().clamp_min(1e-300))
    out.append(f"bwd rows={rows} dz {e:.1e} worst row {int(rowe.argmax())} {float(rowe.max()):.1e} "
               f"dgamma {eg:.1e} dbeta {eb:.1e}")


ops.ln_fwd, ops.ln_bwd = ln_fwd, ln_bwd
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
for o in out:
    bad = any(float(x) > 1e-5 for x in o.replace(",", " ").split() if x[:1].isdigit() and "e" in x)
    print(case, ("BAD " if bad else "") + o)
