# CPU only: fp32 vs fp64 oracle at d=1024, T=449 (position-table gradient conditioning)
import os
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import torch
from oracle import savqa_oracle as O
from savqa_amd.AttModel_x3 import AttModel
from savqa_amd.data import synthetic_batch
torch.manual_seed(0)
d,H,L,Nv,Ns,B = 1024,16,2,100,435,2
Hm, C, Lq = 128, 40, 14
m = AttModel(None, d, Hm, C, 16, 460, 120, L, H, 0.0, 0.0, 2, True, device="meta", init=False)
shapes = {n: p.shape for n, p in m.named_parameters()}
gen = torch.Generator().manual_seed(17)
P = {}
for n, shp in shapes.items():
    leaf = n.rsplit(".", 1)[-1]
    t = torch.empty(shp)
    if leaf == "gamma": t.uniform_(0.8, 1.2, generator=gen)
    elif len(shp) == 1: t.uniform_(-0.2, 0.2, generator=gen)
    else:
        b = 1.0 / shp[-1] ** 0.5; t.uniform_(-b, b, generator=gen)
    P[n] = t.requires_grad_(True)
inp = synthetic_batch(B, Nv=Nv, Lq=Lq, Ns=Ns, topN=5, num_classes=C, seed=29, device="cpu")
P64 = {k: v.detach().double().requires_grad_(True) for k, v in P.items()}
inp64 = {k: (v.double() if v.is_floating_point() else v) for k, v in inp.items()}
def go(PP, ii, dt):
    torch.set_default_dtype(dt)
    rc, rv, rs, rmil, _ = O.attmodel_forward(PP, ii, decMask=True, num_blocks=L, h=H)
    rl, _ = O.train_loss(rc, rv, rs, ii["answer"], rmil)
    rl.backward()
    torch.set_default_dtype(torch.float32)
go(P, inp, torch.float32); go(P64, inp64, torch.float64)
n = "att_syb.syb_positional_encoding.lookup_table"
a, b = P[n].grad.double(), P64[n].grad
err = (a - b).abs().max(1).values
mag = b.abs().max(1).values
top = err.argsort(descending=True)[:10]
print("max|ref|", float(b.abs().max()))
for t in top.tolist():
    print(t, f"err {float(err[t]):.3e} rowmax {float(mag[t]):.3e}")
# decoder cross-attention weights of the syb stack: which keys dominate?
import torch.nn.functional as F
store = {}
orig = O.graph_mha
def spy(P_, pre, queries, keys, values, graph, h=8, return_att=False):
    out, att = orig(P_, pre, queries, keys, values, graph, h, True)
    store[pre] = att.detach()
    return (out, att) if return_att else out
O.graph_mha = spy
with torch.no_grad():
    O.attmodel_forward(P, inp, decMask=True, num_blocks=L, h=H)
for k, att in store.items():
    if "dec_vanilla" in k and "att_syb" in k:
        mx, am = att[:, 0, :].max(-1)
        print(k, "argmax keys", am.tolist()[:16], "max n", [round(float(v), 4) for v in mx[:16]])
