"""GPU debug: every fp32 savqa_gemm call of one forward+backward on a relation golden case,
checked in place against an fp64 recomputation of the descriptor (plain rows only: calls with
row gathers / scatters / grouped rows are skipped). Prints calls whose relative error exceeds
1e-5."""
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

orig = ops.gemm
stats = {"checked": 0, "skipped": 0}
bad = []


def mat(t, rows, cols, ld):
    return torch.as_strided(t, (rows, cols), (ld, 1))


def gemm(A, B, Cm, M, N, K, *, lda, ldb, ldc, a_trans=False, b_trans=False, a_rows=None,
         b_rows=None, c_rows=None, c_group=0, c_stride=0, c_offset=0, bias=None, rowvec=None,
         ldrv=0, rowvec_period=0, resid=None, ldr=0, mask=None, ldmask=0, mask_arows=False,
         rowscale=None, relu=False, alpha=1.0, beta=0.0, atomic=False, split_k=1, colsum_a=None,
         prec=None):
    kw = dict(lda=lda, ldb=ldb, ldc=ldc, a_trans=a_trans, b_trans=b_trans, a_rows=a_rows,
              b_rows=b_rows, c_rows=c_rows, c_group=c_group, c_stride=c_stride, c_offset=c_offset,
              bias=bias, rowvec=rowvec, ldrv=ldrv, rowvec_period=rowvec_period, resid=resid,
              ldr=ldr, mask=mask, ldmask=ldmask, mask_arows=mask_arows, rowscale=rowscale,
              relu=relu, alpha=alpha, beta=beta, atomic=atomic, split_k=split_k,
              colsum_a=colsum_a, prec=prec)
    if M * N * K == 0:
        return orig(A, B, Cm, M, N, K, **kw)
    torch.cuda.synchronize()
    # output rows
    mm = torch.arange(M, device=Cm.device)
    if c_rows is not None:
        crow = c_rows[:M].long()
    elif c_group:
        crow = (mm // c_group) * c_stride + (mm % c_group) + c_offset
    else:
        crow = mm
    Cfull = torch.as_strided(Cm, (int(crow.max()) + 1, N), (ldc, 1))
    C0 = Cfull.double().clone()
    cs0 = colsum_a[:M].double().clone() if colsum_a is not None else None
    orig(A, B, Cm, M, N, K, **kw)
    torch.cuda.synchronize()
    ra = a_rows[: (K if a_trans else M)].long() if a_rows is not None else None
    rb = b_rows[: (N if b_trans else K)].long() if b_rows is not None else None
    if a_trans:
        nrow = int(ra.max()) + 1 if ra is not None else K
        Ad = mat(A, nrow, M, lda).double()
        Ad = (Ad[ra] if ra is not None else Ad).t()
    else:
        nrow = int(ra.max()) + 1 if ra is not None else M
        Ad = mat(A, nrow, K, lda).double()
        Ad = Ad[ra] if ra is not None else Ad
    if b_trans:
        nrow = int(rb.max()) + 1 if rb is not None else N
        Bd = mat(B, nrow, K, ldb).double()
        Bd = (Bd[rb] if rb is not None else Bd).t()
    else:
        nrow = int(rb.max()) + 1 if rb is not None else K
        Bd = mat(B, nrow, N, ldb).double()
        Bd = Bd[rb] if rb is not None else Bd
    v = alpha * (Ad @ Bd)
    if bias is not None:
        v = v + bias[:N].double()
    if rowvec is not None:
        v = v + mat(rowvec, rowvec_period, N, ldrv).double()[mm % rowvec_period]
    if relu:
        v = v.clamp_min(0)
    if rowscale is not None:
        v = v * rowscale[:M].double().unsqueeze(1)
    if mask is not None:
        mr = a_rows[:M].long() if mask_arows else mm
        nmr = int(mr.max()) + 1
        v = v * (mat(mask, nmr, N, ldmask)[mr] > 0).double()
    if resid is not None:
        v = v + mat(resid, M, N, ldr).double()
    exp = C0.clone()
    if atomic:
        exp.index_add_(0, crow, v)
    elif beta == 1.0:
        exp[crow] = C0[crow] + v
    else:
        exp[crow] = v
    got = Cfull.double()
    touched = torch.zeros(exp.shape[0], dtype=torch.bool, device=exp.device)
    touched[crow] = True
    err = float((got[touched] - exp[touched]).norm() / exp[touched].norm().clamp_min(1e-300))
    mx = float((got[touched] - exp[touched]).abs().max() / exp[touched].abs().max().clamp_min(1e-300))
    stats["checked"] += 1
    line = (f"{'T' if a_trans else 'N'}{'T' if b_trans else 'N'} {M}x{N}x{K} atomic={atomic} "
            f"relu={relu} mask={mask is not None} resid={resid is not None} "
            f"rows={a_rows is not None},{b_rows is not None},{c_rows is not None},{c_group} "
            f"rowvec={rowvec is not None} rowscale={rowscale is not None} err {err:.1e} max {mx:.1e}")
    if colsum_a is not None:
        cexp = cs0 + Ad.sum(1)
        cerr = float((colsum_a[:M].double() - cexp).norm() / cexp.norm().clamp_min(1e-300))
        line += f" colsum {cerr:.1e}"
        err = max(err, cerr)
    if err > 1e-5 or mx > 1e-4:
        bad.append(line)


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
torch.cuda.synchronize()
print(case, stats)
for b in bad:
    print(case, "BAD", b)
