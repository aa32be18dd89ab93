#!/usr/bin/env python
"""GEMM-level audit of the x6 kernel on a real cfg-2 training step: every 128x128-tile fp32
GEMM the step launches is re-run on its own operands (geometry only: layout, leading
dimensions, row gathers; no epilogue) with the native fp32 kernel (prec 0) and the x6 kernel
(prec 6), and both are compared with an fp64 product of the same operands. Prints the launches
where x6 lands furthest from fp64 relative to native.  usage: SEED=0 python tools/x6_audit.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from savqa_amd import engine, ops  # noqa: E402
from savqa_amd.data import model_args, synthetic_batch  # noqa: E402
from savqa_amd.loss import smoothed_loss  # noqa: E402

RECS = []


def operand(P, rows, cols, ld, trans, idx):
    """[rows, cols] fp64 matrix of A(m, k) = trans ? P[ri(k)*ld + m] : P[ri(m)*ld + k]."""
    # the kernel's view: the storage from P's data pointer on (P may be a strided slice)
    n = P.untyped_storage().nbytes() // P.element_size() - P.storage_offset()
    flat = P.as_strided((n,), (1,))
    if not trans:
        r = idx if idx is not None else torch.arange(rows, device=P.device)
        ix = r[:, None] * ld + torch.arange(cols, device=P.device)[None, :]
    else:
        r = idx if idx is not None else torch.arange(cols, device=P.device)
        ix = r[None, :] * ld + torch.arange(rows, device=P.device)[:, None]
    if int(ix.max()) >= n or int(ix.min()) < 0:
        raise IndexError("operand geometry outside its storage")
    return flat[ix].double()


def audit(orig, A, B, Cm, M, N, K, kw, xprec=6):
    lda, ldb = kw["lda"], kw["ldb"]
    at, bt = bool(kw.get("a_trans")), bool(kw.get("b_trans"))
    ar, br = kw.get("a_rows"), kw.get("b_rows")
    Am = operand(A, M, K, lda, at, ar)                 # A(m, k)
    Bm = operand(B, N, K, ldb, not bt, br)  # B(k, n) as [n, k]
    ref = Am @ Bm.t()
    errs, stats = {}, {}
    for prec in (0, xprec):  # xprec 5: the two-level form (decoder K/V projection)
        out = torch.zeros(M, N, device=A.device)
        orig(A, B, out, M, N, K, lda=lda, ldb=ldb, ldc=N, a_trans=at, b_trans=bt, a_rows=ar,
             b_rows=br, atomic=at, split_k=-1 if at else 1, prec=prec)
        torch.cuda.synchronize()
        e = out.double() - ref
        errs[6 if prec else 0] = float(e.abs().max() / ref.abs().max().clamp_min(1e-300))
        # bias: error along the sign of the exact value (toward-zero errors give < 0), rms
        stats[6 if prec else 0] = (float((e * ref.sign()).sum() / e.abs().sum().clamp_min(1e-300)),
                       float(e.norm() / ref.norm().clamp_min(1e-300)))
    lay = ("T" if at else "N") + ("T" if bt else "N")
    tag = f"{lay} {M}x{N}x{K}" + (" ar" if ar is not None else "") + (" br" if br is not None else "") \
        + (" two-level" if xprec == 5 else "")
    amax = float(Am.abs().max())
    amin = float(Am[Am != 0].abs().min()) if bool((Am != 0).any()) else 0.0
    bmax = float(Bm.abs().max())
    bmin = float(Bm[Bm != 0].abs().min()) if bool((Bm != 0).any()) else 0.0
    RECS.append((errs[6] / max(errs[0], 1e-30), errs[0], errs[6], tag, amax, amin, bmax, bmin,
                 stats[0], stats[6]))


def main():
    seed = int(os.environ.get("SEED", "0"))
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.utils import init_params_
    model = AttModel(None, 512, 1024, 914, 40, 450, 49, 6, 8, 0.0, 0.1, 311, True, device="cuda",
                     init=False)
    init_params_(model, seed=11 + seed)
    g = torch.Generator(device="cuda").manual_seed(12 + seed)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if n.endswith(".gamma"):
                p.normal_(1.0, 0.2, generator=g)
            elif n.endswith(".beta"):
                p.normal_(0.0, 0.2, generator=g)
    b = synthetic_batch(256, Nv=36, Ns=59, seed=2024 + seed, device="cuda")
    engine.FP32_GEMM = "x6"
    orig = ops.gemm

    def hooked(A, B, Cm, M, N, K, **kw):
        prec = ops._prec if kw.get("prec") is None else kw["prec"]
        if prec in (5, 6) and M * N * K >= 10 ** 8 and min(M, N) >= 128:
            torch.cuda.synchronize()
            audit(orig, A, B, Cm, M, N, K, kw, prec)
        return orig(A, B, Cm, M, N, K, **kw)
    ops.gemm = hooked
    model.train()
    lc, lv, ls, mil, _ = model(*model_args(b), decMask=True, mcb=False)
    loss, _ = smoothed_loss(lc, lv, ls, b["answer"], mil)
    model.zero_grad(set_to_none=False)
    loss.backward()
    torch.cuda.synchronize()
    ops.gemm = orig
    RECS.sort(key=lambda r: -r[0])
    print(f"{len(RECS)} launches audited; worst x6/native error ratios:")
    print(f"{'ratio':>7s} {'native':>9s} {'x6':>9s}  launch  |A| max/min  |B| max/min")
    for r in RECS[:25]:
        print(f"{r[0]:7.2f} {r[1]:9.2e} {r[2]:9.2e}  {r[3]}  {r[4]:.2e}/{r[5]:.2e}  {r[6]:.2e}/{r[7]:.2e}"
              f"  bias {r[8][0]:+.2f}/{r[9][0]:+.2f}  rms {r[8][1]:.1e}/{r[9][1]:.1e}")
    import statistics as st
    print("median bias native / x6:", st.median(r[8][0] for r in RECS), st.median(r[9][0] for r in RECS))
    print("median rms  native / x6:", st.median(r[8][1] for r in RECS), st.median(r[9][1] for r in RECS))


if __name__ == "__main__":
    main()
