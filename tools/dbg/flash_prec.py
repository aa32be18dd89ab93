"""Precision of the key-tiled attention backward at long rows: ours vs fp64 and torch-fp32
(same chain, autograd) vs fp64, Frobenius relative errors of dQ / dK / dV / O."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tests.test_kernels_gpu import _attn_ref  # noqa: E402
from savqa_amd import ops as O  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
dev = "cuda"


def fro(a, b):
    a = a.double().cpu(); b = b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


def run(B, T, H, D, sc, vmode, gden, seed=0):
    gen = torch.Generator().manual_seed(seed)
    Q = (torch.randn(B * T, D, generator=gen) * sc).clamp_min(0)
    K = (torch.randn(B * T, D, generator=gen) * sc).clamp_min(0)
    if vmode == "similar":
        V = (1.0 + 0.01 * torch.randn(B * T, D, generator=gen)).clamp_min(0)
    else:
        V = torch.randn(B * T, D, generator=gen).clamp_min(0)
    G = (torch.rand(B, T, T, generator=gen) < gden).float()
    kf = torch.ones(B, T)
    qf = torch.ones(B, T)
    dO = torch.randn(B * T, D, generator=gen)
    Qd, Kd, Vd, Gd, dOd = (x.to(dev) for x in (Q, K, V, G, dO))
    kfd, qfd = kf.to(dev), qf.to(dev)
    out = torch.empty(B * T, D, device=dev)
    stats = torch.empty(B * H * T * 4, device=dev)
    O.gattn_fwd_flash(Qd, D, Kd, D, Vd, D, Gd, kfd, qfd, B, T, T, H, out, D, stats)
    dq = torch.empty(B * T, D, device=dev); dk = torch.empty_like(dq); dv = torch.empty_like(dq)
    O.gattn_bwd_flash(Qd, D, Kd, D, Vd, D, Gd, kfd, qfd, B, T, T, H, dOd, D, stats, dq, D, dk, D, dv, D)
    res = {}
    for name, dt in (("f64", torch.float64), ("f32", torch.float32)):
        Qr = Q.reshape(B, T, D).to(dev, dt).requires_grad_(True)
        Kr = K.reshape(B, T, D).to(dev, dt).requires_grad_(True)
        Vr = V.reshape(B, T, D).to(dev, dt).requires_grad_(True)
        o, _ = _attn_ref(Qr, Kr, Vr, Gd.to(dt), kfd.to(dt), qfd.to(dt), h=H)
        (o * dOd.view(B, T, D).to(dt)).sum().backward()
        res[name] = (o.detach(), Qr.grad * (Qr > 0), Kr.grad * (Kr > 0), Vr.grad * (Vr > 0))
    torch.cuda.synchronize()
    ref = res["f64"]
    ours = (out.view(B, T, D), dq.view(B, T, D), dk.view(B, T, D), dv.view(B, T, D))
    line = f"T={T} sc={sc} V={vmode} G={gden}: "
    for i, nm in enumerate(("O", "dQ", "dK", "dV")):
        line += f"{nm} ours {fro(ours[i], ref[i]):.1e} t32 {fro(res['f32'][i], ref[i]):.1e} | "
    # direction of the dQ error: the keys' mean per (sample, head)?
    e = (ours[1].double().cpu() - ref[1].cpu()).view(B, T, H, D // H)
    kb = K.view(B, T, H, D // H).double().mean(1, keepdim=True).expand_as(e)
    qm = (Q.view(B, T, H, D // H) > 0).double()
    kbm = kb * qm
    cos = (e * kbm).sum(-1) / (e.norm(dim=-1) * kbm.norm(dim=-1)).clamp_min(1e-300)
    line += f"cos(err, Kmean) median {float(cos.abs().median()):.3f}"
    print(line, flush=True)


for T in (211, 1313):
    for sc in (1.0, 3.0):
        for vmode in ("rand", "similar"):
            for gden in (0.3, 1.0, 0.003):
                run(2, T, 8, 512, sc, vmode, gden)
