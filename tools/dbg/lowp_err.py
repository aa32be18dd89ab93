"""Error of the low-precision modes against the CPU fp32 oracle (prints, no asserts):
logits max-rel error, argmax agreement, loss, gradient cosines. B=48, L=2 model."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from oracle import savqa_oracle as O  # noqa: E402


def rel(a, b):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def cos(a, b):
    a, b = a.detach().cpu().double().reshape(-1), b.detach().cpu().double().reshape(-1)
    return float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-30))


def main():
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    dev = "cuda"
    d, H, L, Hm, C = 512, 8, int(os.environ.get("L", 2)), 256, 100
    Bn = int(os.environ.get("B", 48))
    m = AttModel(None, d, Hm, C, 16, 100, 40, L, H, 0.0, 0.0, 2, True, device=dev, init=False)
    gen = torch.Generator(device=dev).manual_seed(23)
    with torch.no_grad():
        for n, prm in m.named_parameters():
            leaf = n.rsplit(".", 1)[-1]
            if leaf == "gamma":
                prm.uniform_(0.8, 1.2, generator=gen)
            elif prm.dim() == 1:
                prm.uniform_(-0.2, 0.2, generator=gen)
            else:
                bound = 1.0 / prm.shape[-1] ** 0.5
                prm.uniform_(-bound, bound, generator=gen)
    m.train()
    batch = synthetic_batch(Bn, Nv=36, Lq=14, Ns=59, topN=5, num_classes=C, seed=31, device=dev)
    P0 = {n: q.detach().cpu().clone() for n, q in m.named_parameters()}
    for prec in sys.argv[1:] or ["fp32", "bf16", "fp8"]:
        with torch.no_grad():
            for n, q in m.named_parameters():
                q.copy_(P0[n])
        m._engine.gemm_precision = prec
        inp = {k: v.cpu() for k, v in batch.items()}
        if prec == "fp8":  # the oracle sees the dequantised features
            from savqa_amd import ops
            R = Bn * 36
            q8 = torch.empty(R, 2048, dtype=torch.uint8, device=dev)
            s8 = torch.empty(R, 64, dtype=torch.uint8, device=dev)
            ops.quant_fp8(batch["vis_fea"].reshape(R, 2048), R, 2048, 2048, q8, 2048, s8, 64)
            deq = q8.view(torch.float8_e4m3fn).float().cpu() * torch.pow(
                2.0, s8.cpu().float() - 127).repeat_interleave(32, 1)
            inp["vis_fea"] = deq.reshape(Bn, 36, 2048)
        P = {n: q.clone().requires_grad_(True) for n, q in P0.items()}
        rc, rv, rs, rmil, _ = O.attmodel_forward(P, inp, decMask=True, num_blocks=L, h=H)
        rloss, _ = O.train_loss(rc, rv, rs, inp["answer"], rmil)
        rloss.backward()
        args = model_args(batch)
        lc, lv, ls, mil, _ = m(*args, decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
        opt = Adam(m, lr=1e-4)
        opt.zero_grad()
        loss.backward()
        torch.cuda.synchronize()
        params = dict(m.named_parameters())
        out = [prec]
        for a, b, nm in ((lc, rc, "cat"), (lv, rv, "vis"), (ls, rs, "syb")):
            agree = float((a.detach().cpu().argmax(-1) == b.argmax(-1)).float().mean())
            out.append(f"{nm} rel {rel(a, b):.2e} argmax {agree:.3f}")
        out.append(f"loss {abs(float(loss) - float(rloss)) / abs(float(rloss)):.2e} "
                   f"mil {abs(float(mil) - float(rmil)):.2e}")
        errs = sorted((float((params[n].grad.cpu().double() - P[n].grad.double()).norm()
                             / P[n].grad.double().norm()), n) for n in P
                      if P[n].grad is not None and params[n].grad is not None
                      and P[n].grad.abs().sum() > 0 and not n.endswith("K_proj.0.bias"))
        # the same oracle under torch autocast bf16 on the GPU: what stock AMP gets
        Pa = {n: q.clone().to(dev).requires_grad_(True) for n, q in P0.items()}
        inpa = {k: v.to(dev) for k, v in inp.items()}
        with torch.device(dev), torch.autocast("cuda", dtype=torch.bfloat16):
            ac, av, as_, amil, _ = O.attmodel_forward(Pa, inpa, decMask=True, num_blocks=L, h=H)
        with torch.device(dev):
            aloss, _ = O.train_loss(ac.float(), av.float(), as_.float(), inpa["answer"],
                                    amil.float())
            aloss.backward()
        amp = {n: float((Pa[n].grad.cpu().double() - P[n].grad.double()).norm()
                        / P[n].grad.double().norm()) for _, n in errs}
        out.append(f"amp cat rel {rel(ac.float(), rc):.2e}")
        print(" | ".join(out), flush=True)
        for e, n in errs[::-1][:14]:
            print(f"    grad rel-norm err {e:.2e} (autocast-bf16 {amp[n]:.2e}) {n}", flush=True)


if __name__ == "__main__":
    main()
