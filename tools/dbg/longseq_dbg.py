import sys, os
sys.path.insert(0, os.getcwd())
import torch
from oracle import savqa_oracle as O
from savqa_amd.AttModel_x3 import AttModel
from savqa_amd.data import model_args, synthetic_batch
from savqa_amd.loss import smoothed_loss
from savqa_amd.optim import Adam


def rel(a, b):
    a = a.detach().cpu().double(); b = b.detach().cpu().double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def run(d, H, L, Nv, Ns, B, flash):
    os.environ["SAVQA_ATTN_FLASH"] = "1" if flash else "0"
    Hm, C, Lq = 128, 40, 14
    m = AttModel(None, d, Hm, C, 16, 460, 120, L, H, 0.0, 0.0, 2, True, device="cuda", init=False)
    gen = torch.Generator(device="cuda").manual_seed(17)
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
    P = {n: q.detach().cpu().clone().requires_grad_(True) for n, q in m.named_parameters()}
    batch = synthetic_batch(B, Nv=Nv, Lq=Lq, Ns=Ns, topN=5, num_classes=C, seed=29, device="cuda")
    lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
    loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
    opt = Adam(m, lr=1e-4); opt.zero_grad(); loss.backward(); torch.cuda.synchronize()
    inp = {k: v.cpu() for k, v in batch.items()}
    P64 = {k: v.detach().double().requires_grad_(True) for k, v in P.items()}
    inp64 = {k: (v.double() if v.is_floating_point() else v) for k, v in inp.items()}
    torch.set_default_dtype(torch.float64)
    rc, rv, rs, rmil, _ = O.attmodel_forward(P64, inp64, decMask=True, num_blocks=L, h=H)
    rloss, _ = O.train_loss(rc, rv, rs, inp64["answer"], rmil)
    rloss.backward()
    torch.set_default_dtype(torch.float32)
    rc2, rv2, rs2, rmil2, _ = O.attmodel_forward(P, inp, decMask=True, num_blocks=L, h=H)
    rl2, _ = O.train_loss(rc2, rv2, rs2, inp["answer"], rmil2)
    rl2.backward()
    params = dict(m.named_parameters())
    print(f"d={d} H={H} Nv={Nv} Ns={Ns} flash={flash}: logits gpu-vs-f64 {rel(ls, rs):.2e} cpu32-vs-f64 {rel(rs2, rs):.2e}")
    for n in ("att_syb.syb_positional_encoding.lookup_table", "att_syb.syb_mlp2.weight",
              "att_syb.enc_self_attention_0.Q_proj.0.weight", "att_syb.enc_feed_forward_0.conv1.0.weight",
              "att_syb.enc_self_attention_1.V_proj.0.weight"):
        print(f"   {n}: gpu-vs-f64 {rel(params[n].grad, P64[n].grad):.2e}  cpu32-vs-f64 {rel(P[n].grad, P64[n].grad):.2e}")


for cfg in [(1024, 16, 2, 100, 435, 2, True), (256, 4, 2, 100, 435, 2, True), (1024, 16, 2, 100, 100, 2, False),
            (1024, 16, 2, 100, 100, 2, True)]:
    run(*cfg)
