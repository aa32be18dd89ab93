"""Whole-model parity of the bf16-MFMA GEMM modes (include/savqa.h savqa_gemm_desc.prec) at a
batch large enough that the 128x128-tile GEMMs carry the model (B=48: 3504 rows per stack):
  "bf16x3" (three bf16 MFMAs per product, ~2^-16 of sum|a*b| per dot product): outputs at
    the north-star fp32 bar (logits within 1e-3 max-relative of the CPU fp32 oracle, answer
    argmax exact); weight gradients are long sums with heavy cancellation, where 2^-16 of
    the absolute sum shows up as ~4e-3 of the largest entry -- so they are held to 1e-2
    max-relative and cosine > 0.99999 (this is why fp32 products stay the default);
  "bf16" (BASELINE config 3's bf16 training: bf16 products, fp32 accumulation, fp32 master
    weights / LayerNorm / softmax / loss / Adam): a mixed-precision bar -- logits within
    3e-2, loss within 1e-2, every checked gradient with cosine similarity > 0.999 to fp32."""
import pytest
import torch

from oracle import savqa_oracle as O

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _cos(a, b):
    a = a.detach().cpu().double().reshape(-1)
    b = b.detach().cpu().double().reshape(-1)
    return float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-30))


@pytest.fixture(scope="module")
def setup():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.backends.cuda.matmul.allow_tf32 = False
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.data import synthetic_batch
    d, H, L, Hm, C = 512, 8, 2, 256, 100
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
    P = {n: q.detach().cpu().clone().requires_grad_(True) for n, q in m.named_parameters()}
    batch = synthetic_batch(48, Nv=36, Lq=14, Ns=59, topN=5, num_classes=C, seed=31, device=dev)
    inp = {k: v.cpu() for k, v in batch.items()}
    rc, rv, rs, rmil, _ = O.attmodel_forward(P, inp, decMask=True, num_blocks=L, h=H)
    rloss, _ = O.train_loss(rc, rv, rs, inp["answer"], rmil)
    rloss.backward()
    return m, batch, (rc, rv, rs, rloss), P


GRADS = ("cls.0.weight", "cls_syb.3.weight", "att_vis_grid.enc_feed_forward_1.conv1.0.weight",
         "att_syb.enc_self_attention_0.Q_proj.0.weight", "att_syb.dec_vanilla_attention_1.K_proj.0.weight",
         "att_vis_grid.syb_mlp2.weight", "MIL_NCE.syb_mlp.0.weight", "MIL_NCE.vis_mlp.0.weight")


@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
def test_gemm_precision_modes(setup, prec, monkeypatch):
    from savqa_amd.data import model_args
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    m, batch, (rc, rv, rs, rloss), P = setup
    monkeypatch.setattr(m._engine, "gemm_precision", prec)
    lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
    loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
    opt = Adam(m, lr=1e-4)
    opt.zero_grad()
    loss.backward()
    torch.cuda.synchronize()
    params = dict(m.named_parameters())
    if prec == "bf16x3":
        for a, b, name in ((lc, rc, "concat"), (lv, rv, "vis"), (ls, rs, "syb")):
            assert _rel(a, b) < 1e-3, name
            assert torch.equal(a.detach().cpu().argmax(-1), b.argmax(-1)), name
        assert abs(float(loss) - float(rloss)) < 1e-4 * abs(float(rloss))
        for n in GRADS:
            assert _rel(params[n].grad, P[n].grad) < 1e-2, n
            assert _cos(params[n].grad, P[n].grad) > 0.99999, n
    else:
        for a, b, name in ((lc, rc, "concat"), (lv, rv, "vis"), (ls, rs, "syb")):
            assert _rel(a, b) < 3e-2, name
        assert abs(float(loss) - float(rloss)) < 1e-2 * abs(float(rloss))
        for n in GRADS:
            assert _cos(params[n].grad, P[n].grad) > 0.999, n
