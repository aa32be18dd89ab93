"""Dropout (nn.Dropout sites of model_v=3 at the reference's training default p=0.5,
main_itp_ddp_tar_super_node.py:466) on the HIP path, through the C ABI.

Masks: the library's counter-hash stream (include/savqa.h "Dropout"), restated in
oracle/savqa_oracle.py:dropout_keep. Kernel masks must match the restatement bit for
bit; the whole model in training mode with p=0.5 must match the CPU oracle run with the
same masks (1e-3 relative, answer argmax exact)."""
import numpy as np
import pytest
import torch

from oracle import savqa_oracle as O

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.backends.cuda.matmul.allow_tf32 = False


def ops():
    from savqa_amd import ops as K
    return K


def keep(seed, site, n, p):
    return torch.from_numpy(O.dropout_keep(seed, site, n, p)).to(dev)


@pytest.mark.parametrize("n,p", [(4096, 0.5), (1001, 0.1), (77, 0.9), (64, 1.0), (128, 0.0)])
def test_dropout_mask_bit_exact(n, p):
    K = ops()
    seed = 0x1234_5678_9ABC_DEF0
    x = torch.rand(n, device=dev) + 0.5
    out = torch.empty_like(x)
    K.dropout(x, n, (seed, p), 7, out)
    k = keep(seed, 7, n, p)
    scale = 0.0 if p >= 1 else float(np.float32(1) / (np.float32(1) - np.float32(p)))
    assert torch.equal(out, x * k.float() * scale)
    # in place, and as its own backward (same op on dY)
    y = x.clone()
    K.dropout(y, n, (seed, p), 7, y)
    assert torch.equal(y, out)


@pytest.mark.parametrize("site_pos", [1, -1])
def test_posadd_dropout_fwd_bwd(site_pos):
    K = ops()
    B, T, d, p, seed = 37, 9, 64, 0.5, 99
    z = torch.randn(B * T, d, device=dev)
    pos = torch.randn(20, d, device=dev)
    out = torch.empty_like(z)
    K.posadd_dropout(z, pos, B, T, d, (seed, p), site_pos, 2, out)
    kp = keep(seed, site_pos, B * T * d, p).reshape(B, T, d).float() * 2 if site_pos >= 0 else 1.0
    kx = keep(seed, 2, B * T * d, p).reshape(B, T, d).float() * 2
    ref = (z.reshape(B, T, d) + pos[:T].unsqueeze(0) * kp) * kx
    assert torch.allclose(out.reshape(B, T, d), ref, rtol=0, atol=1e-6)
    g = torch.randn(B * T, d, device=dev)
    dpos = torch.randn(20, d, device=dev)
    dpos0 = dpos.clone()
    dz = g.clone()
    K.posadd_dropout_bwd(dz, B, T, d, (seed, p), site_pos, 2, dz, dpos)
    dz_ref = g.reshape(B, T, d) * kx
    assert torch.equal(dz.reshape(B, T, d), dz_ref)
    dpos_ref = dpos0.clone()
    dpos_ref[:T] += (dz_ref * kp).sum(0)
    assert torch.allclose(dpos, dpos_ref, rtol=1e-5, atol=1e-5)


def test_dec_init_dropout():
    K = ops()
    B, d, p, seed = 50, 128, 0.5, 5
    emb, pos = torch.randn(10, d, device=dev), torch.randn(30, d, device=dev)
    out = torch.empty(B, d, device=dev)
    K.dec_init(emb, 2, d ** 0.5, pos, B, d, out, drop=(seed, p), site=3)
    k = keep(seed, 3, B * d, p).reshape(B, d).float() * 2
    ref = (emb[2] * d ** 0.5 + pos[0]).unsqueeze(0) * k
    assert torch.allclose(out, ref, rtol=1e-6, atol=1e-6)
    g = torch.randn(B, d, device=dev)
    demb, dpos = torch.zeros_like(emb), torch.zeros_like(pos)
    K.dec_init_bwd(g, B, d, 2, d ** 0.5, demb, dpos, drop=(seed, p), site=3)
    assert torch.allclose(demb[2], (g * k).sum(0) * d ** 0.5, rtol=1e-5, atol=1e-4)
    assert torch.allclose(dpos[0], (g * k).sum(0), rtol=1e-5, atol=1e-5)


def _small_model(p):
    from savqa_amd.AttModel_x3 import AttModel
    d, H, L, Hm, C = 256, 4, 2, 64, 20
    m = AttModel(None, d, Hm, C, 16, 60, 10, L, H, p, 0.0, 2, True, device=dev, init=False)
    g = torch.Generator(device=dev).manual_seed(3)
    with torch.no_grad():
        for n, prm in m.named_parameters():
            leaf = n.rsplit(".", 1)[-1]
            if leaf == "gamma":
                prm.uniform_(0.8, 1.2, generator=g)
            elif prm.dim() == 1:
                prm.uniform_(-0.2, 0.2, generator=g)
            else:
                bound = 1.0 / prm.shape[-1] ** 0.5
                prm.uniform_(-bound, bound, generator=g)
    return m, (d, H, L, C)


def _rel(a, b):
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def test_model_train_dropout_matches_oracle():
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    m, (d, H, L, C) = _small_model(0.5)
    m.train()
    P = {n: q.detach().cpu().clone().requires_grad_(True) for n, q in m.named_parameters()}
    batch = synthetic_batch(3, Nv=6, Lq=5, Ns=8, topN=5, num_classes=C, seed=21, device=dev)
    torch.manual_seed(1234)
    lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
    drop = m._last_dropout
    assert drop is not None and drop[1] == 0.5
    loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
    opt = Adam(m, lr=1e-4)
    opt.zero_grad()
    loss.backward()
    torch.cuda.synchronize()

    inp = {k: v.cpu() for k, v in batch.items()}
    rc, rv, rs, rmil, _ = O.attmodel_forward(P, inp, decMask=True, num_blocks=L, h=H, drop=drop)
    rloss, _ = O.train_loss(rc, rv, rs, inp["answer"], rmil)
    rloss.backward()
    # dropout must actually change the result (vs the same weights with p = 0)
    r0, _, _, _, _ = O.attmodel_forward(P, inp, decMask=True, num_blocks=L, h=H, drop=None)
    assert _rel(r0, rc) > 1e-2
    for a, b, name in ((lc, rc, "concat"), (lv, rv, "vis"), (ls, rs, "syb")):
        assert _rel(a, b) < 1e-3, name
        assert torch.equal(a.detach().cpu().argmax(-1), b.argmax(-1)), name
    assert abs(float(loss) - float(rloss)) < 1e-4 * abs(float(rloss))
    params = dict(m.named_parameters())
    for n in ("cls.0.weight", "cls.0.bias", "cls_vis.3.weight", "cls_syb.0.weight",
              "att_vis_grid.syb_positional_encoding.0.lookup_table",
              "att_syb.syb_positional_encoding.lookup_table",
              "att_vis_grid.dec_emb.lookup_table", "att_syb.dec_positional_encoding.lookup_table",
              "att_vis_grid.syb_mlp2.weight", "att_syb.syb_mlp2.bias",
              "att_vis_grid.enc_self_attention_0.Q_proj.0.weight",
              "att_syb.dec_feed_forward_1.conv1.0.weight", "MIL_NCE.ipt_mlp.0.weight",
              "MIL_NCE.vis_mlp.0.weight"):
        assert _rel(params[n].grad, P[n].grad) < 1e-3, n
    # the backward regenerated the forward's masks: a second forward under the same
    # torch seed reproduces the logits (up to the fp32 order of split-K atomics)
    torch.manual_seed(1234)
    lc2, _, _, _, _ = m(*model_args(batch), decMask=True, mcb=False)
    assert _rel(lc2, lc) < 1e-5
    # eval mode: no dropout
    m.eval()
    with torch.no_grad():
        le, _, _, _, _ = m(*model_args(batch), decMask=True, mcb=False)
    assert m._last_dropout is None
    assert _rel(le, r0) < 1e-3
