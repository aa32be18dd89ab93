"""Whole-model parity at sequence lengths beyond the full-row attention kernels (T > 128,
key-tiled path): BASELINE config 4's shape family (100 regions, a 435-node scene graph
-> T_syb = 449, d = 1024, 16 heads; the stated 12 heads do not divide d = 1024 in the
reference either) at reduced depth, and a mixed case where the visual stack
(T = 114) stays on the full-row kernels while the semantic stack (T = 154) is tiled.
Checked against the CPU oracle on the same weights, inputs and dropout masks: outputs and
loss at the north-star 1e-3 max-relative tolerance. Gradients: 1e-3 max-relative at
d = 256; at d = 1024, T = 449 (3.7M feed-forward ReLU units per stack layer) a unit whose
pre-activation lies within fp32 rounding of 0 flips its ReLU mask between any two fp32
implementations -- the fp32 CPU oracle itself disagrees with fp64 on one position-table
row (sample 0, t = 331) by 9e-4 of the tensor max for exactly that reason
(tools/dbg/longseq_dbg.py) -- so there the bound is 2e-3 in relative Frobenius norm."""
import pytest
import torch

from oracle import savqa_oracle as O

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _frob(a, b):
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("d,H,L,Nv,Ns,B,p", [(256, 4, 2, 100, 140, 2, 0.5),
                                             (1024, 16, 2, 100, 435, 2, 0.0)])
def test_long_sequence_model_matches_oracle(d, H, L, Nv, Ns, B, p):
    gcheck = (lambda a, b: _rel(a, b) < 1e-3) if d <= 256 else (lambda a, b: _frob(a, b) < 2e-3)
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.backends.cuda.matmul.allow_tf32 = False
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    Hm, C, Lq = 128, 40, 14
    m = AttModel(None, d, Hm, C, 16, 460, 120, L, H, p, 0.0, 2, True, device=dev, init=False)
    gen = torch.Generator(device=dev).manual_seed(17)
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
    batch = synthetic_batch(B, Nv=Nv, Lq=Lq, Ns=Ns, topN=5, num_classes=C, seed=29, device=dev)
    torch.manual_seed(77)
    lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
    loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
    opt = Adam(m, lr=1e-4)
    opt.zero_grad()
    loss.backward()
    torch.cuda.synchronize()
    inp = {k: v.cpu() for k, v in batch.items()}
    torch.set_num_threads(min(16, torch.get_num_threads()))
    rc, rv, rs, rmil, _ = O.attmodel_forward(P, inp, decMask=True, num_blocks=L, h=H,
                                             drop=m._last_dropout)
    rloss, _ = O.train_loss(rc, rv, rs, inp["answer"], rmil)
    rloss.backward()
    for a, b, name in ((lc, rc, "concat"), (lv, rv, "vis"), (ls, rs, "syb")):
        assert _rel(a, b) < 1e-3, name
        assert torch.equal(a.detach().cpu().argmax(-1), b.argmax(-1)), name
    assert abs(float(loss) - float(rloss)) < 1e-4 * abs(float(rloss))
    params = dict(m.named_parameters())
    for n in ("cls.0.weight", "att_syb.enc_self_attention_0.Q_proj.0.weight",
              "att_syb.enc_self_attention_1.K_proj.0.weight",
              "att_syb.enc_self_attention_1.V_proj.0.bias",
              "att_syb.dec_vanilla_attention_0.K_proj.0.weight",
              "att_syb.dec_vanilla_attention_1.Q_proj.0.weight",
              "att_vis_grid.enc_self_attention_1.Q_proj.0.weight",
              "att_syb.syb_positional_encoding.lookup_table", "MIL_NCE.ipt_mlp.0.weight"):
        assert gcheck(params[n].grad, P[n].grad), (n, _rel(params[n].grad, P[n].grad),
                                                   _frob(params[n].grad, P[n].grad))
