"""BASELINE cfg 4 at its benched shape (bench.py --workload cfg4): d = 1024, 16 heads, 6+6
layers (models/AttModel_x3.py:127-154), 100 regions x 2048-d, a 435-node scene graph
(T_vis = 114, T_syb = 449: the key-tiled attention kernels), hidden_size_mil 1024, 914
classes, B = 32 -- the launch plans the benched step uses (the d = 1024 decoder K/V GEMM with
N = 12288, the B = 32 skinny plans, the key-tiled attention at T = 449 in all 6 layers).
  * against the CPU oracle (oracle/savqa_oracle.py) at full depth on 2 of the samples:
    logits 1e-3 max-relative with exact argmax, loss 1e-4, head gradients 1e-3 max-relative;
    the gradients under the 6-layer stacks against fp64 on the HIP path's own ReLU branch
    (tests/branch_masks.py), per parameter within 1.5x of the fp32 CPU oracle's own distance
    to the same fp64 reference (as tests/test_fullsize_gpu.py at cfg 2);
  * batch-slicing invariance at B = 32 (4 chunks of 8: other GEMM tilings, splits and
    attention grids) and gradient linearity (grad(32) = mean of the chunk gradients).
LayerNorm gamma / beta are randomised (exact-zero row masks)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"
B, NV, NS = 32, 100, 435


def _rel(a, b):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _frob(a, b):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def model():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.utils import init_params_
    m = AttModel(None, 1024, 1024, 914, 40, 450, 49, 6, 16, 0.0, 0.1, 311, True, device=dev,
                 init=False)
    init_params_(m, seed=13)
    g = torch.Generator(device=dev).manual_seed(14)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith(".gamma"):
                p.normal_(1.0, 0.2, generator=g)
            elif n.endswith(".beta"):
                p.normal_(0.0, 0.2, generator=g)
    return m


@pytest.fixture(scope="module")
def batch():
    from savqa_amd.data import synthetic_batch
    return synthetic_batch(B, Nv=NV, Ns=NS, seed=4242, device=dev)


def _chunk(b, lo, hi):
    return {k: v[lo:hi] for k, v in b.items()}


def test_cfg4_shape(batch):
    assert batch["vis_fea"].shape == (B, NV, 2048)
    assert batch["macro_ipt"].shape[1] == NS


def test_cfg4_full_depth_against_oracle(model, batch):
    from oracle import savqa_oracle as O
    from savqa_amd.data import model_args
    from savqa_amd.loss import smoothed_loss
    import branch_masks
    b = _chunk(batch, 0, 2)
    model.train()  # dropout 0: train-mode numerics with gradients
    heads = ["cls.0.weight", "cls.3.weight", "cls_vis.0.weight", "cls_syb.3.weight"]
    deep = ["att_syb.enc_self_attention_0.Q_proj.0.weight",
            "att_syb.enc_self_attention_5.K_proj.0.weight",
            "att_syb.dec_vanilla_attention_5.K_proj.0.weight",
            "att_vis_grid.enc_feed_forward_0.conv1.0.weight", "att_syb.syb_mlp.0.weight",
            "att_vis_grid.enc_self_attention_3.V_proj.0.weight",
            "att_syb.enc_feed_forward_2.conv2.weight", "MIL_NCE.ipt_mlp.0.weight",
            "MIL_NCE.vis_mlp.0.weight"]
    params = dict(model.named_parameters())
    box = branch_masks.capture(model)
    lc, lv, ls, mil, _ = model(*model_args(b), decMask=True, mcb=False)
    masks = branch_masks.hip_masks(box[0], d=1024)
    loss, _ = smoothed_loss(lc, lv, ls, b["answer"], mil)
    model.zero_grad(set_to_none=False)
    loss.backward()
    torch.cuda.synchronize()
    mine = {n: params[n].grad.detach().cpu() for n in heads + deep}
    torch.set_num_threads(min(16, torch.get_num_threads()))
    kw = dict(num_blocks=6, h=16)
    ref, (rc, rv, rs, rmil, rloss) = branch_masks.oracle_grads(
        O, params, b, None, torch.float32, "cpu", heads, **kw)
    for a, r, name in ((lc, rc, "concat"), (lv, rv, "vis"), (ls, rs, "syb")):
        assert _rel(a, r) < 1e-3, name
        assert torch.equal(a.detach().cpu().argmax(-1), r.argmax(-1)), name
    assert abs(float(mil) - float(rmil)) < 1e-4 * max(1.0, abs(float(rmil)))
    assert abs(float(loss) - float(rloss)) < 1e-4 * abs(float(rloss))
    errs = {n: _rel(mine[n], ref[n]) for n in heads}
    for n in heads:
        assert errs[n] < 1e-3, (n, errs)
    # the masks the comparison aligns on are themselves checked: against the
    # fp64 oracle's own decisions, HIP flips only units within rounding of 0
    flips = branch_masks.mask_disagreement(O, params, b, masks, deep, **kw)
    print(f"cfg4 ReLU sites compared {len(flips)}, flipped units "
          f"{sum(v[0] for v in flips.values())}")
    r64, _ = branch_masks.oracle_grads(O, params, b, masks, torch.float64, dev, deep, **kw)
    r32, _ = branch_masks.oracle_grads(O, params, b, masks, torch.float32, "cpu", deep, **kw)
    for n in deep:
        e_hip, e_cpu = _frob(mine[n], r64[n]), _frob(r32[n], r64[n])
        print(f"cfg4 {n}: hip {e_hip:.2e} cpu-fp32 {e_cpu:.2e} (branch-aligned fp64)")
        assert float(r64[n].abs().max()) > 0, n
        assert e_hip <= 1.5 * e_cpu + 1e-7, (n, e_hip, e_cpu)


def test_batch_slicing_invariance_cfg4(model, batch):
    from savqa_amd.data import model_args
    model.eval()
    with torch.no_grad():
        full = model(*model_args(batch), decMask=True, mcb=False)[:3]
        parts = [model(*model_args(_chunk(batch, lo, lo + 8)), decMask=True, mcb=False)[:3]
                 for lo in range(0, B, 8)]
    torch.cuda.synchronize()
    for k in range(3):
        cat = torch.cat([p[k] for p in parts])
        assert _rel(full[k], cat) < 1e-4, k
        assert torch.equal(full[k].argmax(-1), cat.argmax(-1)), k


def test_gradient_linearity_cfg4(model, batch):
    from savqa_amd.data import model_args
    from savqa_amd.loss import smoothed_loss
    model.train()
    names = ["cls.3.weight", "cls_vis.0.weight", "att_syb.enc_feed_forward_0.conv1.0.weight",
             "att_syb.enc_self_attention_3.Q_proj.0.weight",
             "att_vis_grid.enc_self_attention_5.V_proj.0.weight",
             "att_syb.dec_vanilla_attention_2.K_proj.0.weight", "MIL_NCE.ipt_mlp.0.weight"]
    params = dict(model.named_parameters())

    def grads(b):
        lc, lv, ls, mil, _ = model(*model_args(b), decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, b["answer"], mil, with_milnce=False)
        model.zero_grad(set_to_none=False)
        loss.backward()
        torch.cuda.synchronize()
        return {n: params[n].grad.detach().clone() for n in names}

    full = grads(batch)
    acc = None
    for lo in range(0, B, 8):
        gk = grads(_chunk(batch, lo, lo + 8))
        acc = gk if acc is None else {n: acc[n] + gk[n] for n in names}
    errs = {n: _frob(full[n], acc[n] / 4) for n in names}
    for n in names:
        assert full[n].abs().max() > 0, n
        assert errs[n] < (1e-4 if n.startswith("cls") else 5e-3), errs
