"""Whole-model parity of the bf16-MFMA GEMM modes (include/savqa.h savqa_gemm_desc.prec) at a
batch large enough that the 128x128-tile GEMMs carry the model (B=48: 3504 rows per stack):
  "bf16x3" (three bf16 MFMAs per product, ~2^-16 of sum|a*b| per dot product): outputs at
    the north-star fp32 bar (logits within 1e-3 max-relative of the CPU fp32 oracle, answer
    argmax exact); weight gradients are long sums with heavy cancellation, where 2^-16 of
    the absolute sum shows up as ~4e-3 of the largest entry -- so they are held to 1e-2
    max-relative and cosine > 0.99999 (this is why fp32 products stay the default);
  "bf16" (BASELINE config 3's bf16 training: bf16-resident activations and weight shadow
    into savqa_gemm_lp, fp32 accumulation, fp32 residual stream / LayerNorm statistics /
    softmax / loss / master weights / Adam) and "fp8" (BASELINE config 5: the region
    features and the two GEMMs that read them, att_vis_grid.syb_mlp2 and MIL_NCE.vis_mlp.0,
    in fp8-e4m3 with per-32 e8m0 block scales, the rest as "bf16") are held against what
    STOCK mixed precision gets on the same model: the oracle itself run under
    torch.autocast(bf16) on the GPU. Gradients here are cancellation-heavy (the key
    projections' weight gradients are sums of rows that add up to zero, since softmax over
    keys ignores a shared shift), so their absolute bf16 error is large (autocast: 12-19% of
    the norm for K_proj weights) and only a calibrated bar means anything.
    Measured (B=48, L=2): bf16 logits 1.1e-3 max-rel (autocast 6.6e-3), every gradient's
    relative-norm error BELOW autocast's (worst 0.74x); fp8 logits 5.1e-3, gradients up to
    2.1x autocast's bf16 error (the fp8 features and weights). Bars: answer argmax exact;
    logits <= autocast's error (bf16) / 2x it (fp8); loss 1e-3 / 2e-3; each gradient's
    relative-norm error <= max(1.25x, 2.5x for fp8) autocast's, floor 1e-2 (3e-2 fp8).
For fp8 the oracle (and the autocast run) is fed the DEQUANTISED features: quantising the
input is a data choice, not kernel error. The key-projection BIASES are left out: their
exact gradient is zero (the same shift invariance), so every implementation returns noise.
Two geometries: "small" (L=2, 100 classes, H_mil=256) and "full" -- the benched model depth
and widths (6+6 layers, 914 classes, H_mil=1024, AttModel_x3.py:141-154 / :267-281 decoders)
at B=48, where the 6-layer decoders' N=6144 K/V projection runs on the 8-phase 256x256
gemm_lp3_kernel (asserted from the launch probe) inside the model-level check."""
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


GEOM = {"small": dict(L=2, Hm=256, C=100), "full": dict(L=6, Hm=1024, C=914)}


@pytest.fixture(scope="module", params=["small", "full"])
def setup(request):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.backends.cuda.matmul.allow_tf32 = False
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.data import synthetic_batch
    geo = GEOM[request.param]
    d, H, L, Hm, C = 512, 8, geo["L"], geo["Hm"], geo["C"]
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
    m._geom = (request.param, L)
    return m, batch, (rc, rv, rs, rloss), P


GRADS = ("cls.0.weight", "cls_syb.3.weight", "att_vis_grid.enc_feed_forward_1.conv1.0.weight",
         "att_syb.enc_self_attention_0.Q_proj.0.weight", "att_syb.dec_vanilla_attention_1.K_proj.0.weight",
         "att_vis_grid.syb_mlp2.weight", "MIL_NCE.syb_mlp.0.weight", "MIL_NCE.vis_mlp.0.weight")


def _quantised_features(batch):
    """fp8-e4m3 codes + e8m0 scales of the region features (savqa_quant_fp8) and their
    dequantised fp32 values (what the oracle sees)."""
    from savqa_amd import ops
    B, Nv, Dv = batch["vis_fea"].shape
    R = B * Nv
    q8 = torch.empty(R, Dv, dtype=torch.uint8, device=dev)
    s8 = torch.empty(R, Dv // 32, dtype=torch.uint8, device=dev)
    ops.quant_fp8(batch["vis_fea"].reshape(R, Dv), R, Dv, Dv, q8, Dv, s8, Dv // 32)
    deq = q8.view(torch.float8_e4m3fn).float().cpu() * torch.pow(
        2.0, s8.cpu().float() - 127).repeat_interleave(32, 1)
    return q8.view(torch.float8_e4m3fn).reshape(B, Nv, Dv), s8.reshape(B, Nv, Dv // 32), \
        deq.reshape(B, Nv, Dv)


@pytest.fixture(scope="module")
def fp8_ref(setup):
    """oracle forward/backward on the dequantised fp8 features"""
    m, batch, _, P0 = setup
    q8, s8, deq = _quantised_features(batch)
    inp = {k: v.cpu() for k, v in batch.items()}
    inp["vis_fea"] = deq
    P = {n: q.detach().clone().requires_grad_(True) for n, q in P0.items()}
    rc, rv, rs, rmil, _ = O.attmodel_forward(P, inp, decMask=True, num_blocks=m._geom[1], h=8)
    rloss, _ = O.train_loss(rc, rv, rs, inp["answer"], rmil)
    rloss.backward()
    return (rc, rv, rs, rloss), P, q8, s8


@pytest.fixture(scope="module")
def autocast_ref(setup, fp8_ref):
    """the oracle under torch.autocast(bf16) on the GPU, for the plain and the dequantised
    fp8 features: logits and gradients of stock mixed precision"""
    m, batch, _, P0 = setup
    out = {}
    for key, vis in (("bf16", None), ("fp8", _quantised_features(batch)[2])):
        inp = {k: v.to(dev) for k, v in batch.items()}
        if vis is not None:
            inp["vis_fea"] = vis.to(dev)
        P = {n: q.detach().to(dev).requires_grad_(True) for n, q in P0.items()}
        with torch.device(dev), torch.autocast("cuda", dtype=torch.bfloat16):
            c, v_, s_, mil, _ = O.attmodel_forward(P, inp, decMask=True, num_blocks=m._geom[1],
                                                   h=8)
        with torch.device(dev):
            loss, _ = O.train_loss(c.float(), v_.float(), s_.float(), inp["answer"], mil.float())
            loss.backward()
        out[key] = ((c.float(), v_.float(), s_.float()), {n: q.grad for n, q in P.items()})
    return out


def _nerr(a, b):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _grads_checked(P):
    # parameters the step does not reach (zero gradient in both) are not compared
    return [n for n in P if P[n].grad is not None and not n.endswith("K_proj.0.bias")
            and bool(P[n].grad.abs().sum() > 0)]


@pytest.mark.parametrize("prec", ["bf16x3", "bf16", "fp8"])
def test_gemm_precision_modes(setup, fp8_ref, autocast_ref, prec, monkeypatch):
    from savqa_amd.data import model_args
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    m, batch, (rc, rv, rs, rloss), P = setup
    if prec == "fp8":
        (rc, rv, rs, rloss), P, _, _ = fp8_ref
    from savqa_amd import ops
    monkeypatch.setattr(m._engine, "gemm_precision", prec)
    probe = ops.GemmProbe()
    ops.set_gemm_probe(probe)
    try:
        lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
        opt = Adam(m, lr=1e-4)
        opt.zero_grad()
        loss.backward()
        torch.cuda.synchronize()
    finally:
        ops.set_gemm_probe(None)
    if prec != "bf16x3" and m._geom[0] == "full":
        # the benched depth: the 8-phase 256x256 kernel carries the decoder K/V projections
        assert any(k.startswith("gemm_lp3_kernel") for k in probe.summary()), probe.summary()
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
        (ac, av, as_), ag = autocast_ref[prec]
        # fp8 floor 3e-2: gradients that run through the fp8 vis_mlp weights (MIL_NCE.syb_mlp
        # meets relu(vis_mlp(v))) inherit the weights' e4m3 rounding (2^-4 relative)
        lmul, lbar, gmul, floor = (1.0, 1e-3, 1.25, 1e-2) if prec == "bf16" else \
            (2.0, 2e-3, 2.5, 3e-2)
        for a, b, amp, name in ((lc, rc, ac, "concat"), (lv, rv, av, "vis"), (ls, rs, as_, "syb")):
            assert _rel(a, b) < lmul * _rel(amp, b), name
            assert torch.equal(a.detach().cpu().argmax(-1), b.argmax(-1)), name
        assert abs(float(loss) - float(rloss)) < lbar * abs(float(rloss))
        for n in _grads_checked(P):
            assert _nerr(params[n].grad, P[n].grad) <= max(gmul * _nerr(ag[n], P[n].grad), floor), n


def test_fp8_prequantised_input_matches_engine_quantisation(setup, fp8_ref, monkeypatch):
    """cfg 5 hands the model fp8 region features + block scales (vis_fea_scale); that path
    must give bit-identical outputs to the engine quantising the fp32 features itself."""
    from savqa_amd.data import model_args
    m, batch, _, _ = setup
    _, _, q8, s8 = fp8_ref
    monkeypatch.setattr(m._engine, "gemm_precision", "fp8")
    with torch.no_grad():
        a = m(*model_args(batch), decMask=True, mcb=False)
        b8 = dict(batch)
        b8["vis_fea"] = q8
        b = m(*model_args(b8), decMask=True, mcb=False, vis_fea_scale=s8)
    for x, y in zip(a[:3], b[:3]):
        assert torch.equal(x, y)
