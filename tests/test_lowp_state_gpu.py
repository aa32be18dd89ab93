"""Low-precision modes (BASELINE cfg 3 bf16 / cfg 5 fp8) around two host-side edges:

* the bf16 weight shadow follows every write to the parameters, including the ones that do
  not go through the package's Adam: `load_state_dict` (param.copy_) after a low-precision
  forward must make the next forward use the new weights (params.state_key folds in the
  Parameters' own version counters) -- checked against a model built with those weights;
* sequences longer than the full-row attention kernels (T_syb > 128: super-node graphs,
  cfg 4's 449-token stack) run in the bf16 / fp8 modes on the key-tiled kernels (widened fp32
  Q / K / V), forward and backward, and agree with the fp32 path on the same weights to the
  bf16 tolerance of tests/test_precision_gpu.py."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a = a.detach().double()
    b = b.detach().double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _model(prec, seed, d=256, H=4, L=2, C=60, maxlen=460):
    """Weights as tests/test_precision_gpu.py draws them (uniform, 1/sqrt(fan_in) bounds, LN
    gains near 1): a well-conditioned model, so that bf16 against fp32 measures rounding.
    (At the reference's own init some samples' semantic-stack logits move O(1) under a
    1e-6 relative weight perturbation, tests/test_ddp_gpu.py -- no precision bar holds there.)"""
    from savqa_amd.AttModel_x3 import AttModel
    m = AttModel(None, d, 128, C, 16, maxlen, 120, L, H, 0.0, 0.0, 2, True, device=dev,
                 init=False, gemm_precision=prec)
    gen = torch.Generator(device=dev).manual_seed(seed)
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
    return m


@pytest.fixture(autouse=True, scope="module")
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.backends.cuda.matmul.allow_tf32 = False


def test_bf16_shadow_follows_load_state_dict():
    from savqa_amd.data import model_args, synthetic_batch
    b = synthetic_batch(4, Nv=36, Lq=14, Ns=59, topN=5, num_classes=60, seed=5, device=dev)
    a = _model("bf16", seed=1)
    a.eval()
    with torch.no_grad():
        before = a(*model_args(b), decMask=True, mcb=False)[0].clone()
        donor = _model("bf16", seed=2)
        donor.eval()
        want = donor(*model_args(b), decMask=True, mcb=False)[0].clone()
        a.load_state_dict(donor.state_dict())
        after = a(*model_args(b), decMask=True, mcb=False)[0].clone()
    torch.cuda.synchronize()
    assert _rel(before, want) > 1e-2          # the two weight sets really differ
    assert torch.equal(after, want), _rel(after, want)


@pytest.mark.parametrize("prec", ["bf16", "fp8"])
def test_lowp_long_syb_sequence_runs_key_tiled(prec):
    """T_syb = 154 (> 128): the semantic stack's encoder self-attention and its decoders'
    cross-attention take the key-tiled kernels in the low-precision modes too."""
    from savqa_amd import ops
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    assert ops.use_flash(154, 154)
    b = synthetic_batch(4, Nv=36, Lq=14, Ns=140, topN=5, num_classes=60, seed=7, device=dev)
    outs = {}
    for mode in ("fp32", prec):
        m = _model(mode, seed=3)
        m.train()
        lc, lv, ls, mil, _ = m(*model_args(b), decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, b["answer"], mil)
        m.zero_grad(set_to_none=False)
        loss.backward()
        g = dict(m.named_parameters())["att_syb.enc_self_attention_1.Q_proj.0.weight"].grad
        outs[mode] = (lc.detach().clone(), ls.detach().clone(), float(loss), g.detach().clone())
    torch.cuda.synchronize()
    bar = 2e-2 if prec == "bf16" else 4e-2
    (c32, s32, l32, g32), (clp, slp, llp, glp) = outs["fp32"], outs[prec]
    assert torch.isfinite(clp).all() and torch.isfinite(glp).all()
    assert _rel(clp, c32) < bar and _rel(slp, s32) < bar
    assert abs(llp - l32) < bar * abs(l32)
    assert float((glp - g32).norm() / g32.norm()) < 5 * bar


def test_adam_writes_the_bf16_shadow_bit_exactly():
    """optim.Adam writes the bf16 weight image in its update pass (savqa_adam_shadow) and the
    next forward skips the cast of the arena: the image must equal a fresh round-to-nearest
    cast of every live non-table parameter after each of three steps."""
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    b = synthetic_batch(4, Nv=36, Lq=14, Ns=59, topN=5, num_classes=60, seed=9, device=dev)
    m = _model("bf16", seed=4)
    m.train()
    opt = Adam(m, lr=1e-3)
    a = m._arena
    for it in range(3):
        lc, lv, ls, mil, _ = m(*model_args(b), decMask=True, mcb=False)
        sh = m._engine._shadow
        assert sh.buf_key == a.state_key()
        loss, _ = smoothed_loss(lc, lv, ls, b["answer"], mil)
        opt.zero_grad()
        loss.backward()
        assert sh.current()
        opt.step()
        assert sh.buf_key == a.state_key(), "the step did not write the shadow"
        want = a.flat[:a.n_live].to(torch.bfloat16)
        lo = 0
        for t0, t1 in a.table_ranges() + [(a.n_live, a.n_live)]:
            if t0 > lo:
                assert torch.equal(sh.buf[lo:t0], want[lo:t0]), (it, lo, t0)
            lo = max(lo, t1)
