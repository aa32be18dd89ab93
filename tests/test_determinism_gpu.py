"""Run-to-run determinism and multi-step drift.

* The GloVe-table gradients (nn.Embedding's backward: the MIL-NCE object words, the question
  tokens of both stacks; AttModel_x3.py:96-99, :216-219, :352-360) are the dense rows dY W summed
  per id in sorted-id order (savqa_segment_add_rows, ops.DET_SCATTER) instead of an atomic
  scatter: with every GEMM K split through slabs and the LayerNorm column sums in block order,
  EVERY gradient of a training step is now bit-identical run to run -- checked here with ids
  drawn from a tiny vocabulary, so duplicates are the rule, in the fp32 (x6) and bf16 modes.
* 50 Adam steps at the cfg-1 shape (B = 4, d = 512, 6 + 6 layers, 914 classes) with the x6
  GEMM and with the native fp32 MFMA kernel, against the same 50 steps of the oracle in fp64
  (main:206, :363-366): x6's parameter drift from fp64 is held to 1.25x native's, which bounds
  the signed truncation bias of its three-term split (gemm_x6.hip) accumulating over steps.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _model(prec, dropout=0.0, seed=3):
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.utils import init_params_
    m = AttModel(None, 512, 1024, 914, 40, 450, 49, 6, 8, dropout, 0.1, 311, True, device=dev,
                 init=False, gemm_precision=prec)
    init_params_(m, seed=seed)
    g = torch.Generator(device=dev).manual_seed(seed + 1)
    with torch.no_grad():  # LN gamma / beta off (1, 0): every key mask decided by non-zero sums
        for n, p in m.named_parameters():
            leaf = n.rsplit(".", 1)[-1]
            if leaf == "gamma":
                p.uniform_(0.8, 1.2, generator=g)
            elif leaf == "beta":
                p.uniform_(-0.1, 0.1, generator=g)
    m.train()
    return m


def _dup_batch(B, vocab=40, seed=5):
    """synthetic_batch with every word id (question tokens, scene-graph nodes, object words)
    from a small vocabulary: each id occurs many times per step."""
    from savqa_amd.data import synthetic_batch
    b = synthetic_batch(B, seed=seed, device=dev)
    for k in ("q_ipt", "macro_ipt", "micro_positive_obj", "micro_negative_obj"):
        b[k] = b[k] % vocab
    return b


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_training_step_gradients_bit_identical(prec):
    from savqa_amd import ops
    from savqa_amd.data import model_args
    from savqa_amd.loss import smoothed_loss
    if not ops.DET_SCATTER:
        pytest.skip("SAVQA_DET_SCATTER=0: the atomic table scatters are run-order dependent")
    m = _model(prec)
    b = _dup_batch(32)
    a = m._arena
    grads = []
    for _ in range(3):
        lc, lv, ls, mil, _ = m(*model_args(b), decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, b["answer"], mil)
        m.zero_grad(set_to_none=False)
        loss.backward()
        torch.cuda.synchronize()
        grads.append(a.grad[:a.n_live].clone())
    bad = []
    for n in a.live_names:
        o, shp = a.offsets[n]
        x = [g[o:o + shp.numel()] for g in grads]
        if not (torch.equal(x[0], x[1]) and torch.equal(x[0], x[2])):
            bad.append(n)
    assert not bad, bad
    # the tables did get duplicate-row gradients
    o, shp = a.offsets["MIL_NCE.syb_emb.weight"]
    tab = grads[0][o:o + shp.numel()].view(shp)
    assert int((tab.abs().sum(1) > 0).sum()) <= 40 and float(tab.abs().max()) > 0


def test_segment_add_rows_matches_index_add():
    """savqa_segment_add_rows against fp64 index_add over ragged runs (ids with 1..50
    duplicates, ids absent, a strided source), and bit-identical reruns."""
    from savqa_amd import ops
    gen = torch.Generator(device=dev).manual_seed(9)
    R, cols, V = 20000, 300, 997
    ids = torch.randint(0, V, (R,), generator=gen, device=dev) ** 2 % V
    T = torch.randn(R, 304, generator=gen, device=dev)
    base = torch.randn(V, cols, generator=gen, device=dev)
    outs = []
    for _ in range(2):
        tab = base.clone()
        ops.segment_add_rows(T, 304, ids, cols, tab, cols)
        outs.append(tab)
    ref = base.double().index_add(0, ids, T[:, :cols].double())
    err = float((outs[0].double() - ref).abs().max() / ref.abs().max())
    assert err < 1e-6, err
    assert torch.equal(outs[0], outs[1])
    untouched = torch.ones(V, dtype=torch.bool, device=dev)
    untouched[ids] = False
    assert torch.equal(outs[0][untouched], base[untouched])


def test_x6_drift_over_50_adam_steps_within_native():
    """50 Adam steps (lr 1e-4, the reference's) at the cfg-1 shape from one initial state:
    the x6 GEMM path, the native fp32 MFMA path and the oracle in fp64 on the GPU. The live
    parameters' distance to the fp64 trajectory, relative to how far fp64 moved them, is held
    to 1.25x native's (both move off the fp64 path by rounding and the ReLU units that rounding
    flips; a truncation bias that accumulated would show here as x6 drifting further)."""
    from oracle import savqa_oracle as O
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    steps = 50
    b = synthetic_batch(4, seed=21, device=dev)
    finals = {}
    for prec in ("fp32", "fp32_native"):
        m = _model(prec, seed=11)
        a = m._arena
        if prec == "fp32":
            init = {n: p.detach().clone() for n, p in m.named_parameters()}
            live = list(a.live_names)
        opt = Adam(m, lr=1e-4)
        for _ in range(steps):
            lc, lv, ls, mil, _ = m(*model_args(b), decMask=True, mcb=False)
            loss, _ = smoothed_loss(lc, lv, ls, b["answer"], mil)
            opt.zero_grad()
            loss.backward()
            opt.step()
        torch.cuda.synchronize()
        finals[prec] = {n: p.detach().clone() for n, p in m.named_parameters() if n in live}
        del m, opt
    # the same steps in fp64 (the oracle restates the reference's forward, loss and Adam)
    P = {n: p.double().requires_grad_(n in live) for n, p in init.items()}
    inp = {k: (v.double() if v.is_floating_point() else v) for k, v in b.items()}
    state = {}
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        with torch.device(dev):
            _fp64_steps(O, P, inp, state, steps)
    finally:
        torch.set_default_dtype(old)
    num = {k: 0.0 for k in finals}
    den = 0.0
    for n in live:
        r = P[n].detach()
        den += float((r - init[n].double()).pow(2).sum())
        for k in finals:
            num[k] += float((finals[k][n].double() - r).pow(2).sum())
    e = {k: (v / den) ** 0.5 for k, v in num.items()}
    print(f"\n50-step drift from fp64, relative to fp64's own movement: x6 {e['fp32']:.3e}, "
          f"native {e['fp32_native']:.3e}, ratio {e['fp32'] / e['fp32_native']:.3f}")
    assert den > 0
    assert e["fp32"] <= 1.25 * e["fp32_native"] + 1e-9, e


def _fp64_steps(O, P, inp, state, steps):
    for t in range(1, steps + 1):
        for p in P.values():
            p.grad = None
        rc, rv, rs, rmil, _ = O.attmodel_forward(P, inp)
        rloss, _ = O.train_loss(rc, rv, rs, inp["answer"], rmil)
        rloss.backward()
        with torch.no_grad():
            O.adam_step(P, {k: v.grad for k, v in P.items() if v.grad is not None}, state, t)
