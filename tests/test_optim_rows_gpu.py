"""Row-tracked optimizer for the three 407000 x 300 GloVe tables (main:206 Adam
over dense embedding gradients): the engine's backward flags the rows it writes
(savqa_mark_rows), Adam updates only rows that were ever touched (savqa_adam_rows) and
zero_grad clears only the rows touched since the last zero (savqa_zero_rows). A row never
touched has m = v = 0 and g = 0, where torch.optim.Adam's update is exactly zero, so the
result must be BIT-identical to the dense Adam over the whole live range -- checked here on
the real step: each of 3 steps (different token ids per step, so rows touched at step 1
but not at step 2 keep decaying) snapshots (p, g, m, v) before the row-tracked step and
replays the dense savqa_adam on the snapshot."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model():
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.utils import init_params_
    m = AttModel(None, 256, 64, 12, 16, 60, 10, 2, 4, 0.0, 0.0, 2, True, device="cuda",
                 init=False)
    init_params_(m, seed=5)
    m.train()
    return m


def test_row_tracked_adam_is_bit_identical_to_dense_adam():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from savqa_amd import ops
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    m = _model()
    a = m._arena
    opt = Adam(m, lr=1e-3)
    tables = ("att_vis_grid.syb_emb.weight", "att_syb.syb_emb.weight", "MIL_NCE.syb_emb.weight")
    for step in range(3):
        batch = synthetic_batch(4, Nv=6, Lq=5, Ns=8, topN=5, num_classes=12, seed=100 + step,
                                device="cuda")
        lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
        opt.zero_grad()
        torch.cuda.synchronize()
        if a.grad is not None:
            assert int(torch.count_nonzero(a.grad)) == 0, "zero_grad left touched rows non-zero"
        loss.backward()
        torch.cuda.synchronize()
        assert set(a.row_flags) == set(tables)
        if opt.m is None:  # the state the first step allocates
            opt.m = torch.zeros(a.n_live, device="cuda")
            opt.v = torch.zeros(a.n_live, device="cuda")
        n = a.n_live
        p0, g0 = a.flat[:n].clone(), a.grad[:n].clone()
        m0, v0 = opt.m.clone(), opt.v.clone()
        touched = {t: int((a.row_flags[t] & 2).ne(0).sum()) for t in tables}
        opt.step()
        torch.cuda.synchronize()
        # dense replay of the same update on the snapshot
        t = opt.step_count
        b1, b2 = opt.param_groups[0]["betas"]
        ops.adam(p0, g0, m0, v0, n, 1e-3, b1, b2, 1e-8, 1 - b1 ** t, 1 - b2 ** t, 1.0)
        torch.cuda.synchronize()
        assert torch.equal(a.flat[:n], p0), step
        assert torch.equal(opt.m, m0), step
        assert torch.equal(opt.v, v0), step
        for name in tables:
            rows = a.row_flags[name]
            ever = int((rows & 1).ne(0).sum())
            assert 0 < touched[name] <= ever < rows.numel(), (name, touched[name], ever)
    # only the few touched rows carry state: the skipped part of the tables is the bulk
    for name in tables:
        assert int((a.row_flags[name] & 1).ne(0).sum()) < a.row_flags[name].numel() // 100


def test_untracked_tables_under_foreign_data_parallel_exchange_update_densely(monkeypatch):
    """With a multi-rank process group but no GradReducer (e.g. the model wrapped in torch
    DDP), the all-reduced table gradient has rows other ranks touched: Adam must not skip
    rows by the local flags -- it updates the tables densely and marks every row as holding
    state, so a later row-tracked step stays exact."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.distributed as dist
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    m = _model()
    opt = Adam(m, lr=1e-3)
    batch = synthetic_batch(4, Nv=6, Lq=5, Ns=8, topN=5, num_classes=12, seed=7, device="cuda")
    lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
    loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
    opt.zero_grad()
    loss.backward()
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_world_size", lambda *a, **k: 2)
    assert opt._row_tables(None) == ()
    a = m._arena
    # a row only another rank touched: the exchanged gradient is non-zero there
    for n in a.row_flags:
        o, shp = a.offsets[n]
        a.gview(n)[shp[0] - 1].fill_(0.25)
    opt.step()
    torch.cuda.synchronize()
    for f in a.row_flags.values():
        assert bool((f & 1).ne(0).all())
    # ... so the next zero_grad clears the whole table, not just the locally touched rows
    opt.zero_grad()
    torch.cuda.synchronize()
    assert int(torch.count_nonzero(a.grad)) == 0
