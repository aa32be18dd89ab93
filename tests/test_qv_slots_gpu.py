"""The pruned encoder layers 0-1 keep persistent Q|V buffers (engine._zeroed_qv). Their node
rows must read as exact zeros for every batch layout: a batch with the same B*T rows but a
different (Nn, Lq) split must not see the previous batch's question rows, and two forwards in
flight must not share a buffer. Both are checked bit-exactly against a model whose buffers are
fresh (same weights, same batch, same kernels)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model():
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.utils import init_params_
    m = AttModel(None, 512, 1024, 914, 40, 450, 49, 6, 8, 0.0, 0.0, 4, True, device="cuda",
                 init=False)
    init_params_(m, seed=3)
    m.train()
    return m


def _fwd(m, batch):
    from savqa_amd.data import model_args
    return m(*model_args(batch), decMask=True, mcb=False)


def test_layout_change_and_two_forwards_in_flight():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from savqa_amd import engine
    from savqa_amd.data import synthetic_batch
    # same rows per stack (T_vis = 34, T_syb = 44), other (Nn, Lq) split
    a = synthetic_batch(4, Nv=20, Lq=14, Ns=30, seed=11)
    b = synthetic_batch(4, Nv=24, Lq=10, Ns=34, seed=12)
    fresh = _model()
    ref_b = [t.clone() for t in _fwd(fresh, b)[:3]]
    ref_a = [t.clone() for t in _fwd(_model(), a)[:3]]
    del fresh
    m = _model()
    out_a = _fwd(m, a)
    sum(o.sum() for o in out_a[:3]).backward()       # releases a's slots
    out_b = _fwd(m, b)                                # reuses them: re-zeroed
    for x, y in zip(out_b[:3], ref_b):
        assert torch.equal(x, y)
    out_a2 = _fwd(m, a)                               # b still in flight: other slots
    for x, y in zip(out_a2[:3], ref_a):
        assert torch.equal(x, y)
    for x, y in zip(out_b[:3], ref_b):                # b's outputs untouched
        assert torch.equal(x, y)
    slots = [L.get("_qv", []) for L in m._engine.vis.enc[:2]] if hasattr(m._engine, "vis") \
        else []
    assert all(len(s) <= engine._QV_SLOTS for s in slots)
