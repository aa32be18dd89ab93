"""On-device batch collation (savqa_collate / savqa_collate_edges through
savqa_amd.collate) against the reference collate_fn: bit-exact on the golden cases
(tests/golden/collate.npz, produced by the reference itself), and against the oracle's
restatement at the full cfg-2 batch (B=256, 2048-d regions) and at the super-node
relation batch (T_syb = 1300 nodes, 31.5k relation entries per sample)."""
import os

import numpy as np
import pytest
import torch

from oracle import collate as ocol

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "collate.npz")
CASES = {"onlyobj": dict(B=9, relations=False, fea_dim=16, topN=5, tag="col"),
         "super_node": dict(B=10, relations=True, fea_dim=16, topN=3, tag="colrel")}


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _check(res, ref):
    assert list(res) == list(ref)
    for k, g in ref.items():
        t = res[k]
        assert t.is_cuda, k
        v = t.cpu().numpy()
        assert v.dtype == g.dtype and v.shape == g.shape, (k, v.dtype, g.dtype, v.shape, g.shape)
        assert np.array_equal(v, g), k


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("pinned", [False, True])
def test_device_collate_matches_reference_golden(name, pinned):
    _need_gpu()
    from savqa_amd.collate import pack, to_device
    gold = np.load(GOLD)
    pk = pack(ocol.make_samples(**CASES[name]))
    if pinned:
        pk.pin_memory()
    res = to_device(pk)
    torch.cuda.synchronize()
    ref = {k.split(":", 1)[1]: gold[k] for k in gold.files if k.startswith(name + ":")}
    _check(res, ref)


def test_device_collate_cfg2_batch():
    _need_gpu()
    from savqa_amd.collate import collate_fn
    from savqa_amd.data import synthetic_samples
    data = synthetic_samples(256, seed=11)
    data[3] = None  # the loader's failed-sample path (onlyobj:333-334)
    res = collate_fn(data)
    torch.cuda.synchronize()
    _check(res, ocol.collate_onlyobj(data))


def test_device_collate_super_node_batch():
    _need_gpu()
    from savqa_amd.collate import collate_fn
    from savqa_amd.data import synthetic_samples
    data = synthetic_samples(4, relations=True, Nv=(30, 36), seed=5)
    s = list(data[2])  # a sample without relations keeps padding rows only (super_node:434)
    for i in (6, 7, 8, 9):
        s[i] = s[i][:0]
    data[2] = tuple(s)
    res = collate_fn(data)
    torch.cuda.synchronize()
    assert res["macro_graph_ipt"].shape[1] >= 900
    _check(res, ocol.collate_super_node(data))


def test_staging_ring_reuses_pinned_buffers():
    _need_gpu()
    from savqa_amd.collate import StagingRing
    ring = StagingRing(2)
    batches = [ocol.make_samples(6, relations=r, fea_dim=32, topN=3, tag=f"ring{i}")
               for i, r in enumerate([False, False, True, False])]
    outs = [ring.collate(b) for b in batches]  # buffers 0,1 refilled after their copies
    torch.cuda.synchronize()
    assert all(b is not None and b.is_pinned() for b in ring.bufs)
    for b, res in zip(batches, outs):
        ref = (ocol.collate_super_node if len(b[0]) == 14 else ocol.collate_onlyobj)(b)
        _check(res, ref)


def test_device_collate_feeds_the_model():
    """collate -> AttModel.forward == forward on the host-collated batch (bit-exact)."""
    _need_gpu()
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.collate import collate_fn, forward_inputs
    from savqa_amd.utils import init_params_
    data = ocol.make_samples(5, fea_dim=2048, topN=5, tag="fm")
    m = AttModel(None, 256, 64, 914, 16, 80, 40, 2, 4, 0.0, 0.0, 2, True, device="cuda",
                 init=False)
    init_params_(m, seed=1)
    m.eval()
    ref = ocol.collate_onlyobj(data)
    host = {k: torch.from_numpy(v).cuda() for k, v in ref.items()}
    with torch.no_grad():
        a = m(*forward_inputs(collate_fn(data)), decMask=True, mcb=False)
        b = m(*forward_inputs(host), decMask=True, mcb=False)
    torch.cuda.synchronize()
    for x, y in zip(a[:4], b[:4]):
        assert torch.equal(x, y)


def test_to_device_refuses_host():
    from savqa_amd import _lib
    from savqa_amd.collate import pack, to_device
    pk = pack(ocol.make_samples(2, fea_dim=8, topN=3, tag="h"))
    with pytest.raises(_lib.SavqaError):
        to_device(pk, "cpu")
