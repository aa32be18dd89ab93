"""Block-level API (savqa_amd.modules, mirror of models/modules.py) on the HIP path vs the
reference's golden vectors in tests/golden/blocks.npz."""
import os

import numpy as np
import pytest
import torch

from oracle import cases, hashfill

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.fixture(scope="module")
def G():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return np.load(os.path.join(GOLD, "blocks.npz"))


def mk(cls, name, *a, **k):
    m = cls(*a, **k)
    with torch.no_grad():
        for pn, p in m.named_parameters():
            p.copy_(torch.from_numpy(hashfill.param_value(f"{name}.{pn}", tuple(p.shape))))
    return m.cuda()


@pytest.mark.parametrize("T,gname", [(50, "rand"), (50, "diag"), (73, "rand"), (73, "ones")])
def test_new_multihead_attention(G, T, gname):
    from savqa_amd.modules import new_multihead_attention
    key = f"mha_T{T}_{gname}"
    x, graphs = cases.block_mha_inputs(T)
    m = mk(new_multihead_attention, f"blk.mha{T}", 512, 8, 0, False, True)
    xx = x.cuda().requires_grad_(True)
    out, att = m(xx, xx, xx, graphs[gname].cuda())
    assert rel(out.detach().cpu(), G[f"{key}:out"]) < 1e-4
    assert rel(att.cpu(), G[f"{key}:att"]) < 1e-4
    dout = torch.from_numpy(hashfill.fill(f"blk:dout:{T}:{gname}", out.shape, 1.0)).cuda()
    (out * dout).sum().backward()
    assert rel(xx.grad.cpu(), G[f"{key}:dx"]) < 1e-3
    for pn, p in m.named_parameters():
        ref = float(G[f"{key}:gsum:{pn}"])
        got = float(p.grad.double().sum())
        assert abs(got - ref) <= 1e-3 * max(1.0, float(p.grad.abs().sum())), pn


def test_cross_and_causal(G):
    from savqa_amd.modules import multihead_attention, new_multihead_attention
    m = mk(new_multihead_attention, "blk.cross", 512, 8, 0, False, True)
    q = torch.from_numpy(G["cross:q"]).cuda().requires_grad_(True)
    kv = torch.from_numpy(G["cross:kv"]).cuda().requires_grad_(True)
    out, att = m(q, kv, kv, torch.from_numpy(G["cross:dm"]).cuda())
    assert rel(out.detach().cpu(), G["cross:out"]) < 1e-4
    assert rel(att.cpu(), G["cross:att"]) < 1e-4
    (out * torch.from_numpy(G["cross:dout"]).cuda()).sum().backward()
    assert rel(q.grad.cpu(), G["cross:dq"]) < 1e-3
    assert rel(kv.grad.cpu(), G["cross:dkv"]) < 1e-3
    m = mk(multihead_attention, "blk.causal", 512, 8, 0, True)
    q = torch.from_numpy(G["cross:q"]).cuda().requires_grad_(True)
    out = m(q, q, q)
    assert rel(out.detach().cpu(), G["causal:out"]) < 1e-4
    (out * torch.from_numpy(G["cross:dout"]).cuda()).sum().backward()
    assert rel(q.grad.cpu(), G["causal:dq"]) < 1e-3
    assert float(m.Q_proj[0].weight.grad.abs().sum()) == 0.0


def test_layer_norm_and_feedforward(G):
    from savqa_amd.modules import feedforward, layer_normalization
    ln = mk(layer_normalization, "blk.ln", 512)
    x = torch.from_numpy(G["ln:x"]).cuda().requires_grad_(True)
    out = ln(x)
    assert rel(out.detach().cpu(), G["ln:out"]) < 1e-5
    (out * torch.from_numpy(G["ln:dout"]).cuda()).sum().backward()
    assert rel(x.grad.cpu(), G["ln:dx"]) < 1e-4
    assert rel(ln.gamma.grad.cpu(), G["ln:dgamma"]) < 1e-4
    assert rel(ln.beta.grad.cpu(), G["ln:dbeta"]) < 1e-4
    ff = mk(feedforward, "blk.ffn", 512, [2048, 512])
    x = torch.from_numpy(G["ln:x"]).cuda().requires_grad_(True)
    out = ff(x)
    assert rel(out.detach().cpu(), G["ffn:out"]) < 1e-4
    (out * torch.from_numpy(G["ln:dout"]).cuda()).sum().backward()
    assert rel(x.grad.cpu(), G["ffn:dx"]) < 1e-3
    assert rel(ff.conv2.bias.grad.cpu(), G["ffn:g:conv2.bias"]) < 1e-4
