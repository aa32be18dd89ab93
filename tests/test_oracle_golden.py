"""Pin the CPU oracle (oracle/savqa_oracle.py) against the reference's golden vectors.

tests/golden/*.npz were produced by tools/make_golden.py, which imported and ran
the reference (/root/reference/models) in the build container.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import cases, hashfill
from oracle import savqa_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _blocks():
    return np.load(os.path.join(GOLD, "blocks.npz"))


def _prefixed(prefix):
    class P(dict):
        def __missing__(self, k):
            name = k[len("m."):]
            raise KeyError(k)
    return P


def _block_params(name, shapes):
    return {f"m.{k}": torch.from_numpy(hashfill.param_value(f"{name}.{k}", s)).requires_grad_(True)
            for k, s in shapes.items()}


def _mha_shapes(d=512):
    s = {}
    for p in ("Q_proj", "K_proj", "V_proj"):
        s[f"{p}.0.weight"] = (d, d)
        s[f"{p}.0.bias"] = (d,)
    s["normalization.gamma"] = (d,)
    s["normalization.beta"] = (d,)
    return s


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


@pytest.mark.parametrize("T,gname", [(50, "rand"), (50, "diag"), (73, "rand"), (73, "ones")])
def test_graph_mha_block(T, gname):
    g = _blocks()
    key = f"mha_T{T}_{gname}"
    x, graphs = cases.block_mha_inputs(T)
    P = _block_params(f"blk.mha{T}", _mha_shapes())
    xx = x.clone().requires_grad_(True)
    out, att = O.graph_mha(P, "m", xx, xx, xx, graphs[gname], return_att=True)
    assert rel_err(out.detach(), g[f"{key}:out"]) < 1e-5
    assert rel_err(att.detach(), g[f"{key}:att"]) < 1e-5
    dout = torch.from_numpy(hashfill.fill(f"blk:dout:{T}:{gname}", out.shape, 1.0))
    (out * dout).sum().backward()
    assert rel_err(xx.grad, g[f"{key}:dx"]) < 1e-4
    for k, p in P.items():
        pn = k[2:]
        ref_sum = float(g[f"{key}:gsum:{pn}"])
        assert abs(float(p.grad.double().sum()) - ref_sum) <= 1e-4 * max(1.0, abs(ref_sum)) + 1e-3


def test_cross_and_causal_blocks():
    g = _blocks()
    P = _block_params("blk.cross", _mha_shapes())
    q = torch.from_numpy(g["cross:q"]).requires_grad_(True)
    kv = torch.from_numpy(g["cross:kv"]).requires_grad_(True)
    out, att = O.graph_mha(P, "m", q, kv, kv, torch.from_numpy(g["cross:dm"]), return_att=True)
    assert rel_err(out.detach(), g["cross:out"]) < 1e-5
    (out * torch.from_numpy(g["cross:dout"])).sum().backward()
    assert rel_err(q.grad, g["cross:dq"]) < 1e-4
    assert rel_err(kv.grad, g["cross:dkv"]) < 1e-4
    P = _block_params("blk.causal", _mha_shapes())
    q = torch.from_numpy(g["cross:q"]).requires_grad_(True)
    out = O.causal_mha(P, "m", q, q, q)
    assert rel_err(out.detach(), g["causal:out"]) < 1e-5
    (out * torch.from_numpy(g["cross:dout"])).sum().backward()
    assert rel_err(q.grad, g["causal:dq"]) < 1e-4
    assert float(P["m.Q_proj.0.weight"].grad.abs().sum()) == float(g["causal:gQ"]) == 0.0


def test_ln_ffn_blocks():
    g = _blocks()
    x = torch.from_numpy(g["ln:x"]).requires_grad_(True)
    gam = torch.from_numpy(hashfill.param_value("blk.ln.gamma", (512,))).requires_grad_(True)
    bet = torch.from_numpy(hashfill.param_value("blk.ln.beta", (512,))).requires_grad_(True)
    out = O.layer_norm(x, gam, bet)
    assert rel_err(out.detach(), g["ln:out"]) < 1e-6
    (out * torch.from_numpy(g["ln:dout"])).sum().backward()
    assert rel_err(x.grad, g["ln:dx"]) < 1e-5
    assert rel_err(gam.grad, g["ln:dgamma"]) < 1e-5
    P = {f"m.{k}": torch.from_numpy(hashfill.param_value(f"blk.ffn.{k}", s)).requires_grad_(True)
         for k, s in {"conv1.0.weight": (2048, 512), "conv1.0.bias": (2048,), "conv2.weight": (512, 2048),
                      "conv2.bias": (512,), "normalization.gamma": (512,), "normalization.beta": (512,)}.items()}
    x = torch.from_numpy(g["ln:x"]).requires_grad_(True)
    out = O.feedforward(P, "m", x)
    assert rel_err(out.detach(), g["ffn:out"]) < 1e-5
    (out * torch.from_numpy(g["ln:dout"])).sum().backward()
    assert rel_err(x.grad, g["ffn:dx"]) < 1e-4
    assert rel_err(P["m.conv2.bias"].grad, g["ffn:g:conv2.bias"]) < 1e-5


def test_state_dict_keys_match_oracle_table():
    ref = json.load(open(os.path.join(GOLD, "state_dict_keys.json")))
    mine = O.model_param_shapes(num_relations=ref["num_relations"])
    assert [(k, list(s)) for k, s in mine] == [tuple(x) for x in ref["keys"]] or \
        [[k, list(s)] for k, s in mine] == ref["keys"]


@pytest.mark.slow
@pytest.mark.parametrize("case", ["full_b4", "full_b2_nodec"])
def test_full_model_forward_loss_grads(case):
    g = np.load(os.path.join(GOLD, f"{case}.npz"))
    P = hashfill.HashParams(requires_grad=True)
    inp = {k: torch.from_numpy(g[k]) for k in
           ("vis_fea", "vis_mask", "q_ipt", "q_mask", "q_graph", "macro_ipt", "macro_mask",
            "macro_graph", "macro_obj_loc", "micro_positive_obj", "micro_negative_obj",
            "micro_obj_mask", "answer")}
    lc, lv, ls, mil, _ = O.attmodel_forward(P, inp, decMask=bool(g["decMask"]))
    assert rel_err(lc.detach(), g["logits_concat"]) < 1e-5
    assert rel_err(lv.detach(), g["logits_vis"]) < 1e-5
    assert rel_err(ls.detach(), g["logits_syb"]) < 1e-5
    assert abs(float(mil) - float(g["mil_nce_obj"])) < 1e-5 * max(1, abs(float(g["mil_nce_obj"])))
    loss, _ = O.train_loss(lc, lv, ls, inp["answer"], mil)
    assert abs(float(loss) - float(g["loss"])) < 1e-5 * abs(float(g["loss"]))
    loss.backward()
    names = [str(n) for n in g["grad_names"]]
    for n in names:
        gr = P[n].grad
        assert gr is not None, n
        flat = gr.reshape(-1)
        idx = torch.from_numpy(g[f"g:{n}:idx"])
        ref = g[f"g:{n}:val"]
        scale = max(float(g[f"g:{n}:abssum"]) / flat.numel() * 50, np.abs(ref).max(), 1e-12)
        assert np.abs(flat[idx].detach().numpy() - ref).max() <= 2e-4 * scale, n
        assert abs(float(flat.double().sum()) - float(g[f"g:{n}:sum"])) <= 1e-4 * max(float(g[f"g:{n}:abssum"]), 1e-9), n
    # params that get no grad in the reference get none here either
    with_grad = {k for k, v in P.items() if v.grad is not None and k in P.shapes}
    assert with_grad == set(names)


REL_INPUTS = ("vis_fea", "vis_mask", "q_ipt", "q_mask", "q_graph", "macro_ipt", "macro_mask",
              "macro_graph", "macro_obj_loc", "micro_positive_obj", "micro_negative_obj",
              "micro_obj_mask", "micro_positive_rel", "micro_negative_rel",
              "micro_positive_rel_loc", "micro_negative_rel_loc", "answer")


@pytest.mark.slow
@pytest.mark.parametrize("case", ["full_rel_b2", "full_rel_sn", "full_rel_big"])
def test_relation_branch_full_model(case):
    """MIL-NCE relation branch (only_obj=False, AttModel_x3.py:382-437) end to end: logits,
    mil_nce_obj, mil_nce_rel, loss and every trained gradient (R included) against the
    reference run on super-node batches (tests/golden/full_rel_{b2,sn,big}.npz; sn: T_syb=211;
    big: the reference's relation configuration, hidden_size_mil 64 / maxlen 1600 / 311
    categories, T_syb=1313, ~6k listed relations)."""
    g = np.load(os.path.join(GOLD, f"{case}.npz"))
    geo = {k: int(g[k]) for k in ("hidden_mil", "maxlen") if k in g}
    P = hashfill.HashParams(requires_grad=True, num_relations=int(g["num_relations"]), **geo)
    inp = {k: torch.from_numpy(g[k]) for k in REL_INPUTS}
    lc, lv, ls, mil, mil_rel = O.attmodel_forward(P, inp, decMask=True, only_obj=False)
    assert rel_err(lc.detach(), g["logits_concat"]) < 1e-5
    assert rel_err(ls.detach(), g["logits_syb"]) < 1e-5
    assert abs(float(mil_rel) - float(g["mil_nce_rel"])) < 1e-5 * max(1, abs(float(g["mil_nce_rel"])))
    loss, _ = O.train_loss(lc, lv, ls, inp["answer"], mil, mil_nce_rel=mil_rel)
    assert abs(float(loss) - float(g["loss"])) < 1e-5 * abs(float(g["loss"]))
    loss.backward()
    names = [str(n) for n in g["grad_names"]]
    assert "MIL_NCE.R" in names
    for n in names:
        gr = P[n].grad
        assert gr is not None, n
        flat = gr.reshape(-1)
        idx = torch.from_numpy(g[f"g:{n}:idx"])
        ref = g[f"g:{n}:val"]
        scale = max(float(g[f"g:{n}:abssum"]) / flat.numel() * 50, np.abs(ref).max(), 1e-12)
        assert np.abs(flat[idx].detach().numpy() - ref).max() <= 2e-4 * scale, n
        assert abs(float(flat.double().sum()) - float(g[f"g:{n}:sum"])) <= \
            1e-4 * max(float(g[f"g:{n}:abssum"]), 1e-9), n
    used = torch.from_numpy(g["R_used"])
    assert rel_err(P["MIL_NCE.R"].grad[used, :4].detach(), g["R_grad_used"]) < 1e-4
