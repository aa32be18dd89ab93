#!/usr/bin/env python
"""Generate golden vectors by importing and running the REFERENCE (build container only).

Runs /root/reference/models/{modules.py, AttModel_x3.py} on CPU with the harness
shims of SURVEY.md section 8(c) (the reference files are never modified, no
bytecode is written under /root/reference):
  (1) torch.Tensor.cuda -> identity (hard-coded .cuda() calls),
  (2) construction under torch.no_grad() (in-place writes into leaf Parameters),
  (3) glove = SimpleNamespace(vectors=...) (torchtext absent),
  (4) dropout_rate = 0 (ReLU -> inplace Dropout backward error on torch 2.x),
  (5) mcb=False (torch.rfft removed).
All weights and inputs come from oracle/hashfill.py, so no weights are committed.
The loss / Adam step restate main_itp_ddp_tar_super_node.py:335-366 inline here
because that file imports azureml (not installed) and cannot be imported.

Outputs (committed): tests/golden/*.npz and tests/golden/state_dict_keys.json.
No-op when /root/reference is absent (e.g. on the GPU box).
"""
from __future__ import annotations

import json
import os
import sys
import types

sys.dont_write_bytecode = True
REF = "/root/reference/models"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import cases, hashfill  # noqa: E402

torch.Tensor.cuda = lambda self, *a, **k: self  # shim (1)
torch.set_num_threads(os.cpu_count() or 8)

# geometry of the parity cases (cfg 1 shapes; num_relations kept small: R/bilinear are
# dead in only_obj mode and only their shapes enter the state_dict)
CFG = dict(hidden=512, hidden_mil=1024, num_classes=914, maxlen_q=40, maxlen=450,
           maxlen_v=49, num_blocks=6, heads=8, num_relations=4)


def n_sample(name, n, k=24):
    return np.unique(hashfill.randint("sample:" + name, (k,), 0, n))


def grad_digest(name, g: torch.Tensor):
    """Compact digest of a gradient: sums + sampled entries (+ touched rows for tables)."""
    flat = g.detach().reshape(-1).double()
    idx = n_sample(name, flat.numel())
    d = {"sum": float(flat.sum()), "abssum": float(flat.abs().sum()),
         "idx": idx.astype(np.int64), "val": flat[idx].float().numpy()}
    return d


make_inputs = cases.make_inputs

def fill_params(model):
    with torch.no_grad():
        for name, p in model.named_parameters():
            p.copy_(torch.from_numpy(hashfill.param_value(name, tuple(p.shape))))
        for name, b in model.named_buffers():
            pass


def ref_loss(lc, lv, ls, answer, mil_obj, eps=0.1, mil_rel=0):
    # main_itp_ddp_tar_super_node.py:335-361 (with_smooth_labeling, with_MILNCE_loss)
    lsm = (F.log_softmax(lv, -1) + F.log_softmax(ls, -1) + F.log_softmax(lc, -1)) / 3
    oh = torch.zeros((lc.size(0), lc.size(1)))
    oh.scatter_(1, answer.view(-1, 1), 1)
    oh = ((1 - eps) * oh) + (eps / oh.size(-1))
    loss = -(oh * lsm).sum(-1)
    loss = loss.mean()
    loss = loss + (-mil_obj - mil_rel)  # main:326-329 (mil_rel = 0 when only_obj)
    return loss


def to_t(inp):
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in inp.items()}


def full_model_cases(modules_mod, att_mod):
    glove = types.SimpleNamespace(vectors=torch.zeros(8, 300))
    with torch.no_grad():
        model = att_mod.AttModel(glove, CFG["hidden"], CFG["hidden_mil"], CFG["num_classes"],
                                 CFG["maxlen_q"], CFG["maxlen"], CFG["maxlen_v"],
                                 CFG["num_blocks"], CFG["heads"], 0.0, 0.0,
                                 CFG["num_relations"], True)
    model.train()
    keys = [(k, list(v.shape)) for k, v in model.state_dict().items()]
    with open(os.path.join(OUT, "state_dict_keys.json"), "w") as f:
        json.dump({"num_relations": CFG["num_relations"], "keys": keys}, f)
    print("state_dict keys:", len(keys))
    fill_params(model)

    runs = {
        "full_b4": dict(B=4, Nv=[36, 30, 22, 36], Lq=[14, 9, 12, 6], Ns=[59, 40, 31, 50], decMask=True),
        "full_b2_nodec": dict(B=2, Nv=[36, 17], Lq=[14, 11], Ns=[59, 23], decMask=False),
    }
    for cname, c in runs.items():
        inp = make_inputs(c["B"], c["Nv"], c["Lq"], c["Ns"], tag=cname)
        t = to_t(inp)
        empty = torch.empty((c["B"], 0))
        fill_params(model)
        opt = torch.optim.Adam(model.parameters(), 1e-4)

        def fwd():
            return model(t["vis_fea"], t["vis_mask"], t["q_ipt"], t["q_mask"], t["q_graph"],
                         t["macro_ipt"], t["macro_mask"], t["macro_graph"], t["macro_obj_loc"],
                         t["micro_positive_obj"], t["micro_negative_obj"], t["micro_obj_mask"],
                         empty, empty, empty, empty, decMask=c["decMask"], mcb=False)

        lc, lv, ls, mil, _ = fwd()
        loss = ref_loss(lc, lv, ls, t["answer"], mil)
        opt.zero_grad()
        loss.backward()
        out = dict(inp)
        out.update(logits_concat=lc.detach().numpy(), logits_vis=lv.detach().numpy(),
                   logits_syb=ls.detach().numpy(), mil_nce_obj=np.float32(mil.item()),
                   loss=np.float32(loss.item()), decMask=np.int32(c["decMask"]))
        gnames = []
        for name, p in model.named_parameters():
            if p.grad is None:
                continue
            gnames.append(name)
            d = grad_digest(name, p.grad)
            out[f"g:{name}:sum"] = np.float64(d["sum"])
            out[f"g:{name}:abssum"] = np.float64(d["abssum"])
            out[f"g:{name}:idx"] = d["idx"]
            out[f"g:{name}:val"] = d["val"]
            if name.endswith("syb_emb.weight"):
                rows = np.unique(np.concatenate([inp["q_ipt"].ravel(), inp["micro_negative_obj"].ravel()]))
                rows = rows[:12]
                out[f"g:{name}:rows"] = rows
                out[f"g:{name}:rowval"] = p.grad[torch.from_numpy(rows)].numpy()
        out["grad_names"] = np.array(gnames)
        # two Adam steps: logits after each (exercises loss->backward->Adam end to end)
        opt.step()
        for s in (1, 2):
            lc, lv, ls, mil, _ = fwd()
            out[f"step{s}_logits_concat"] = lc.detach().numpy()
            out[f"step{s}_mil"] = np.float32(mil.item())
            if s == 1:
                loss = ref_loss(lc, lv, ls, t["answer"], mil)
                opt.zero_grad()
                loss.backward()
                opt.step()
        np.savez_compressed(os.path.join(OUT, f"{cname}.npz"), **out)
        print("wrote", cname, "loss", float(out["loss"]))
    del model


# relation-branch cases: (objects per sample, question lengths, options). full_rel_sn has a
# super-node graph of T_syb = 14 + 3 + 14*13 + 12 = 211 > 128 positions, so the key-tiled
# attention (csrc/attn_flash.hip) runs inside the semantic stack of the parity case.
# full_rel_big is the reference's own relation configuration (submit.py:87 maxlen 1600,
# :101 hidden_size_mil 64) at the benched super-node size: B = 2 (the reference squeezes a
# B = 1 batch away at AttModel_x3.py:540), 36 objects -> T_syb = 36 + 3 +
# 36*35 + 14 = 1313 positions, 311 relation categories, up to 8 listed relations per object
# pair (~5.7k positive entries), 6 encoder/decoder blocks (the reference hard-codes 6 in its
# forwards, AttModel_x3.py:127-139; its per-entry Python loop :421-436 dominates the CPU time).
RELATION_RUNS = {"full_rel_b2": ([5, 4], [7, 5], {}),
                 "full_rel_sn": ([14, 11], [12, 9], {}),
                 "full_rel_big": ([36, 9], [14, 10], dict(hidden_mil=64, num_blocks=6, nrel=311,
                                                   max_rel_per_pair=8, maxlen=1600))}


def relation_cases(att_mod, only=None):
    for cname, (nobj, lq, opt) in RELATION_RUNS.items():
        if only is None or cname in only:
            relation_case(att_mod, cname, nobj, lq, **opt)


def relation_case(att_mod, cname, nobj, lq, hidden_mil=None, num_blocks=None, nrel=7,
                  max_rel_per_pair=2, maxlen=None):
    """Full model with the MIL-NCE relation branch (only_obj=False, AttModel_x3.py:382-437)
    on a super-node batch (oracle/cases.make_relation_inputs)."""
    import time
    hidden_mil = hidden_mil or CFG["hidden_mil"]
    num_blocks = num_blocks or CFG["num_blocks"]
    maxlen = maxlen or CFG["maxlen"]
    glove = types.SimpleNamespace(vectors=torch.zeros(8, 300))
    with torch.no_grad():
        model = att_mod.AttModel(glove, CFG["hidden"], hidden_mil, CFG["num_classes"],
                                 CFG["maxlen_q"], maxlen, CFG["maxlen_v"], num_blocks, CFG["heads"],
                                 0.0, 0.0, nrel, False)
    model.train()
    fill_params(model)
    tag = "relcase" if cname == "full_rel_b2" else cname
    inp = cases.make_relation_inputs(len(nobj), nobj, lq, nrel, tag=tag,
                                     max_rel_per_pair=max_rel_per_pair)
    t0 = time.time()
    t = to_t(inp)
    lc, lv, ls, mil, mil_rel = model(
        t["vis_fea"], t["vis_mask"], t["q_ipt"], t["q_mask"], t["q_graph"], t["macro_ipt"],
        t["macro_mask"], t["macro_graph"], t["macro_obj_loc"], t["micro_positive_obj"],
        t["micro_negative_obj"], t["micro_obj_mask"], t["micro_positive_rel"],
        t["micro_negative_rel"], t["micro_positive_rel_loc"], t["micro_negative_rel_loc"],
        decMask=True, mcb=False)
    loss = ref_loss(lc, lv, ls, t["answer"], mil, mil_rel=mil_rel)
    model.zero_grad()
    loss.backward()
    out = dict(inp)
    out.update(logits_concat=lc.detach().numpy(), logits_vis=lv.detach().numpy(),
               logits_syb=ls.detach().numpy(), mil_nce_obj=np.float32(mil.item()),
               mil_nce_rel=np.float32(mil_rel.item()), loss=np.float32(loss.item()),
               num_relations=np.int32(nrel), num_blocks=np.int32(num_blocks),
               hidden_mil=np.int32(hidden_mil), maxlen=np.int32(maxlen))
    gnames = []
    for name, p in model.named_parameters():
        if p.grad is None:
            continue
        gnames.append(name)
        d = grad_digest(name, p.grad)
        out[f"g:{name}:sum"] = np.float64(d["sum"])
        out[f"g:{name}:abssum"] = np.float64(d["abssum"])
        out[f"g:{name}:idx"] = d["idx"]
        out[f"g:{name}:val"] = d["val"]
    # R: the used categories' slices in full (sparse gradient)
    used = np.unique(np.concatenate([inp["micro_positive_rel_loc"][..., 2].ravel(),
                                     inp["micro_negative_rel_loc"][..., 2].ravel()]))
    used = used[used >= 0]
    out["R_used"] = used
    out["R_grad_used"] = model.MIL_NCE.R.grad[torch.from_numpy(used), :4].numpy()  # 4 rows each
    out["grad_names"] = np.array(gnames)
    np.savez_compressed(os.path.join(OUT, f"{cname}.npz"), **out)
    print("wrote", cname, "T_syb", inp["macro_ipt"].shape[1] + inp["q_ipt"].shape[1], "loss",
          float(out["loss"]), "mil_rel", float(out["mil_nce_rel"]), "entries",
          int((inp["micro_positive_rel_loc"][..., 3] >= 0).sum()), f"{time.time() - t0:.1f}s")
    del model


def block_cases(modules_mod):
    out = {}
    torch.manual_seed(0)
    d = 512

    def mk(cls, name, *a, **k):
        m = cls(*a, **k)
        with torch.no_grad():
            for pn, p in m.named_parameters():
                p.copy_(torch.from_numpy(hashfill.param_value(f"{name}.{pn}", tuple(p.shape))))
        return m

    # encoder self-attention, several graph patterns
    for T, gnames in ((50, ("rand", "diag")), (73, ("rand", "ones"))):
        x, graphs = cases.block_mha_inputs(T)
        m = mk(modules_mod.new_multihead_attention, f"blk.mha{T}", d, 8, 0, False, True)
        for gname in gnames:
            g = graphs[gname]
            xx = x.clone().requires_grad_(True)
            o, att = m(xx, xx, xx, g)
            dout = torch.from_numpy(hashfill.fill(f"blk:dout:{T}:{gname}", o.shape, 1.0))
            m.zero_grad()
            (o * dout).sum().backward()
            key = f"mha_T{T}_{gname}"
            out[f"{key}:out"] = o.detach().numpy()
            out[f"{key}:att"] = att.detach().numpy()
            out[f"{key}:dx"] = xx.grad.numpy()
            for pn, p in m.named_parameters():
                out[f"{key}:g:{pn}"] = p.grad.numpy().copy() if p.grad.numel() <= 1024 else \
                    p.grad.numpy()[:4].copy()
                out[f"{key}:gsum:{pn}"] = np.float64(p.grad.double().sum())

    # decoder cross attention (T_q = 1) with a dec_mask that has zeros
    B, T = 3, 73
    q = torch.from_numpy(hashfill.fill("blk:xq", (B, 1, d), 1.0))
    kv = torch.from_numpy(hashfill.fill("blk:kv", (B, T, d), 1.0))
    dm = torch.from_numpy(hashfill.bernoulli("blk:dm", (B, 1, T), 0.7)).float()
    dm[2] = 0.0  # a sample whose decoder attends to nothing
    m = mk(modules_mod.new_multihead_attention, "blk.cross", d, 8, 0, False, True)
    qq = q.clone().requires_grad_(True)
    kk = kv.clone().requires_grad_(True)
    o, att = m(qq, kk, kk, dm)
    dout = torch.from_numpy(hashfill.fill("blk:cross:dout", o.shape, 1.0))
    (o * dout).sum().backward()
    out.update({"cross:q": q.numpy(), "cross:kv": kv.numpy(), "cross:dm": dm.numpy(),
                "cross:out": o.detach().numpy(), "cross:att": att.detach().numpy(),
                "cross:dout": dout.numpy(), "cross:dq": qq.grad.numpy(), "cross:dkv": kk.grad.numpy()})

    # decoder causal self-attention, T = 1
    m = mk(modules_mod.multihead_attention, "blk.causal", d, 8, 0, True)
    qq = q.clone().requires_grad_(True)
    o = m(qq, qq, qq)
    (o * dout).sum().backward()
    out.update({"causal:out": o.detach().numpy(), "causal:dq": qq.grad.numpy(),
                "causal:gQ": np.float64(m.Q_proj[0].weight.grad.abs().sum()),
                "causal:gV": np.float64(m.V_proj[0].weight.grad.double().sum())})

    # layer norm and feed-forward
    x = torch.from_numpy(hashfill.fill("blk:lnx", (4, 7, d), 2.0, 0.3))
    ln = mk(modules_mod.layer_normalization, "blk.ln", d)
    xx = x.clone().requires_grad_(True)
    o = ln(xx)
    dout = torch.from_numpy(hashfill.fill("blk:ln:dout", o.shape, 1.0))
    (o * dout).sum().backward()
    out.update({"ln:x": x.numpy(), "ln:out": o.detach().numpy(), "ln:dout": dout.numpy(),
                "ln:dx": xx.grad.numpy(), "ln:dgamma": ln.gamma.grad.numpy(), "ln:dbeta": ln.beta.grad.numpy()})
    ff = mk(modules_mod.feedforward, "blk.ffn", d, [4 * d, d])
    xx = x.clone().requires_grad_(True)
    o = ff(xx)
    (o * dout).sum().backward()
    out.update({"ffn:out": o.detach().numpy(), "ffn:dx": xx.grad.numpy(),
                "ffn:g:conv1.0.bias": ff.conv1[0].bias.grad.numpy(),
                "ffn:g:conv2.bias": ff.conv2.bias.grad.numpy(),
                "ffn:gsum:conv1.0.weight": np.float64(ff.conv1[0].weight.grad.double().sum())})
    np.savez_compressed(os.path.join(OUT, "blocks.npz"), **out)
    print("wrote blocks.npz")


COLLATE_CASES = {"onlyobj": dict(B=9, relations=False, fea_dim=16, topN=5, tag="col"),
                 "super_node": dict(B=10, relations=True, fea_dim=16, topN=3, tag="colrel")}


def collate_cases():
    """Reference collate_fn outputs (onlyobj:341-445, super_node:366-497) on the
    oracle/collate.py sample recipe -> tests/golden/collate.npz."""
    from oracle import collate as ocol
    sys.path.insert(0, os.path.join(os.path.dirname(REF), "dataloader"))
    import data_loader_itp_bbox_super_node_onlyobj as onlyobj_mod  # noqa: E402  (reference)
    import data_loader_itp_bbox_super_node as super_mod  # noqa: E402  (reference)
    out = {}
    for name, kw in COLLATE_CASES.items():
        data = ocol.make_samples(**kw)
        fn = super_mod.collate_fn if kw["relations"] else onlyobj_mod.collate_fn
        res = fn(data)
        for k, v in res.items():
            out[f"{name}:{k}"] = v.numpy()
    np.savez_compressed(os.path.join(OUT, "collate.npz"), **out)
    print("wrote collate.npz")


READER_CASES = {"loc_top5": dict(with_loc=True, pred_rel=False, topN=5),
                "noloc_pred_top3": dict(with_loc=False, pred_rel=True, topN=3),
                "rel_loc_top3": dict(with_loc=True, pred_rel=False, topN=3, rel=True),
                "rel_noloc_top2": dict(with_loc=False, pred_rel=False, topN=2, rel=True)}


def reader_cases():
    """Reference GQADataset_super_node (onlyobj:41-334) items on the synthetic GQA files of
    oracle/gqa_fixture.py, python `random` seeded per item -> tests/golden/gqa_reader.npz."""
    import random
    import tempfile
    from oracle import gqa_fixture as fx
    import data_loader_itp_bbox_super_node_onlyobj as onlyobj_mod  # noqa: E402  (reference)
    sys.path.insert(0, os.path.join(os.path.dirname(REF), "dataloader"))
    import data_loader_itp_bbox_super_node as super_mod  # noqa: E402  (reference)
    # the relation loader's category order is python's set order (PYTHONHASHSEED)
    assert os.environ.get("PYTHONHASHSEED") == "0", "run with PYTHONHASHSEED=0"
    out = {"hashseed": np.int64(0)}
    with tempfile.TemporaryDirectory() as root:
        fx.write_dataset(root)
        for name, kw in READER_CASES.items():
            mod = super_mod if kw.get("rel") else onlyobj_mod
            fields = fx.ITEM_FIELDS_REL if kw.get("rel") else fx.ITEM_FIELDS
            ds = mod.GQADataset_super_node(
                "train", fx.Opt(root, pred_rel=kw["pred_rel"]), "gt_bua_npz.tar", "train.tar",
                "gt_bua_npz.tar", kw["topN"], with_loc=kw["with_loc"])
            out[f"{name}:len"] = np.int64(len(ds))
            for i in range(len(ds)):
                random.seed(1000 + i)
                item = ds[i]
                out[f"{name}:{i}:none"] = np.bool_(item is None)
                if item is None:
                    continue
                for f, v in zip(fields, item):
                    out[f"{name}:{i}:{f}"] = np.asarray(v)
    np.savez_compressed(os.path.join(OUT, "gqa_reader.npz"), **out)
    print("wrote gqa_reader.npz", len(out))


def main():
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return
    os.makedirs(OUT, exist_ok=True)
    sys.path.insert(0, REF)
    import modules as modules_mod  # noqa: E402  (reference)
    import AttModel_x3 as att_mod  # noqa: E402  (reference)
    which = sys.argv[1:] or ["blocks", "full"]
    if "blocks" in which:
        block_cases(modules_mod)
    if "full" in which:
        full_model_cases(modules_mod, att_mod)
    if "rel" in which:
        relation_cases(att_mod)
    if "rel_big" in which:  # only the large relation case (minutes of reference CPU time)
        relation_cases(att_mod, only=("full_rel_big",))
    if "collate" in which:
        collate_cases()
    if "reader" in which:
        reader_cases()


if __name__ == "__main__":
    main()
