"""TEST INFRASTRUCTURE ONLY -- shared recipes for parity-case inputs.

Used by tools/make_golden.py (reference side) and tests/ (HIP side) so both see
the same inputs; the fixtures in tests/golden/ hold the reference's outputs.
"""
from __future__ import annotations

import numpy as np
import torch

from . import hashfill


def make_inputs(B, Nv_list, Lq_list, Ns_list, Nv_max=36, Lq_max=14, Ns_max=59, topN=5,
                num_classes=914, tag="full"):
    """Ragged synthetic batch padded exactly like collate_fn
    (models/data_loader_itp_bbox_super_node_onlyobj.py:341-445)."""
    PAD, LOC_PAD = 400000, -1
    vis = np.zeros((B, Nv_max, 2048), np.float32)
    vis_mask = np.zeros((B, Nv_max, Nv_max), np.int32)
    macro = np.full((B, Ns_max), PAD, np.int64)
    macro_mask = np.zeros((B, Ns_max, Ns_max), np.int32)
    macro_graph = np.zeros((B, Ns_max, Ns_max), np.int32)
    loc = np.full((B, Nv_max), LOC_PAD, np.int64)
    pos = np.full((B, Nv_max, topN), PAD, np.int64)
    neg = np.full((B, Nv_max, topN), PAD, np.int64)
    omask = np.zeros((B, Nv_max, topN), np.int32)
    q = np.full((B, Lq_max), PAD, np.int64)
    q_mask = np.zeros((B, Lq_max, Lq_max), np.int32)
    q_graph = np.zeros((B, Lq_max, Lq_max), np.int32)
    for b in range(B):
        nv, lq, ns = Nv_list[b], Lq_list[b], Ns_list[b]
        f = hashfill.fill(f"{tag}:vis:{b}", (nv, 2048), 1.0, 0.0)
        vis[b, :nv] = np.maximum(f, 0)  # pooled RCNN features are non-negative
        vis_mask[b, :nv, :nv] = 1
        macro[b, :ns] = hashfill.randint(f"{tag}:macro:{b}", (ns,), 0, 400000)
        macro_mask[b, :ns, :ns] = 1
        macro_graph[b, :ns, :ns] = hashfill.bernoulli(f"{tag}:mg:{b}", (ns, ns), 0.08)
        nobj = min(nv, ns)
        perm = np.argsort(hashfill.uniform_bits(f"{tag}:loc:{b}", ns))[:nobj]
        loc[b, :nobj] = perm
        pos[b, :nobj] = hashfill.randint(f"{tag}:pos:{b}", (nobj, topN), 0, 407000)
        neg[b, :nobj] = hashfill.randint(f"{tag}:neg:{b}", (nobj, topN), 0, 407000)
        omask[b, :nobj] = 1
        q[b, :lq] = hashfill.randint(f"{tag}:q:{b}", (lq,), 0, 400000)
        q_mask[b, :lq, :lq] = 1
        q_graph[b, :lq, :lq] = hashfill.bernoulli(f"{tag}:qg:{b}", (lq, lq), 0.25)
    answer = hashfill.randint(f"{tag}:ans", (B,), 1, num_classes)
    return dict(vis_fea=vis, vis_mask=vis_mask, q_ipt=q, q_mask=q_mask, q_graph=q_graph,
                macro_ipt=macro, macro_mask=macro_mask, macro_graph=macro_graph,
                macro_obj_loc=loc, micro_positive_obj=pos, micro_negative_obj=neg,
                micro_obj_mask=omask, answer=answer)



def block_mha_inputs(T, B=2, d=512):
    """Inputs of the block-level graph-MHA cases (x, graph patterns)."""
    x = torch.from_numpy(hashfill.fill(f"blk:x:{T}", (B, T, d), 1.0))
    graphs = {
        "rand": torch.from_numpy(hashfill.bernoulli(f"blk:g:{T}", (B, T, T), 0.3)).float(),
        "diag": torch.zeros(B, T, T),
        "ones": torch.ones(B, T, T),
    }
    graphs["diag"][:, T - 14:, T - 14:] = 1.0
    # exact-zero feature rows exercise the key/query masks (modules.py:257, :289)
    x[1, 3] = 0.0
    x[0, T - 1] = 0.0
    return x, graphs


def make_relation_inputs(B, nobj_list, Lq_list, num_relations, topN=3, Nv_max=None,
                         num_classes=914, tag="rel", max_rel_per_pair=2, n_attr=3):
    """Super-node batch with relation tensors, laid out like the relation loader
    (dataloader/data_loader_itp_bbox_super_node.py:150-252, collate :366-497): macro
    nodes = object nodes, a few attribute nodes, one empty relation node per ordered
    object pair (i != j); per pair 1..max_rel_per_pair positive entries
    [obj_i, obj_j, rel_category, macro_rel_loc, micro_rel_loc] with micro_rel_loc a
    per-sample running counter (:208-237) and as many negatives [i, j, r, macro_rel_loc]
    (:241-246); padding rows are LOC_PAD = -1, padding ids PAD."""
    PAD, LOC_PAD = 400000, -1
    Nv_max = Nv_max or max(nobj_list)
    Ns_list = [n + n_attr + n * (n - 1) for n in nobj_list]
    inp = make_inputs(B, [min(n, Nv_max) for n in nobj_list], Lq_list, Ns_list, Nv_max=Nv_max,
                      Lq_max=max(Lq_list), Ns_max=max(Ns_list), topN=topN, num_classes=num_classes,
                      tag=tag)
    pos_rows, neg_rows, pos_ids, neg_ids = [], [], [], []
    for b in range(B):
        n = nobj_list[b]
        ns = Ns_list[b]
        # obj nodes first (as the loader does), then attributes, then pair nodes
        inp["macro_obj_loc"][b, :] = LOC_PAD
        inp["macro_obj_loc"][b, :n] = np.arange(n)
        pair_loc, p = {}, n + n_attr
        for i in range(n):
            for j in range(n):
                if i != j:
                    pair_loc[(i, j)] = p
                    p += 1
        assert p == ns
        cnt = hashfill.randint(f"{tag}:npos:{b}", (len(pair_loc),), 1, max_rel_per_pair + 1)
        rp, rn, ip, ineg = [], [], [], []
        for q, ((i, j), loc3) in enumerate(sorted(pair_loc.items())):
            cats = hashfill.randint(f"{tag}:cat:{b}:{q}", (2 * int(cnt[q]),), 0, num_relations)
            for t in range(int(cnt[q])):
                rp.append([i, j, int(cats[t]), loc3, len(rp)])
                rn.append([i, j, int(cats[int(cnt[q]) + t]), loc3])
        ip = hashfill.randint(f"{tag}:relw:{b}", (len(rp),), 0, 407000)
        ineg = hashfill.randint(f"{tag}:nrelw:{b}", (len(rn),), 0, 407000)
        pos_rows.append(rp)
        neg_rows.append(rn)
        pos_ids.append(ip)
        neg_ids.append(ineg)
    L = max(len(r) for r in pos_rows)
    pr = np.full((B, L), PAD, np.int64)
    nr = np.full((B, L), PAD, np.int64)
    pl = np.full((B, L, 5), LOC_PAD, np.int64)
    nl = np.full((B, L, 4), LOC_PAD, np.int64)
    for b in range(B):
        k = len(pos_rows[b])
        pr[b, :k] = pos_ids[b]
        nr[b, :k] = neg_ids[b]
        pl[b, :k] = np.asarray(pos_rows[b], np.int64)
        nl[b, :k] = np.asarray(neg_rows[b], np.int64)
    inp.update(micro_positive_rel=pr, micro_negative_rel=nr, micro_positive_rel_loc=pl,
               micro_negative_rel_loc=nl)
    return inp
