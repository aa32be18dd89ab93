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
