"""Synthetic batches with the tensor contract of the reference's collate_fn
(models/data_loader_itp_bbox_super_node_onlyobj.py:341-445), generated on device.

The GQA tar/npz/json data is not available offline, so throughput runs use this
generator: relu(N(0,1)) 2048-d region features (pooled
Faster-RCNN features are non-negative), all-valid masks, Bernoulli question /
scene graphs, uniform GloVe ids, macro_obj_loc = region index, uniform answers.
"""
from __future__ import annotations

import torch

PAD = 400000


def synthetic_batch(B: int, Nv: int = 36, Lq: int = 14, Ns: int = 59, topN: int = 5,
                    num_classes: int = 914, seed: int = 1234, device="cuda"):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    dev = device

    def ri(low, high, shape):
        return torch.randint(low, high, shape, generator=g, device=dev, dtype=torch.int64)

    vis = torch.randn(B, Nv, 2048, generator=g, device=dev).clamp_min_(0)
    batch = {
        "vis_fea": vis,
        "vis_mask": torch.ones(B, Nv, Nv, dtype=torch.int32, device=dev),
        "q_ipt": ri(0, PAD, (B, Lq)),
        "q_mask": torch.ones(B, Lq, Lq, dtype=torch.int32, device=dev),
        "q_graph": (torch.rand(B, Lq, Lq, generator=g, device=dev) < 0.2).to(torch.int32),
        "macro_ipt": ri(0, PAD, (B, Ns)),
        "macro_mask": torch.ones(B, Ns, Ns, dtype=torch.int32, device=dev),
        "macro_graph": (torch.rand(B, Ns, Ns, generator=g, device=dev) < 0.05).to(torch.int32),
        "macro_obj_loc": torch.arange(Nv, device=dev, dtype=torch.int64).repeat(B, 1),
        "micro_positive_obj": ri(0, PAD, (B, Nv, topN)),
        "micro_negative_obj": ri(0, PAD, (B, Nv, topN)),
        "micro_obj_mask": torch.ones(B, Nv, topN, dtype=torch.int32, device=dev),
        "answer": ri(1, num_classes, (B,)),
    }
    return batch


MODEL_INPUTS = ("vis_fea", "vis_mask", "q_ipt", "q_mask", "q_graph", "macro_ipt", "macro_mask",
                "macro_graph", "macro_obj_loc", "micro_positive_obj", "micro_negative_obj",
                "micro_obj_mask")


def model_args(batch):
    """Positional args of AttModel.forward (the 4 relation tensors are empty, main:290-308)."""
    B = batch["vis_fea"].shape[0]
    empty = torch.empty((B, 0), device=batch["vis_fea"].device)
    return [batch[k] for k in MODEL_INPUTS] + [empty, empty, empty, empty]


REL_INPUTS = ("micro_positive_rel", "micro_negative_rel", "micro_positive_rel_loc",
              "micro_negative_rel_loc")


def model_args_rel(batch):
    """Positional args of AttModel.forward with the relation tensors (only_obj=False)."""
    return [batch[k] for k in MODEL_INPUTS] + [batch[k] for k in REL_INPUTS]


def synthetic_relation_batch(B: int, Nv: int = 36, Lq: int = 14, topN: int = 5,
                             num_relations: int = 311, n_attr: int = 4, num_classes: int = 914,
                             seed: int = 1234, device="cuda"):
    """Super-node batch with the relation tensors of the relation loader
    (dataloader/data_loader_itp_bbox_super_node.py:150-252, collate :366-497), synthetic:
    macro nodes = Nv objects, n_attr attribute nodes, one relation node per ordered object
    pair (Nv*(Nv-1)); edges obj<->attr and obj_i -> rel(i,j) -> obj_j (:165-206); every pair
    contributes topN*topN positive entries [i, j, category, macro_rel_loc, running counter]
    (:215-237) and as many negatives [i, j, category', macro_rel_loc] (:241-246).
    At Nv = 36: T_syb = 36 + 4 + 1260 + Lq = 1314 tokens, 31,500 entries per sample."""
    import numpy as np
    rng = np.random.default_rng(seed)
    Ns = Nv + n_attr + Nv * (Nv - 1)
    pairs = [(i, j) for i in range(Nv) for j in range(Nv) if i != j]
    K = topN * topN
    L = len(pairs) * K
    pi = np.repeat(np.array([p[0] for p in pairs]), K)
    pj = np.repeat(np.array([p[1] for p in pairs]), K)
    ploc = np.repeat(Nv + n_attr + np.arange(len(pairs)), K)
    pos_loc = np.zeros((B, L, 5), np.int64)
    neg_loc = np.zeros((B, L, 4), np.int64)
    graph = np.zeros((B, Ns, Ns), np.int32)
    for b in range(B):
        cat = rng.integers(0, num_relations, L)
        ncat = (cat + rng.integers(1, max(num_relations, 2), L)) % max(num_relations, 1)
        pos_loc[b] = np.stack([pi, pj, cat, ploc, np.arange(L)], 1)
        neg_loc[b] = np.stack([pi, pj, ncat, ploc], 1)
        attr = Nv + rng.integers(0, n_attr, Nv)
        graph[b, np.arange(Nv), attr] = 1
        graph[b, attr, np.arange(Nv)] = 1
        q = Nv + n_attr + np.arange(len(pairs))
        graph[b, [p[0] for p in pairs], q] = 1
        graph[b, q, [p[1] for p in pairs]] = 1
    batch = synthetic_batch(B, Nv=Nv, Lq=Lq, Ns=Ns, topN=topN, num_classes=num_classes,
                            seed=seed, device=device)
    dev = batch["vis_fea"].device
    batch["macro_graph"] = torch.from_numpy(graph).to(dev)
    g = torch.Generator(device=dev).manual_seed(seed + 1)
    batch["micro_positive_rel"] = torch.randint(0, PAD, (B, L), generator=g, device=dev)
    batch["micro_negative_rel"] = torch.randint(0, PAD, (B, L), generator=g, device=dev)
    batch["micro_positive_rel_loc"] = torch.from_numpy(pos_loc).to(dev)
    batch["micro_negative_rel_loc"] = torch.from_numpy(neg_loc).to(dev)
    return batch


def synthetic_samples(B: int, relations: bool = False, Nv=(10, 36), Lq=(5, 14), topN: int = 5,
                      fea_dim: int = 2048, n_attr: int = 4, extra_nodes=(0, 23),
                      num_relations: int = 311, num_classes: int = 914, seed: int = 1234):
    """Per-sample tuples shaped like the loaders' Dataset.__getitem__ (onlyobj:330-332;
    super_node:353-357) for the device collate (collate.pack): ragged region counts in
    [Nv[0], Nv[1]], question lengths in [Lq[0], Lq[1]]. only_obj: Nv object nodes +
    n_attr attribute nodes + U(extra_nodes) relation nodes with Bernoulli(0.05) edges.
    relations: the super-node layout of synthetic_relation_batch (one relation node per
    ordered object pair, topN^2 positive and negative entries per pair)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(B):
        nv = int(rng.integers(Nv[0], Nv[1] + 1))
        lq = int(rng.integers(Lq[0], Lq[1] + 1))
        vis = np.maximum(rng.standard_normal((nv, fea_dim), dtype=np.float32), 0)
        q = rng.integers(0, PAD, lq)
        qedge = np.argwhere(rng.random((lq, lq)) < 0.2)
        if len(qedge) == 0:
            qedge = np.zeros((1, 2), np.int64)
        pos = rng.integers(0, PAD, (nv, topN))
        neg = rng.integers(0, PAD, (nv, topN))
        ans = np.int64(rng.integers(1, num_classes))
        if not relations:
            ns = nv + n_attr + int(rng.integers(extra_nodes[0], extra_nodes[1] + 1))
            nodes = rng.integers(0, PAD, ns)
            edges = np.argwhere(rng.random((ns, ns)) < 0.05)
            out.append((vis, nodes, np.arange(nv), edges, pos, neg, q, qedge, ans, topN))
            continue
        pairs = np.array([(i, j) for i in range(nv) for j in range(nv) if i != j], np.int64)
        ns = nv + n_attr + len(pairs)
        nodes = rng.integers(0, PAD, ns)
        attr = nv + rng.integers(0, n_attr, nv)
        rel = nv + n_attr + np.arange(len(pairs))
        edges = np.concatenate([np.stack([np.arange(nv), attr], 1), np.stack([attr, np.arange(nv)], 1),
                                np.stack([pairs[:, 0], rel], 1), np.stack([rel, pairs[:, 1]], 1)])
        K = topN * topN
        L = len(pairs) * K
        pi, pj, ploc = (np.repeat(pairs[:, 0], K), np.repeat(pairs[:, 1], K), np.repeat(rel, K))
        cat = rng.integers(0, num_relations, L)
        ncat = (cat + rng.integers(1, max(num_relations, 2), L)) % max(num_relations, 1)
        prl = np.stack([pi, pj, cat, ploc, np.arange(L)], 1)
        nrl = np.stack([pi, pj, ncat, ploc], 1)
        out.append((vis, nodes, np.arange(nv), edges, pos, neg, rng.integers(0, PAD, L),
                    rng.integers(0, PAD, L), prl, nrl, q, qedge, ans, topN))
    return out
