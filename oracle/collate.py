"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's batch collation.

Restates in numpy the two collate functions that turn a list of per-sample tuples
(Dataset.__getitem__ output) into the padded dense tensors AttModel.forward takes:
  collate_onlyobj     models/data_loader_itp_bbox_super_node_onlyobj.py:341-445
  collate_super_node  dataloader/data_loader_itp_bbox_super_node.py:366-497
(the relation loader: the same plus the four relation tensors, :426-447).
Outputs are numpy arrays under the reference's dict keys.

`make_samples` builds per-sample tuples (hash-filled, oracle/hashfill.py) with the
edge cases the reference code paths distinguish: ragged lengths per field, an empty
macro edge list (skipped, :398-399), a single edge given as a flat pair (:400-401),
duplicate and negative (numpy-wrapped) edge indices, fewer micro rows than object
locations, and a sample without relations (its relation rows stay padding, :434).

Pinning: tests/golden/collate.npz holds the reference collate_fn outputs on these
samples (tools/make_golden.py collate); tests/test_collate_cpu.py checks this
restatement against them bit for bit.
"""
from __future__ import annotations

import numpy as np

from . import hashfill

PAD = 400000    # onlyobj:34
LOC_PAD = -1    # onlyobj:39

OBJ_FIELDS = ("vis_fea", "macro_nodes_idx", "macro_obj_locs", "macro_edges",
              "micro_positive_nodes_wrd", "micro_negative_nodes_wrd")
REL_FIELDS = ("micro_positive_relations_wrd", "micro_negative_relations_wrd",
              "micro_positive_relations_loc", "micro_negative_relations_loc")
TAIL_FIELDS = ("qnode_idx", "qedge", "answer", "topN")


def sample_fields(relations: bool):
    """Order of the per-sample tuple (onlyobj:343-345; super_node:367-369)."""
    return OBJ_FIELDS + (REL_FIELDS if relations else ()) + TAIL_FIELDS


def _graph(batch_size, T, edges_list, skip_empty):
    g = np.zeros((batch_size, T, T), dtype="int32")
    for row, edge in enumerate(edges_list):
        edge = np.asarray(edge).astype("int32")
        if skip_empty:  # macro edges (onlyobj:397-401)
            if edge.size == 0:
                continue
            if len(edge.shape) == 1:
                edge = edge[np.newaxis, :]
        g[row, edge[:, 0], edge[:, 1]] = 1
    return g


def _collate(data, relations: bool):
    data = [d for d in data if d is not None]
    cols = dict(zip(sample_fields(relations), zip(*data)))
    topN = cols["topN"][0]
    vis_fea = cols["vis_fea"]
    answer = np.stack(cols["answer"], axis=0)
    B = len(cols["macro_nodes_idx"])
    out = {}
    # visual features (onlyobj:351-359)
    T_v = max(f.shape[0] for f in vis_fea)
    fea = np.zeros((B, T_v, vis_fea[0].shape[1]), dtype="float32")
    fea_mask = np.zeros((B, T_v, T_v), dtype="int32")
    for i in range(B):
        n = vis_fea[i].shape[0]
        fea[i, :n, :] = vis_fea[i]
        fea_mask[i, :n, :n] = 1
    # symbolic nodes + graph (onlyobj:363-402)
    nodes = cols["macro_nodes_idx"]
    T_s = max(n.shape[0] for n in nodes)
    node_ipt = np.full((B, T_s), PAD, dtype="int64")
    node_mask = np.zeros((B, T_s, T_s), dtype="int32")
    for i in range(B):
        n = nodes[i].shape[0]
        node_ipt[i, :n] = nodes[i]
        node_mask[i, :n, :n] = 1
    node_graph = _graph(B, T_s, cols["macro_edges"], skip_empty=True)
    # object locations + micro (word) nodes, rows padded to T_v (onlyobj:404-420)
    loc = np.full((B, T_v), LOC_PAD, dtype="int64")
    pos = np.full((B, T_v, topN), PAD, dtype="int64")
    neg = np.full((B, T_v, topN), PAD, dtype="int64")
    omask = np.zeros((B, T_v, topN), dtype="int32")
    for i in range(B):
        locs = cols["macro_obj_locs"][i]
        loc[i, :locs.shape[0]] = locs
        p = cols["micro_positive_nodes_wrd"][i]
        q = cols["micro_negative_nodes_wrd"][i]
        pos[i, :p.shape[0], :] = p
        neg[i, :q.shape[0], :] = q
        omask[i, :locs.shape[0], :] = 1
    if relations:  # super_node:422-439
        prw = cols["micro_positive_relations_wrd"]
        T_r = max(r.shape[0] for r in prw)
        pr = np.full((B, T_r), PAD, dtype="int64")
        nr = np.full((B, T_r), PAD, dtype="int64")
        pl = np.full((B, T_r, 5), LOC_PAD, dtype="int64")
        nl = np.full((B, T_r, 4), LOC_PAD, dtype="int64")
        for i in range(B):
            if prw[i].shape[0] != 0:
                pr[i, :prw[i].shape[0]] = prw[i]
                nrw = cols["micro_negative_relations_wrd"][i]
                nr[i, :nrw.shape[0]] = nrw
                prl = cols["micro_positive_relations_loc"][i]
                pl[i, :prl.shape[0], :] = prl
                nrl = cols["micro_negative_relations_loc"][i]
                nl[i, :nrl.shape[0], :] = nrl
    # question nodes + graph (onlyobj:422-435)
    qn = cols["qnode_idx"]
    T_q = max(n.shape[0] for n in qn)
    q_ipt = np.full((B, T_q), PAD, dtype="int64")
    q_mask = np.zeros((B, T_q, T_q), dtype="int32")
    for i in range(B):
        n = qn[i].shape[0]
        q_ipt[i, :n] = qn[i]
        q_mask[i, :n, :n] = 1
    q_graph = _graph(B, T_q, cols["qedge"], skip_empty=False)
    out["vis_fea"] = fea
    out["vis_fea_mask"] = fea_mask
    out["macro_node_ipt"] = node_ipt
    out["macro_graph_ipt"] = node_graph
    out["macro_node_mask"] = node_mask
    out["macro_obj_loc_ipt"] = loc
    out["micro_positive_obj_ipt"] = pos
    out["micro_negative_obj_ipt"] = neg
    out["micro_obj_mask"] = omask
    if relations:
        out["micro_positive_rel_ipt"] = pr
        out["micro_negative_rel_ipt"] = nr
        out["micro_positive_rel_loc"] = pl
        out["micro_negative_rel_loc"] = nl
    out["q_ipt"] = q_ipt
    out["q_ipt_mask"] = q_mask
    out["q_ipt_graph"] = q_graph
    out["answer"] = answer.astype("int64")
    return out


def collate_onlyobj(data):
    """models/data_loader_itp_bbox_super_node_onlyobj.py:341-445."""
    return _collate(data, relations=False)


def collate_super_node(data):
    """dataloader/data_loader_itp_bbox_super_node.py:366-497."""
    return _collate(data, relations=True)


def make_samples(B, relations=False, fea_dim=2048, topN=5, tag="col", nv_range=(3, 36),
                 edge_cases=True):
    """Per-sample tuples shaped like the loaders' __getitem__ (onlyobj:330-332;
    super_node:353-357), ragged; see the module docstring for the edge cases."""
    out = []
    for b in range(B):
        t = f"{tag}:{b}"
        nv = int(hashfill.randint(t + ":nv", (1,), nv_range[0], nv_range[1] + 1)[0])
        n_attr = int(hashfill.randint(t + ":na", (1,), 0, 5)[0])
        ns = nv + n_attr + int(hashfill.randint(t + ":nr", (1,), 0, 8)[0])
        lq = int(hashfill.randint(t + ":lq", (1,), 2, 15)[0])
        vis = np.maximum(hashfill.fill(t + ":vis", (nv, fea_dim)), 0).astype(np.float32)
        nodes = hashfill.randint(t + ":nodes", (ns,), 0, PAD + 4)
        n_loc = nv
        locs = np.argsort(hashfill.uniform_bits(t + ":locs", ns))[:n_loc].astype(np.int64)
        n_micro = nv - (1 if edge_cases and b % 3 == 1 else 0)  # fewer micro rows than locs
        pos = hashfill.randint(t + ":pos", (n_micro, topN), 0, 407000)
        neg = hashfill.randint(t + ":neg", (n_micro, topN), 0, 407000)
        ne = int(hashfill.randint(t + ":ne", (1,), 1, 3 * ns)[0])
        e = hashfill.randint(t + ":edges", (ne, 2), 0, ns)
        if edge_cases and b % 4 == 0:
            macro_edges = []                       # empty edge list: skipped (onlyobj:398)
        elif edge_cases and b % 4 == 1:
            macro_edges = [int(e[0, 0]), int(e[0, 1])]  # one edge as a flat pair (:400)
        elif edge_cases and b % 4 == 2:
            e = np.concatenate([e, e[:2], -1 - e[:1]], 0)  # duplicates, negative index
            macro_edges = e.tolist()
        else:
            macro_edges = e.tolist()
        nq = int(hashfill.randint(t + ":nqe", (1,), 1, 2 * lq)[0])
        qe = hashfill.randint(t + ":qedges", (nq, 2), 0, lq).tolist()
        q = hashfill.randint(t + ":q", (lq,), 0, PAD)
        answer = np.int64(hashfill.randint(t + ":ans", (1,), 1, 914)[0])
        fields = [vis, nodes, locs, macro_edges, pos, neg]
        if relations:
            nrel = 0 if (edge_cases and b % 5 == 3) else \
                int(hashfill.randint(t + ":nrel", (1,), 1, 40)[0])
            prw = hashfill.randint(t + ":prw", (nrel,), 0, 407000)
            nrw = hashfill.randint(t + ":nrw", (nrel,), 0, 407000)
            prl = np.stack([hashfill.randint(t + ":prl0", (nrel,), 0, nv),
                            hashfill.randint(t + ":prl1", (nrel,), 0, nv),
                            hashfill.randint(t + ":prl2", (nrel,), 0, 311),
                            hashfill.randint(t + ":prl3", (nrel,), 0, ns),
                            np.arange(nrel, dtype=np.int64)], 1).reshape(nrel, 5)
            nrl = np.stack([hashfill.randint(t + ":nrl0", (nrel,), 0, nv),
                            hashfill.randint(t + ":nrl1", (nrel,), 0, nv),
                            hashfill.randint(t + ":nrl2", (nrel,), 0, 311),
                            hashfill.randint(t + ":nrl3", (nrel,), 0, ns)], 1).reshape(nrel, 4)
            fields += [prw, nrw, prl, nrl]
        fields += [q, qe, answer, topN]
        out.append(tuple(fields))
    return out
