"""GQA real-data reader (rank 1's relation loader): the only_obj
super-node dataset of models/data_loader_itp_bbox_super_node_onlyobj.py:41-334 and the
relation loader of dataloader/data_loader_itp_bbox_super_node.py:41-357, same constructor, same
per-item tuple, same failure behaviour (an item that cannot be built is None and is
dropped by the collate), same use of python's `random` for the negative words -- so
seeded runs reproduce the reference's items exactly (tests/test_gqa_reader_cpu.py).

Differences (host side only, no behaviour change): tar members are indexed once and
each worker process keeps its tar files open (the reference reopens three tar files per
item); vocabulary look-ups use precomputed space-stripped class lists; the composite-
word table is a constructor argument (`synonyms`, {multi word: single word}) that
defaults to the reference's `synonym_word_converter` module when it is importable.
Batches go through savqa_amd.collate.pack (DataLoader collate_fn) and
collate.to_device / StagingRing, which pad on the device.
"""
from __future__ import annotations

import codecs
import io
import json
import os
import random
import tarfile
from typing import Dict, Optional

import numpy as np
import torch.utils.data as tud

PAD = 400000   # onlyobj:34
UNK = 400001


def load_graph_vocab(fn):
    """onlyobj:20-26: `word index` per line."""
    lines = codecs.open(fn, "r", "utf-8").read().splitlines()
    vocab = [ln.split()[0] for ln in lines]
    index = [int(ln.split()[1]) for ln in lines]
    return ({w: index[i] for i, w in enumerate(vocab)}, {index[i]: w for i, w in enumerate(vocab)})


def load_answer_vocab(fn, min_cnt):
    """onlyobj:28-32: `answer words... count` per line; ids from 1 over count >= min_cnt."""
    lines = codecs.open(fn, "r", "utf-8").read().splitlines()
    vocab = [" ".join(ln.split()[:-1]) for ln in lines if int(ln.split()[-1]) >= min_cnt]
    return ({w: i + 1 for i, w in enumerate(vocab)}, {i + 1: w for i, w in enumerate(vocab)})


def _default_synonyms() -> Dict[str, str]:
    try:  # the reference's table, when this reader runs inside the reference tree
        from synonym_word_converter import syn_dict_composit_multiwrds  # type: ignore
        return dict(syn_dict_composit_multiwrds)
    except ImportError:
        return {}


class _Tar:
    """A tar file indexed once; reopened lazily in each (forked) worker process."""

    def __init__(self, path):
        self.path = path
        with tarfile.open(path) as t:
            self.members = t.getmembers()
        self._fid, self._pid = None, None

    def read(self, member) -> bytes:
        if self._fid is None or self._pid != os.getpid():
            self._fid, self._pid = tarfile.open(self.path), os.getpid()
        return self._fid.extractfile(member).read()

    def __getstate__(self):
        # spawned loader workers get the index, never the parent's open handle
        return {"path": self.path, "members": self.members, "_fid": None, "_pid": None}


class GQADataset_super_node(tud.Dataset):
    """onlyobj:41-99 constructor; opt carries data_dir_azure, maxlen, gt_relation_fn,
    enc_vocab_fn, ans_vocab_fn, min_cnt, bg_class, obj_vocab_fn, attr_vocab_fn, pred_rel,
    bbox_bin_num (main:430-500)."""

    def __init__(self, split, opt, fea_tar_fn, q_tar_fn, g_tar_fn, topN, with_loc=True,
                 synonyms: Optional[Dict[str, str]] = None):
        super().__init__()
        self.split = split
        self.opt = opt
        self.with_loc = with_loc
        self.topN = topN
        self.len_threshold = opt.maxlen
        root = opt.data_dir_azure
        self.fea_tar_fn = os.path.join(root, fea_tar_fn)
        self.q_tar_fn = os.path.join(root, q_tar_fn)
        self.g_tar_fn = os.path.join(root, g_tar_fn)
        self.gt_graph_fn = os.path.join(
            root, "train_sceneGraphs.json" if split == "train" else "val_sceneGraphs.json")
        self.enc_w2id, _ = load_graph_vocab(os.path.join(root, opt.enc_vocab_fn))
        self.ans_w2id, _ = load_answer_vocab(os.path.join(root, opt.ans_vocab_fn), opt.min_cnt)
        self._fea = _Tar(self.fea_tar_fn)
        self._g = self._fea if self.g_tar_fn == self.fea_tar_fn else _Tar(self.g_tar_fn)
        self._q = _Tar(self.q_tar_fn)
        self.fea_dict = {os.path.splitext(os.path.basename(m.name))[0]: m
                         for m in self._fea.members}
        self.g_dict = {os.path.splitext(os.path.basename(m.name))[0]: m for m in self._g.members}
        self.q_list = [m for m in self._q.members if m.name.endswith(".json")]
        self.bg_class = opt.bg_class
        with open(os.path.join(root, opt.gt_relation_fn)) as f:
            self.gt_relations = json.load(f)
        # category order = python's set order of the names, as in the reference (it follows
        # PYTHONHASHSEED; pin that variable for reproducible relation indices)
        self.gt_relation_clean = list(set(self.gt_relations.values()))
        self.num_relations = len(self.gt_relation_clean)
        with open(self.gt_graph_fn) as f:
            self.gt_graph = json.load(f)
        with open(os.path.join(root, opt.obj_vocab_fn)) as f:
            self.vg_classes = [o.split(",")[0].lower().strip() for o in f.readlines()]
        with open(os.path.join(root, opt.attr_vocab_fn)) as f:
            self.vg_attrs = [o.split(",")[0].lower().strip() for o in f.readlines()]
        self._vg_nospace = [c.replace(" ", "") for c in self.vg_classes]
        syn = _default_synonyms() if synonyms is None else synonyms
        self.word_converter = {}
        for key, val in syn.items():  # onlyobj:94-98
            nk = key.replace(" ", "")
            if nk != val:
                self.word_converter[nk] = val

    def __len__(self):
        return len(self.q_list)

    # ------------------------------------------------------------------ graph building
    def convert_graph(self, data_info, bg_class, bbox, gt_graph):
        """onlyobj:123-242: macro nodes (object placeholders, attribute, bbox-corner and
        relation nodes) + edges, object locations, positive / negative micro words."""
        micro_pos, micro_neg, empty, attrs, correct = [], [], [], [], []
        for obj_idxs, obj, attr_idx in zip(data_info["objects_id"], gt_graph["objects"],
                                           data_info["attrs_id"]):
            gt_name = gt_graph["objects"][obj]["name"].strip().replace(" ", "")
            nodes_obj = [gt_name]
            corr = 0
            for oi in obj_idxs:
                if len(nodes_obj) < self.topN:
                    if oi < len(self.vg_classes):
                        cls = self._vg_nospace[oi]
                        if cls != gt_name:
                            nodes_obj.append(cls)
                        else:
                            corr = 1
                else:
                    break
            correct.append(corr)
            empty.append(PAD)
            attrs.append(self.vg_attrs[attr_idx].replace(" ", ""))
            micro_pos.append(nodes_obj)
            population = [c for c in self._vg_nospace if c not in nodes_obj]
            micro_neg.append(random.sample(population, self.topN))

        n_obj = len(empty)
        macro_node, macro_rel, obj_loc, idx_obj = [], [], [], []
        attr_pos, corner_pos = {}, {}

        def node_at(table, name):
            if name in table:
                return table[name]
            table[name] = len(macro_node)
            macro_node.append(name)
            return table[name]

        for i in range(n_obj):
            p_obj = len(macro_node)
            macro_node.append(empty[i])
            obj_loc.append(p_obj)
            p_attr = node_at(attr_pos, attrs[i])
            macro_rel += [[p_obj, p_attr], [p_attr, p_obj]]
            idx_obj.append(p_obj)
            if self.with_loc:
                for cx, cy in ((0, 1), (2, 3)):  # top-left / bottom-right bbox corners
                    p = node_at(corner_pos, "x" + str(bbox[i][cx].item()) + "y" + str(bbox[i][cy]))
                    macro_rel += [[p_obj, p], [p, p_obj]]

        rel_pos = {}
        for i in range(n_obj):
            for j in range(n_obj):
                if self.opt.pred_rel:
                    oi = micro_pos[i][0] if correct[i] == 1 else micro_pos[i][1]
                    oj = micro_pos[j][0] if correct[j] == 1 else micro_pos[j][1]
                else:
                    oi, oj = micro_pos[i][0], micro_pos[j][0]
                key = oi + "," + oj
                if key not in self.gt_relations:
                    continue
                r_name = self.gt_relations[key].replace(" ", "")
                if r_name in rel_pos:
                    p_rel = rel_pos[r_name]
                else:
                    p_rel = len(macro_node)
                    rel_pos[r_name] = p_rel
                    r_name = "".join(r_name.split())
                    # spatial relation names follow the boxes (onlyobj:216-227)
                    sx = lambda k: bbox[k][0].item() + bbox[k][2].item()  # noqa: E731
                    sy = lambda k: bbox[k][1].item() + bbox[k][3].item()  # noqa: E731
                    if "left" in r_name and sx(i) > sx(j):
                        r_name = "right"
                    if "right" in r_name and sx(i) < sx(j):
                        r_name = "left"
                    if "bottom" in r_name and sy(i) < sy(j):
                        r_name = "top"
                    if "top" in r_name and sy(i) > sy(j):
                        r_name = "bottom"
                    macro_node.append(r_name)
                macro_rel += [[idx_obj[i], p_rel], [p_rel, idx_obj[j]]]
        return macro_node, macro_rel, obj_loc, micro_pos, micro_neg

    def _word_id(self, w):
        return self.enc_w2id.get(self.word_converter.get(w, w), UNK)

    def _question(self, index):
        qinfo = json.loads(self._q.read(self.q_list[index]))
        answer = np.asarray(self.ans_w2id.get(qinfo["answer"], 0)).astype("int32")
        return qinfo["node_list"], qinfo["edge_pair"], answer, qinfo["image_id"]

    def _image(self, image_id):
        """Features, binned boxes and the detector info of one image (onlyobj:253-285)."""
        gt_graph = self.gt_graph[image_id]
        vis_fea = np.load(io.BytesIO(self._fea.read(self.fea_dict[image_id])))["x"]
        # the graph archive carries a pickled `info` dict, as written by the GQA
        # preprocessing; it is the user's data file, read like the reference does
        data = np.load(io.BytesIO(self._g.read(self.g_dict[image_id])), allow_pickle=True)
        bbox = data["bbox"]
        if len(bbox.shape) == 1:
            bbox = np.reshape(bbox, (1, bbox.size))
        bbox[:, 0] /= data["image_w"]
        bbox[:, 2] /= data["image_w"]
        bbox[:, 1] /= data["image_h"]
        bbox[:, 3] /= data["image_h"]
        bbox = np.floor(bbox * self.opt.bbox_bin_num).astype("int32")
        return gt_graph, vis_fea, bbox, data["info"].tolist()

    def _too_long(self, n_macro, n_q):
        if n_macro + n_q >= self.len_threshold:
            if self.split in ("val", "test"):
                print("len", n_macro + n_q)
            return True
        return False

    def __getitem__(self, index):
        """onlyobj:243-334. Returns the collate tuple or None."""
        qnode, qedge, answer, image_id = self._question(index)
        try:
            gt_graph, vis_fea, bbox, info = self._image(image_id)
            macro_nodes, macro_edges, obj_locs, pos_nodes, neg_nodes = self.convert_graph(
                info, self.opt.bg_class, bbox, gt_graph)
            macro_idx = [PAD if n == PAD else self._word_id(n) for n in macro_nodes]
            q_idx = [self.enc_w2id.get(w, UNK) for w in qnode]
            if self._too_long(len(macro_idx), len(q_idx)):
                return None
            pos_w = [[self._word_id(w) for w in ws] for ws in pos_nodes]
            neg_w = [[self._word_id(w) for w in ws] for ws in neg_nodes]
            return (vis_fea, np.asarray(macro_idx).astype("int64"),
                    np.asarray(obj_locs).astype("int64"), macro_edges,
                    np.asarray(pos_w).astype("int64"), np.asarray(neg_w).astype("int64"),
                    np.asarray(q_idx).astype("int64"), qedge, answer, self.topN)
        except Exception:  # the reference's bare except: an unreadable item is None
            return None


class GQADataset_super_node_rel(GQADataset_super_node):
    """The relation loader (dataloader/data_loader_itp_bbox_super_node.py:41-357): same
    files and constructor; every ordered object pair gets an empty relation node, and the
    item carries the positive / negative relation words and their locations
    [obj_i, obj_j, category, macro_rel_loc(, micro_rel_loc)] for the MIL-NCE relation
    branch (14-field tuple, collate_fn :366-497)."""

    def convert_graph(self, data_info, bg_class, bbox, gt_graph):
        """super_node:123-249."""
        micro_pos, micro_neg, empty, attrs = [], [], [], []
        for obj_idxs, obj, attr_idx in zip(data_info["objects_id"], gt_graph["objects"],
                                           data_info["attrs_id"]):
            gt_name = gt_graph["objects"][obj]["name"].strip().replace(" ", "")
            nodes_obj = [gt_name]
            for oi in obj_idxs:  # (no detection-correctness flag in this loader)
                if len(nodes_obj) < self.topN:
                    if oi < len(self.vg_classes) and self._vg_nospace[oi] != gt_name:
                        nodes_obj.append(self._vg_nospace[oi])
                else:
                    break
            empty.append(PAD)
            attrs.append(self.vg_attrs[attr_idx].replace(" ", ""))
            micro_pos.append(nodes_obj)
            population = [c for c in self._vg_nospace if c not in nodes_obj]
            micro_neg.append(random.sample(population, self.topN))

        n_obj = len(empty)
        macro_node, macro_rel, obj_loc, idx_obj = [], [], [], []
        attr_pos, corner_pos, rel_loc = {}, {}, {}

        def node_at(table, name):
            if name in table:
                return table[name]
            table[name] = len(macro_node)
            macro_node.append(name)
            return table[name]

        for i in range(n_obj):
            p_obj = len(macro_node)
            macro_node.append(empty[i])
            obj_loc.append(p_obj)
            p_attr = node_at(attr_pos, attrs[i])
            macro_rel += [[p_obj, p_attr], [p_attr, p_obj]]
            idx_obj.append(p_obj)
            if self.with_loc:
                for cx, cy in ((0, 1), (2, 3)):
                    p = node_at(corner_pos, "x" + str(bbox[i][cx].item()) + "y" + str(bbox[i][cy]))
                    macro_rel += [[p_obj, p], [p, p_obj]]
        for i in range(n_obj):  # one empty relation node per ordered pair (:190-201)
            for j in range(n_obj):
                if i != j:
                    rel_loc[(i, j)] = len(macro_node)
                    macro_node.append("__empty__")
                    macro_rel += [[idx_obj[i], rel_loc[(i, j)]], [rel_loc[(i, j)], idx_obj[j]]]

        n_cat = len(self.gt_relation_clean)
        cat_of = {name: k for k, name in reversed(list(enumerate(self.gt_relation_clean)))}
        pos_words, neg_words, pos_loc, neg_loc = [], [], [], []
        micro_pos_ctr = 0
        for i in range(n_obj):  # every (word_i, word_j) of every ordered pair (:203-247)
            for j in range(n_obj):
                if i == j:
                    continue
                pair_words, pair_idx = [], []
                for wi in micro_pos[i]:
                    for wj in micro_pos[j]:
                        key = wi + "," + wj
                        if key in self.gt_relations:
                            name = self.gt_relations[key]
                            r_idx = cat_of[name]
                            pair_words.append(name.replace(" ", ""))
                        else:
                            r_idx = self.num_relations  # the PAD category
                            pair_words.append(PAD)
                        pos_loc.append([i, j, r_idx, rel_loc[(i, j)], micro_pos_ctr])
                        pair_idx.append(r_idx)
                        micro_pos_ctr += 1
                pos_words += pair_words
                neg_pool = [k for k in range(n_cat) if k not in pair_idx]
                for r_idx in random.sample(neg_pool, len(pair_words)):
                    neg_loc.append([i, j, r_idx, rel_loc[(i, j)]])
                    neg_words.append(self.gt_relation_clean[r_idx] if r_idx != n_cat else PAD)
        return (macro_node, macro_rel, obj_loc, micro_pos, micro_neg, pos_words, neg_words,
                pos_loc, neg_loc)

    def __getitem__(self, index):
        """super_node:250-357. Returns the 14-field collate tuple or None."""
        qnode, qedge, answer, image_id = self._question(index)
        try:
            gt_graph, vis_fea, bbox, info = self._image(image_id)
            (macro_nodes, macro_edges, obj_locs, pos_nodes, neg_nodes, pos_rel, neg_rel,
             pos_rel_loc, neg_rel_loc) = self.convert_graph(info, self.opt.bg_class, bbox,
                                                            gt_graph)
            macro_idx = [PAD if n == PAD else self._word_id(n) for n in macro_nodes]
            q_idx = [self.enc_w2id.get(w, UNK) for w in qnode]
            if self._too_long(len(macro_idx), len(q_idx)):
                return None
            pos_w = [[self._word_id(w) for w in ws] for ws in pos_nodes]
            neg_w = [[self._word_id(w) for w in ws] for ws in neg_nodes]
            pos_rw = [self._word_id(w) for w in pos_rel]  # PAD words look up as UNK (:340)
            neg_rw = [self._word_id(w) for w in neg_rel]
            return (vis_fea, np.asarray(macro_idx).astype("int64"),
                    np.asarray(obj_locs).astype("int64"), macro_edges,
                    np.asarray(pos_w).astype("int64"), np.asarray(neg_w).astype("int64"),
                    np.asarray(pos_rw).astype("int64"), np.asarray(neg_rw).astype("int64"),
                    np.asarray(pos_rel_loc).astype("int64"),
                    np.asarray(neg_rel_loc).astype("int64"),
                    np.asarray(q_idx).astype("int64"), qedge, answer, self.topN)
        except Exception:  # the reference's bare except: an unreadable item is None
            return None
