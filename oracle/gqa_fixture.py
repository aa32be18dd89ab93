"""TEST INFRASTRUCTURE ONLY -- a tiny synthetic GQA dataset in the reference's on-disk
layout, for the real-data reader row.

Writes, under `root`, the files GQADataset_super_node reads
(models/data_loader_itp_bbox_super_node_onlyobj.py:41-99, 244-334):
  train.tar              question json members {node_list, edge_pair, answer, image_id}
  gt_bua_npz.tar         <image_id>.npz: x (features), bbox, image_w, image_h, info (a
                         pickled dict {objects_id: [[vg class idx]*], attrs_id: [idx]*})
  train_sceneGraphs.json {image_id: {objects: {obj_id: {name}}}}
  GT_relations_dict_compsite.json   {"obj_i,obj_j": relation name}
  objects_vocab.txt, attributes_vocab.txt, preprocessed/de.vocab.composite2.tsv,
  preprocessed/en.vocab.tsv
Deterministic (numpy Generator seeded by `seed`). Edge cases the reader distinguishes:
composite object names that the word converter rewrites ("stop sign" -> "stop"), words
missing from the vocabulary (UNK), answers below min_cnt (class 0), a single-object
image (1-D bbox), a question whose image is missing (exception -> None), a question
whose node count crosses maxlen (-> None), relation names with left/right/top/bottom
that the bbox test flips.
"""
from __future__ import annotations

import io
import json
import os
import tarfile

import numpy as np

OBJECTS = ["stop sign", "man", "woman", "tennis court", "dog", "cat", "tree", "car", "ball",
           "table", "chair", "cup", "window", "door", "sky", "grass", "tv", "sail boat",
           "alarm clock", "shirt"]
ATTRS = ["red", "blue", "green", "small", "large", "wooden", "white", "black"]
RELS = {"man,dog": "to the left of", "dog,man": "to the right of", "cup,table": "on top of",
        "table,cup": "at the bottom of", "woman,car": "near", "tree,sky": "below",
        "man,shirt": "wearing", "cat,ball": "to the left of", "stop,car": "in front of"}
# more categories, so that negative relation sampling (up to topN^2 per pair, super_node
# :238-240) has a large enough pool
for _k, (_a, _b) in enumerate(zip(OBJECTS[::2], OBJECTS[1::2] + OBJECTS[:1])):
    RELS[_a.replace(" ", "") + "," + _b.replace(" ", "")] = f"extra relation {_k}"
    RELS[_b.replace(" ", "") + "," + _a.replace(" ", "")] = f"extra inverse {_k}"
QWORDS = ["what", "color", "is", "the", "left", "of", "man", "dog", "who", "wearing"]


def _add(tar, name, data: bytes):
    ti = tarfile.TarInfo(name)
    ti.size = len(data)
    tar.addfile(ti, io.BytesIO(data))


def write_dataset(root: str, n_images: int = 5, n_questions: int = 12, seed: int = 0,
                  fea_dim: int = 16):
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, "preprocessed"), exist_ok=True)
    with open(os.path.join(root, "objects_vocab.txt"), "w") as f:
        for o in OBJECTS:
            f.write(o + ",alias\n")
    with open(os.path.join(root, "attributes_vocab.txt"), "w") as f:
        for a in ATTRS:
            f.write(a + "\n")
    # encoder vocab: most words, some left out (-> UNK); index column = id
    words = sorted({o.replace(" ", "") for o in OBJECTS} | set(ATTRS) | set(QWORDS)
                   | {"stop", "field", "television", "sailboat", "clock", "left", "right",
                      "top", "bottom", "near", "below", "wearing", "infrontof"})
    words = [w for w in words if w not in ("grass", "blue", "who")]
    with open(os.path.join(root, "preprocessed", "de.vocab.composite2.tsv"), "w") as f:
        for i, w in enumerate(words):
            f.write(f"{w}\t{1000 + 7 * i}\n")
        for x in range(0, 64, 3):      # a few bbox position nodes
            for y in range(0, 64, 5):
                f.write(f"x{x}y{y}\t{5000 + 64 * x + y}\n")
    answers = [("yes", 50), ("no", 40), ("red", 12), ("dog", 9), ("left side", 30)]
    with open(os.path.join(root, "preprocessed", "en.vocab.tsv"), "w") as f:
        for a, c in answers:
            f.write(f"{a} {c}\n")
    with open(os.path.join(root, "GT_relations_dict_compsite.json"), "w") as f:
        json.dump(RELS, f)

    graphs, image_ids = {}, []
    with tarfile.open(os.path.join(root, "gt_bua_npz.tar"), "w") as tar:
        for k in range(n_images):
            iid = f"img{k}"
            image_ids.append(iid)
            n = 1 if k == 1 else int(rng.integers(2, 7))
            names = [OBJECTS[int(i)] for i in rng.integers(0, len(OBJECTS), n)]
            if k == 0:  # guarantee relation hits (man/dog, cup/table)
                names[:2] = ["man", "dog"] if n >= 2 else names[:2]
            graphs[iid] = {"objects": {str(100 + j): {"name": nm} for j, nm in enumerate(names)}}
            objects_id = []
            for j in range(n):
                cand = [int(c) for c in rng.integers(0, len(OBJECTS) + 3, 6)]  # some >= vocab
                if rng.random() < 0.5:
                    cand.insert(int(rng.integers(0, 3)), OBJECTS.index(names[j]))
                objects_id.append(cand)
            info = {"objects_id": objects_id,
                    "attrs_id": [int(a) for a in rng.integers(0, len(ATTRS), n)]}
            W, H = 640.0, 480.0
            x0 = rng.uniform(0, W * 0.6, n)
            y0 = rng.uniform(0, H * 0.6, n)
            bbox = np.stack([x0, y0, x0 + rng.uniform(10, W * 0.4, n),
                             y0 + rng.uniform(10, H * 0.4, n)], 1).astype(np.float32)
            if n == 1:
                bbox = bbox.reshape(-1)
            buf = io.BytesIO()
            np.savez(buf, x=rng.standard_normal((n, fea_dim)).astype(np.float32), bbox=bbox,
                     image_w=np.float32(W), image_h=np.float32(H),
                     info=np.array(info, dtype=object))
            _add(tar, f"feats/{iid}.npz", buf.getvalue())
    with open(os.path.join(root, "train_sceneGraphs.json"), "w") as f:
        json.dump(graphs, f)

    with tarfile.open(os.path.join(root, "train.tar"), "w") as tar:
        for q in range(n_questions):
            lq = int(rng.integers(2, 8))
            if q == 7:
                lq = 400  # crosses maxlen -> None
            nodes = [QWORDS[int(i)] for i in rng.integers(0, len(QWORDS), lq)]
            edges = [[int(a), int(b)] for a, b in rng.integers(0, lq, (max(1, lq - 1), 2))]
            iid = image_ids[q % n_images] if q != 5 else "missing_image"
            ans = answers[int(rng.integers(0, len(answers)))][0]
            qinfo = {"node_list": nodes, "edge_pair": edges, "answer": ans, "image_id": iid}
            _add(tar, f"q/{q:05d}.json", json.dumps(qinfo).encode())
        _add(tar, "q/README.txt", b"not a question")
    # the val split (main:236-249) reads the same files under its own names
    import shutil
    shutil.copy(os.path.join(root, "train.tar"), os.path.join(root, "val.tar"))
    shutil.copy(os.path.join(root, "train_sceneGraphs.json"),
                os.path.join(root, "val_sceneGraphs.json"))
    return image_ids


class Opt:
    """The argparse fields GQADataset_super_node reads (main:430-500 defaults)."""

    def __init__(self, root, maxlen=300, pred_rel=False):
        self.data_dir_azure = root
        self.maxlen = maxlen
        self.gt_relation_fn = "GT_relations_dict_compsite.json"
        self.enc_vocab_fn = "preprocessed/de.vocab.composite2.tsv"
        self.ans_vocab_fn = "preprocessed/en.vocab.tsv"
        self.obj_vocab_fn = "objects_vocab.txt"
        self.attr_vocab_fn = "attributes_vocab.txt"
        self.min_cnt = 10
        self.bbox_bin_num = 64
        self.pred_rel = pred_rel
        self.bg_class = len(OBJECTS) + 1  # main:185


# fields of one __getitem__ tuple (onlyobj:330-332)
ITEM_FIELDS = ("vis_fea", "macro_nodes_idx", "macro_obj_locs", "macro_edges",
               "micro_positive_nodes_wrd", "micro_negative_nodes_wrd", "qnode_idx", "qedge",
               "answer", "topN")

# The entries of the reference's composite-word table (models/synonym_word_converter.py)
# that touch the fixture vocabulary, in that table's {multi word: single word} form; the
# reader builds its converter from it the way onlyobj:94-98 does.
SYNONYMS = {"alarm clock": "clock", "in front of": "front", "on top of": "top",
            "stop sign": "stop", "tennis court": "field", "to the left of": "left",
            "to the right of": "right", "tv": "television"}

# fields of one relation-loader item (super_node:353-357)
ITEM_FIELDS_REL = ITEM_FIELDS[:6] + ("micro_positive_relations_wrd",
                                     "micro_negative_relations_wrd",
                                     "micro_positive_relations_loc",
                                     "micro_negative_relations_loc") + ITEM_FIELDS[6:]
