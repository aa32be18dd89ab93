"""GQA real-data reader: savqa_amd.gqa.GQADataset_super_node
against the reference's own dataset class on a synthetic GQA directory
(oracle/gqa_fixture.py; reference outputs in tests/golden/gqa_reader.npz, produced by
tools/make_golden.py reader with python's `random` seeded per item), then through a
DataLoader whose collate_fn is collate.pack."""
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from oracle import collate as ocol
from oracle import gqa_fixture as fx

GOLD = os.path.join(os.path.dirname(__file__), "golden", "gqa_reader.npz")
CASES = {"loc_top5": dict(with_loc=True, pred_rel=False, topN=5),
         "noloc_pred_top3": dict(with_loc=False, pred_rel=True, topN=3),
         "rel_loc_top3": dict(with_loc=True, pred_rel=False, topN=3, rel=True),
         "rel_noloc_top2": dict(with_loc=False, pred_rel=False, topN=2, rel=True)}


def _dataset(root, kw):
    from savqa_amd.gqa import GQADataset_super_node, GQADataset_super_node_rel
    cls = GQADataset_super_node_rel if kw.get("rel") else GQADataset_super_node
    return cls("train", fx.Opt(root, pred_rel=kw["pred_rel"]), "gt_bua_npz.tar", "train.tar",
               "gt_bua_npz.tar", kw["topN"], with_loc=kw["with_loc"], synonyms=fx.SYNONYMS)


def compare_case(root, name):
    """Every item of case `name` equals the reference's (golden), None items included."""
    gold = np.load(GOLD)
    kw = CASES[name]
    fields = fx.ITEM_FIELDS_REL if kw.get("rel") else fx.ITEM_FIELDS
    ds = _dataset(root, kw)
    assert len(ds) == int(gold[f"{name}:len"])
    n_none = 0
    for i in range(len(ds)):
        random.seed(1000 + i)
        item = ds[i]
        assert (item is None) == bool(gold[f"{name}:{i}:none"]), i
        if item is None:
            n_none += 1
            continue
        assert len(item) == len(fields)
        for f, v in zip(fields, item):
            g = gold[f"{name}:{i}:{f}"]
            a = np.asarray(v)
            assert a.shape == g.shape and a.dtype == g.dtype, (i, f, a.shape, g.shape)
            assert np.array_equal(a, g), (i, f)
    assert 0 < n_none < len(ds)


@pytest.mark.parametrize("name", list(CASES))
def test_reader_items_match_reference(tmp_path, name):
    fx.write_dataset(str(tmp_path))
    if not CASES[name].get("rel") or os.environ.get("PYTHONHASHSEED") == "0":
        compare_case(str(tmp_path), name)
        return
    # the relation loader's category order is python's set order of the relation names,
    # i.e. it follows PYTHONHASHSEED (the golden was made with 0): compare in a child
    here = os.path.abspath(__file__)
    code = ("import importlib.util, sys; sys.path.insert(0, %r); "
            "s = importlib.util.spec_from_file_location('t', %r); m = importlib.util.module_from_spec(s); "
            "s.loader.exec_module(m); m.compare_case(%r, %r)"
            % (os.path.dirname(os.path.dirname(here)), here, str(tmp_path), name))
    env = dict(os.environ, PYTHONHASHSEED="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]


def test_reader_feeds_pack_through_a_dataloader(tmp_path):
    import torch.utils.data as tud
    from savqa_amd.collate import pack
    fx.write_dataset(str(tmp_path))
    ds = _dataset(str(tmp_path), CASES["loc_top5"])
    random.seed(7)
    items = [ds[i] for i in range(len(ds))]
    random.seed(7)
    dl = tud.DataLoader(ds, batch_size=len(ds), shuffle=False, collate_fn=pack, num_workers=0)
    pk = next(iter(dl))
    kept = [x for x in items if x is not None]
    assert pk.B == len(kept)
    ref = ocol.collate_onlyobj(kept)  # the reference collate on the same items
    for k, shp in pk.shapes.items():
        assert tuple(shp) == ref[k].shape, k


def test_relation_reader_items_pack_like_the_reference_collate(tmp_path):
    """Relation-loader items (incl. single-object images without relation rows) through
    collate.pack expand to the reference super_node collate_fn's tensors."""
    from savqa_amd.collate import pack
    from test_collate_cpu import _expand
    fx.write_dataset(str(tmp_path), n_questions=16)
    ds = _dataset(str(tmp_path), dict(with_loc=True, pred_rel=False, topN=2, rel=True))
    random.seed(3)
    kept = [x for x in (ds[i] for i in range(len(ds))) if x is not None]
    assert any(x[6].shape[0] == 0 for x in kept) and any(x[6].shape[0] > 0 for x in kept)
    ref = ocol.collate_super_node(kept)
    got = _expand(pack(kept))
    for k in ref:
        assert np.array_equal(ref[k], got[k]), k


def test_spawned_loader_workers(tmp_path):
    """Once the device is initialised train.gqa_loaders spawns its workers instead of
    forking them: the dataset (tar index without the parent's handle) and collate.pack
    must cross a spawn boundary and yield the same batches as in-process loading."""
    import torch.utils.data as tud
    from savqa_amd.gqa import GQADataset_super_node
    from savqa_amd.collate import pack
    fx.write_dataset(str(tmp_path), n_questions=16)
    ds = _dataset(str(tmp_path), dict(with_loc=True, pred_rel=False, topN=5))
    ds[0]  # opens the tar handle in this process; it must not be pickled
    kw = dict(batch_size=4, drop_last=True, collate_fn=pack, shuffle=False)
    here = [pk.B for pk in tud.DataLoader(ds, num_workers=0, **kw)]
    there = [pk.B for pk in tud.DataLoader(ds, num_workers=2, multiprocessing_context="spawn",
                                           **kw)]
    assert isinstance(ds, GQADataset_super_node)
    assert here == there and len(here) > 0
