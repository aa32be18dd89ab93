"""GQA real-data reader: savqa_amd.gqa.GQADataset_super_node
against the reference's own dataset class on a synthetic GQA directory
(oracle/gqa_fixture.py; reference outputs in tests/golden/gqa_reader.npz, produced by
tools/make_golden.py reader with python's `random` seeded per item), then through a
DataLoader whose collate_fn is collate.pack."""
import os
import random

import numpy as np
import pytest

from oracle import collate as ocol
from oracle import gqa_fixture as fx

GOLD = os.path.join(os.path.dirname(__file__), "golden", "gqa_reader.npz")
CASES = {"loc_top5": dict(with_loc=True, pred_rel=False, topN=5),
         "noloc_pred_top3": dict(with_loc=False, pred_rel=True, topN=3)}


def _dataset(root, kw):
    from savqa_amd.gqa import GQADataset_super_node
    return GQADataset_super_node("train", fx.Opt(root, pred_rel=kw["pred_rel"]), "gt_bua_npz.tar",
                                 "train.tar", "gt_bua_npz.tar", kw["topN"],
                                 with_loc=kw["with_loc"], synonyms=fx.SYNONYMS)


@pytest.mark.parametrize("name", list(CASES))
def test_reader_items_match_reference(tmp_path, name):
    gold = np.load(GOLD)
    fx.write_dataset(str(tmp_path))
    ds = _dataset(str(tmp_path), CASES[name])
    assert len(ds) == int(gold[f"{name}:len"])
    n_none = 0
    for i in range(len(ds)):
        random.seed(1000 + i)
        item = ds[i]
        assert (item is None) == bool(gold[f"{name}:{i}:none"]), i
        if item is None:
            n_none += 1
            continue
        for f, v in zip(fx.ITEM_FIELDS, item):
            g = gold[f"{name}:{i}:{f}"]
            a = np.asarray(v)
            assert a.shape == g.shape and a.dtype == g.dtype, (i, f, a.shape, g.shape)
            assert np.array_equal(a, g), (i, f)
    assert 0 < n_none < len(ds)


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
