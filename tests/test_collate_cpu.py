"""Batch collation: the oracle's restatement of the
reference collate_fn (both loaders) against the reference's own outputs, and the host
side of the on-device collate (packing, validation, numpy-compatible index rules).
No GPU needed."""
import os

import numpy as np
import pytest

from oracle import collate as ocol

GOLD = os.path.join(os.path.dirname(__file__), "golden", "collate.npz")
CASES = {"onlyobj": dict(B=9, relations=False, fea_dim=16, topN=5, tag="col"),
         "super_node": dict(B=10, relations=True, fea_dim=16, topN=3, tag="colrel")}


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_collate_matches_reference(name):
    gold = np.load(GOLD)
    kw = CASES[name]
    data = ocol.make_samples(**kw)
    res = (ocol.collate_super_node if kw["relations"] else ocol.collate_onlyobj)(data)
    keys = sorted(k.split(":", 1)[1] for k in gold.files if k.startswith(name + ":"))
    assert sorted(res) == keys
    for k in keys:
        g = gold[f"{name}:{k}"]
        assert res[k].dtype == g.dtype and res[k].shape == g.shape, k
        assert np.array_equal(res[k], g), k


@pytest.mark.parametrize("relations", [False, True])
def test_pack_layout_and_offsets(relations):
    from savqa_amd.collate import pack
    data = ocol.make_samples(7, relations=relations, fea_dim=16, topN=3, tag="pk")
    pk = pack(data, relations=relations)
    ref = (ocol.collate_super_node if relations else ocol.collate_onlyobj)(data)
    # dense shapes the device will produce = the reference's
    for k, shp in pk.shapes.items():
        assert tuple(shp) == ref[k].shape, k
    # staging buffer sections are 256-B aligned and the offsets are prefix sums of counts
    for f in pk.fields:
        for k in ("src", "off"):
            assert f[k] is None or f[k] % 256 == 0
    vis = pk.field("vis_fea")
    buf = pk.staging.numpy()
    off = buf[vis["off"]:vis["off"] + 8 * (len(data) + 1)].view(np.int64)
    assert np.array_equal(np.diff(off), [d[0].shape[0] for d in data])


def test_pack_rejects_what_numpy_rejects():
    from savqa_amd.collate import pack
    data = ocol.make_samples(3, fea_dim=8, topN=3, tag="bad", edge_cases=False)
    T = max(d[1].shape[0] for d in data)
    bad = list(data)
    s = list(bad[0])
    s[3] = [[0, T]]  # node index == padded length: IndexError in the reference too
    bad[0] = tuple(s)
    with pytest.raises(IndexError):
        pack(bad)
    s[3] = [[-T - 1, 0]]
    bad[0] = tuple(s)
    with pytest.raises(IndexError):
        pack(bad)
    s[3] = [[-T, T - 1]]  # numpy wraps negatives in [-T, 0)
    bad[0] = tuple(s)
    pack(bad)
    s = list(data[1])
    s[2] = np.arange(40, dtype=np.int64)  # more object locations than padded rows
    bad = [data[0], tuple(s), data[2]]
    with pytest.raises(ValueError):
        pack(bad)


def test_pack_filters_none_samples():
    from savqa_amd.collate import pack
    data = ocol.make_samples(3, fea_dim=8, topN=3, tag="none")
    pk = pack([data[0], None, data[1], data[2], None])
    assert pk.B == 3


def _expand(pk):
    """numpy statement of savqa_collate / savqa_collate_edges (include/savqa.h) over a
    PackedBatch: checks the host plan without a device."""
    import torch
    from savqa_amd.collate import BOX, FILL, ROWS
    npt = {torch.float32: np.float32, torch.int64: np.int64, torch.int32: np.int32}
    buf = pk.staging.numpy()
    B = pk.B
    out = {}
    for f in pk.fields:
        dt = np.dtype(npt[f["dtype"]])
        T, R = f["T"], f["row_elems"]
        d = np.zeros((B, T, R), dt)
        fill = np.array([f["fill"]], np.uint64 if dt.itemsize == 8 else np.uint32).view(dt)[0]
        off = None if f["off"] is None else buf[f["off"]:f["off"] + 8 * (B + 1)].view(np.int64)
        if f["kind"] == ROWS:
            src = buf[f["src"]:].view(np.uint8)
            for b in range(B):
                n = off[b + 1] - off[b]
                rows = src[off[b] * R * dt.itemsize:(off[b] + n) * R * dt.itemsize].view(dt)
                d[b] = fill
                d[b, :n] = rows.reshape(n, R)
        elif f["kind"] == BOX:
            for b in range(B):
                n = off[b + 1] - off[b]
                d[b, :n, :(n if f["square"] else R)] = 1
        else:
            d[:] = fill
        out[f["key"]] = d.reshape(pk.shapes[f["key"]])
    for key, T, o_e, o_off, E in pk.edges:
        eo = buf[o_off:o_off + 8 * (B + 1)].view(np.int64)
        e = buf[o_e:o_e + 8 * E].view(np.int32).reshape(E, 2)
        for b in range(B):
            for i, j in e[eo[b]:eo[b + 1]]:
                out[key][b, i, j] = 1
    return out


@pytest.mark.parametrize("name", list(CASES))
def test_pack_plan_expands_to_reference(name):
    from savqa_amd.collate import OUTPUT_KEYS, pack
    gold = np.load(GOLD)
    kw = CASES[name]
    res = _expand(pack(ocol.make_samples(**kw)))
    keys = [k.split(":", 1)[1] for k in gold.files if k.startswith(name + ":")]
    assert sorted(res) == sorted(keys)
    assert [k for k in OUTPUT_KEYS if k in res] == keys  # the reference's key order
    for k in keys:
        g = gold[f"{name}:{k}"]
        assert res[k].dtype == g.dtype and res[k].shape == g.shape, k
        assert np.array_equal(res[k], g), k



def test_object_location_past_the_macro_nodes_raises():
    """A macro_obj_locs entry >= the padded macro-node count is an IndexError in the
    reference's MIL_NCE (AttModel_x3.py:377-380); pack() raises it on the host (the kernels
    never dereference such a row)."""
    from savqa_amd.collate import pack
    data = ocol.make_samples(3, fea_dim=8, topN=3, tag="loc", edge_cases=False)
    T_s = max(np.asarray(d[1]).reshape(-1).shape[0] for d in data)
    s = list(data[0])
    locs = np.asarray(s[2], dtype=np.int64).reshape(-1).copy()
    locs[0] = T_s
    s[2] = locs
    with pytest.raises(IndexError):
        pack([tuple(s), data[1], data[2]])
    locs[0] = T_s - 1
    s[2] = locs
    pack([tuple(s), data[1], data[2]])
