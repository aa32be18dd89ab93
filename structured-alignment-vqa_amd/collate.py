"""Batch collation with the padding done on the device.

Mirror of the reference's collate_fn
  models/data_loader_itp_bbox_super_node_onlyobj.py:341-445      (only_obj loader)
  dataloader/data_loader_itp_bbox_super_node.py:366-497          (relation loader)
with the same input (a list of per-sample tuples from Dataset.__getitem__, None
entries dropped) and the same output dict (keys, dtypes, shapes, values), split in two:

  pack(data)        host side, usable as DataLoader(collate_fn=pack) in worker
                    processes: validates the samples with numpy's own indexing rules
                    and copies each field's per-sample arrays back to back into ONE
                    uint8 staging tensor (+ per-sample row offsets). No padding, no
                    dense (B,T,T) masks: the staging holds the ragged data only.
  to_device(pk)     one H2D copy of the staging tensor, then savqa_collate (every padded
                    field + the masks, one launch) and savqa_collate_edges (graphs).

`collate_fn(data)` = to_device(pack(data)). There is no host fallback: without the
HIP library / a device, to_device raises.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from . import _lib
from ._lib import CollateField, call

PAD = 400000   # onlyobj:34
LOC_PAD = -1   # onlyobj:39
_ALIGN = 256
ROWS, BOX, FILL = 0, 1, 2

OBJ_FIELDS = ("vis_fea", "macro_nodes_idx", "macro_obj_locs", "macro_edges",
              "micro_positive_nodes_wrd", "micro_negative_nodes_wrd")
REL_FIELDS = ("micro_positive_relations_wrd", "micro_negative_relations_wrd",
              "micro_positive_relations_loc", "micro_negative_relations_loc")
TAIL_FIELDS = ("qnode_idx", "qedge", "answer", "topN")

# AttModel.forward positional order (main_itp_ddp_tar_super_node.py:321-325)
FORWARD_KEYS = ("vis_fea", "vis_fea_mask", "q_ipt", "q_ipt_mask", "q_ipt_graph",
                "macro_node_ipt", "macro_node_mask", "macro_graph_ipt", "macro_obj_loc_ipt",
                "micro_positive_obj_ipt", "micro_negative_obj_ipt", "micro_obj_mask",
                "micro_positive_rel_ipt", "micro_negative_rel_ipt", "micro_positive_rel_loc",
                "micro_negative_rel_loc")

# collate_fn's output keys, in its order (onlyobj:414-444, super_node:466-496)
OUTPUT_KEYS = ("vis_fea", "vis_fea_mask", "macro_node_ipt", "macro_graph_ipt", "macro_node_mask",
               "macro_obj_loc_ipt", "micro_positive_obj_ipt", "micro_negative_obj_ipt",
               "micro_obj_mask", "micro_positive_rel_ipt", "micro_negative_rel_ipt",
               "micro_positive_rel_loc", "micro_negative_rel_loc", "q_ipt", "q_ipt_mask",
               "q_ipt_graph", "answer")

_NP = {torch.float32: np.float32, torch.int64: np.int64, torch.int32: np.int32}


def _bits(value, dtype) -> int:
    return int(np.array([value], dtype=_NP[dtype]).view(
        np.uint64 if _NP[dtype] == np.int64 else np.uint32)[0])


def _edges(edge_lists, T: int, skip_empty: bool):
    """Edge lists of all samples as one int32 [E][2] array in [0, T) + per-sample counts,
    with the reference's rules: np.asarray(edge).astype('int32'); macro lists: empty
    skipped and a flat pair promoted (onlyobj:397-401); graph[row, e[:,0], e[:,1]] = 1 ->
    numpy index semantics (negative indices wrap once, anything outside [-T, T) raises
    IndexError, extra columns unused). T is the batch's padded size, shared by all rows."""
    parts, counts = [], []
    for edge in edge_lists:
        e = np.asarray(edge)
        if e.dtype.kind not in "iu" or e.dtype.itemsize > 4:
            e = e.astype("int32")
        if skip_empty:
            if e.size == 0:
                counts.append(0)
                continue
            if e.ndim == 1:
                e = e[np.newaxis, :]
        if e.ndim != 2 or e.shape[1] < 2:
            raise IndexError(f"edge list of shape {e.shape}: too many indices for array")
        parts.append(e[:, :2])
        counts.append(e.shape[0])
    if not parts:
        return np.zeros((0, 2), np.int32), counts
    e = np.concatenate(parts).astype(np.int32, copy=False)
    if e.size and (e.min() < -T or e.max() >= T):
        raise IndexError(f"edge index out of bounds for graph of size {T}")
    if e.size and e.min() < 0:
        e = np.where(e < 0, e + T, e).astype(np.int32)
    return e, counts


class PackedBatch:
    """Ragged batch in one staging tensor + the plan that expands it on the device."""

    def __init__(self, B, relations, staging, fields, edges, shapes):
        self.B = B
        self.relations = relations
        self.staging = staging   # uint8 CPU tensor (pinned by pin_memory())
        self.fields = fields     # list of dicts, see pack()
        self.edges = edges       # list of (key, T, edge byte offset, offsets byte offset, E)
        self.shapes = shapes     # key -> dense output shape

    def field(self, key):
        return next(f for f in self.fields if f["key"] == key)

    def pin_memory(self):
        """DataLoader(pin_memory=True) calls this in the main process."""
        if not self.staging.is_pinned():
            self.staging = self.staging.pin_memory()
        return self

    @property
    def nbytes(self) -> int:
        return int(self.staging.numel())


class _Layout:
    def __init__(self):
        self.size = 0

    def add(self, nbytes: int) -> int:
        o = self.size
        self.size += (nbytes + _ALIGN - 1) // _ALIGN * _ALIGN
        return o


def pack(data, relations: Optional[bool] = None,
         staging: Optional[torch.Tensor] = None) -> PackedBatch:
    """Host half of collate_fn: validate + copy the ragged arrays into one staging buffer.
    staging: an optional reusable (e.g. pinned) uint8 buffer, used when large enough
    (the caller must not refill it while a copy out of it is in flight; StagingRing)."""
    data = [d for d in data if d is not None]
    if not data:
        raise ValueError("collate: empty batch")
    if relations is None:
        relations = len(data[0]) == len(OBJ_FIELDS) + len(REL_FIELDS) + len(TAIL_FIELDS)
    names = OBJ_FIELDS + (REL_FIELDS if relations else ()) + TAIL_FIELDS
    if any(len(d) != len(names) for d in data):
        raise ValueError(f"collate: every sample must be a {len(names)}-tuple")
    cols = {k: [d[i] for d in data] for i, k in enumerate(names)}
    B = len(data)
    topN = int(cols["topN"][0])

    vis = [np.asarray(v, dtype=np.float32) for v in cols["vis_fea"]]
    D = vis[0].shape[1]
    if any(v.ndim != 2 or v.shape[1] != D for v in vis):
        raise ValueError("collate: vis_fea rows must share one feature size")
    T_v = max(v.shape[0] for v in vis)
    nodes = [np.asarray(n, dtype=np.int64).reshape(-1) for n in cols["macro_nodes_idx"]]
    T_s = max(n.shape[0] for n in nodes)
    qn = [np.asarray(n, dtype=np.int64).reshape(-1) for n in cols["qnode_idx"]]
    T_q = max(n.shape[0] for n in qn)

    def rows_of(arrs, R, T, what):
        out = []
        shape_ok = (lambda a: a.ndim == 2 and a.shape[1] == R) if R > 1 else \
            (lambda a: a.ndim == 1)
        for a in arrs:
            a = np.asarray(a, dtype=np.int64)
            if a.size == 0:  # nothing to place (e.g. a single-object image's relations)
                out.append(np.zeros((0, R) if R > 1 else (0,), np.int64))
                continue
            n = a.shape[0] if a.ndim else 1
            if n > T:
                raise ValueError(f"collate: {what} has {n} rows, more than the padded {T}")
            # numpy assignment semantics: the sample broadcasts into its (n, R) slot
            out.append(a if shape_ok(a) else np.broadcast_to(a, (n, R) if R > 1 else (n,)))
        return out

    locs = rows_of(cols["macro_obj_locs"], 1, T_v, "macro_obj_locs")
    if any(l.size and int(l.max()) >= T_s for l in locs):
        # the model would index new_macro_ipt past its T_s rows: the reference's MIL_NCE raises
        # IndexError there (AttModel_x3.py:377-380); the kernels never dereference such a row
        raise IndexError(f"collate: a macro_obj_locs entry is >= the {T_s} macro nodes")
    pos = rows_of(cols["micro_positive_nodes_wrd"], topN, T_v, "micro_positive_nodes_wrd")
    neg = rows_of(cols["micro_negative_nodes_wrd"], topN, T_v, "micro_negative_nodes_wrd")
    macro_edges = _edges(cols["macro_edges"], T_s, True)
    q_edges = _edges(cols["qedge"], T_q, False)
    answer = np.stack(cols["answer"], axis=0).astype(np.int64).reshape(B, -1)
    if answer.shape[1] != 1:
        raise ValueError("collate: one answer per sample")

    # field plan: (key, kind, torch dtype, T, row_elems, fill, per-sample arrays | count key)
    plan = [("vis_fea", ROWS, torch.float32, T_v, D, 0.0, vis),
            ("vis_fea_mask", BOX, torch.int32, T_v, T_v, 1, "vis_fea"),
            ("macro_node_ipt", ROWS, torch.int64, T_s, 1, PAD, nodes),
            ("macro_graph_ipt", FILL, torch.int32, T_s, T_s, 0, None),
            ("macro_node_mask", BOX, torch.int32, T_s, T_s, 1, "macro_node_ipt"),
            ("macro_obj_loc_ipt", ROWS, torch.int64, T_v, 1, LOC_PAD, locs),
            ("micro_positive_obj_ipt", ROWS, torch.int64, T_v, topN, PAD, pos),
            ("micro_negative_obj_ipt", ROWS, torch.int64, T_v, topN, PAD, neg),
            ("micro_obj_mask", BOX, torch.int32, T_v, topN, 0, "macro_obj_loc_ipt")]
    if relations:  # super_node:422-439 (a sample without positives keeps only padding)
        prw = [np.asarray(a).astype(np.int64).reshape(-1)
               for a in cols["micro_positive_relations_wrd"]]
        T_r = max(a.shape[0] for a in prw)
        keep = [a.shape[0] != 0 for a in prw]

        def only_kept(name):  # samples without positives are never read (super_node:434)
            return [a if k else () for a, k in zip(cols[name], keep)]
        nrw = rows_of(only_kept("micro_negative_relations_wrd"), 1, T_r,
                      "micro_negative_relations_wrd")
        prl = rows_of(only_kept("micro_positive_relations_loc"), 5, T_r,
                      "micro_positive_relations_loc")
        nrl = rows_of(only_kept("micro_negative_relations_loc"), 4, T_r,
                      "micro_negative_relations_loc")
        plan += [("micro_positive_rel_ipt", ROWS, torch.int64, T_r, 1, PAD, prw),
                 ("micro_negative_rel_ipt", ROWS, torch.int64, T_r, 1, PAD, nrw),
                 ("micro_positive_rel_loc", ROWS, torch.int64, T_r, 5, LOC_PAD, prl),
                 ("micro_negative_rel_loc", ROWS, torch.int64, T_r, 4, LOC_PAD, nrl)]
    plan += [("q_ipt", ROWS, torch.int64, T_q, 1, PAD, qn),
             ("q_ipt_mask", BOX, torch.int32, T_q, T_q, 1, "q_ipt"),
             ("q_ipt_graph", FILL, torch.int32, T_q, T_q, 0, None),
             ("answer", ROWS, torch.int64, 1, 1, 0, list(answer))]

    lay = _Layout()
    fields, offsets_of, writes = [], {}, []
    for key, kind, dt, T, R, fill, srcs in plan:
        f = dict(key=key, kind=kind, dtype=dt, T=T, row_elems=R,
                 square=int(kind == BOX and key != "micro_obj_mask"),
                 fill=_bits(fill, dt) if kind != BOX else 0, src=None, off=None)
        if kind == ROWS:
            counts = np.array([a.shape[0] if np.ndim(a) else 1 for a in srcs], np.int64)
            off = np.zeros(B + 1, np.int64)
            np.cumsum(counts, out=off[1:])
            item = np.dtype(_NP[dt]).itemsize
            f["off"] = lay.add(8 * (B + 1))
            f["src"] = lay.add(int(off[-1]) * R * item)
            writes.append((f["off"], off, None))
            writes.append((f["src"], srcs, _NP[dt]))
            offsets_of[key] = f["off"]
        elif kind == BOX:
            f["off"] = offsets_of[srcs]
        fields.append(f)
    edges = []
    for key, T, (e_all, counts) in (("macro_graph_ipt", T_s, macro_edges),
                                    ("q_ipt_graph", T_q, q_edges)):
        off = np.zeros(B + 1, np.int64)
        np.cumsum(np.asarray(counts, np.int64), out=off[1:])
        E = int(off[-1])
        o_off = lay.add(8 * (B + 1))
        o_e = lay.add(8 * E)
        writes.append((o_off, off, None))
        writes.append((o_e, [e_all], np.int32))
        edges.append((key, T, o_e, o_off, E))

    need = max(lay.size, _ALIGN)
    if staging is None or staging.numel() < need:
        staging = torch.empty(need, dtype=torch.uint8)
    else:
        staging = staging[:need]
    buf = staging.numpy()
    for o, arr, dt in writes:
        if dt is None:  # offsets
            buf[o:o + arr.nbytes] = arr.view(np.uint8)
            continue
        parts = [np.asarray(a).reshape(-1) for a in arr]
        n = sum(p.shape[0] for p in parts)
        if n:  # one C-level copy of every sample's rows into the section
            np.concatenate(parts, out=buf[o:o + n * np.dtype(dt).itemsize].view(dt),
                           casting="same_kind")
    shapes = {f["key"]: ((B, f["T"], f["row_elems"]) if f["row_elems"] > 1 or f["kind"] != ROWS
                         else (B, f["T"])) for f in fields}
    shapes["answer"] = (B,)
    return PackedBatch(B, relations, staging, fields, edges, shapes)


class DeviceBatch:
    """Dense outputs of one packed batch + the launch arguments that fill them
    (built once; launch() may be repeated, e.g. to time the kernels)."""

    def __init__(self, pk: PackedBatch, device, staging_dev: torch.Tensor):
        self.pk = pk
        self.device = device
        self.staging_dev = staging_dev  # keeps the packed bytes alive until the launch
        base = staging_dev.data_ptr()
        self.out = {}
        self.args = (CollateField * len(pk.fields))()
        for i, f in enumerate(pk.fields):
            t = torch.empty(pk.shapes[f["key"]], dtype=f["dtype"], device=device)
            self.out[f["key"]] = t
            c = self.args[i]
            c.kind, c.square, c.reserved = f["kind"], f["square"], 0
            c.elem_bytes = t.element_size()
            c.T, c.row_elems, c.fill = f["T"], f["row_elems"], f["fill"]
            c.src = base + f["src"] if f["src"] is not None else None
            c.off = base + f["off"] if f["off"] is not None else None
            c.dst = t.data_ptr()
        self.edges = [(base + o_e, base + o_off, E, T, self.out[key].data_ptr())
                      for key, T, o_e, o_off, E in pk.edges]

    def launch(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        with torch.cuda.device(self.device):
            call("savqa_collate", s, self.args, len(self.pk.fields), self.pk.B)
            for e, eo, E, T, g in self.edges:
                call("savqa_collate_edges", s, e, eo, self.pk.B, E, T, g)

    def result(self) -> Dict[str, torch.Tensor]:
        return {k: self.out[k] for k in OUTPUT_KEYS if k in self.out}  # reference key order


def to_device(pk: PackedBatch, device=None, staging_dev: Optional[torch.Tensor] = None
              ) -> Dict[str, torch.Tensor]:
    """Device half of collate_fn: one H2D copy + two launches on the current stream.
    staging_dev: the staging bytes already in HBM (skips the copy)."""
    device = torch.device(device) if device is not None else \
        torch.device("cuda", torch.cuda.current_device())
    if device.type != "cuda":
        raise _lib.SavqaError("collate.to_device needs a HIP device (no host fallback)")
    _lib.load()  # raises when the library is missing
    if staging_dev is None:
        staging_dev = torch.empty(pk.staging.numel(), dtype=torch.uint8, device=device)
        staging_dev.copy_(pk.staging, non_blocking=pk.staging.is_pinned())
    db = DeviceBatch(pk, device, staging_dev)
    db.launch()
    return db.result()


class StagingRing:
    """Reusable pinned staging buffers for in-process collation: buffer i is refilled
    only after the H2D copy that last read it has completed (event per buffer), so the
    host never pays fresh-page faults or pinning per batch."""

    def __init__(self, depth: int = 2):
        self.bufs = [None] * depth
        self.events = [None] * depth
        self.i = 0

    def collate(self, data, relations: Optional[bool] = None, device=None):
        k = self.i
        self.i = (self.i + 1) % len(self.bufs)
        if self.events[k] is not None:
            self.events[k].synchronize()
        pk = pack(data, relations, staging=self.bufs[k])
        if self.bufs[k] is None or pk.staging.data_ptr() != self.bufs[k].data_ptr():
            pk.pin_memory()
            self.bufs[k] = pk.staging
        res = to_device(pk, device)
        ev = torch.cuda.Event()
        ev.record()
        self.events[k] = ev
        return res


def collate_fn(data, device=None) -> Dict[str, torch.Tensor]:
    """The reference collate_fn with its output already in HBM."""
    return to_device(pack(data), device)


def forward_inputs(batch: Dict[str, torch.Tensor]) -> List[torch.Tensor]:
    """Positional inputs of AttModel.forward (main:321-325); the relation tensors are
    empty (B, 0) for the only_obj loader (main:290-308)."""
    B = batch["vis_fea"].shape[0]
    empty = torch.empty((B, 0), device=batch["vis_fea"].device)
    return [batch[k] if k in batch else empty for k in FORWARD_KEYS]
