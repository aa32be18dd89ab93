"""Flat parameter / gradient arena for AttModel.

All 498 reference parameters (state_dict keys unchanged) become views into ONE flat
fp32 buffer laid out MI355X-first:
  * "live" parameters (those the reference's Adam updates in only_obj mode) come
    first, in the order the backward pass FINISHES them, so the gradient all-reduce
    can stream contiguous finished buckets while backward is still running;
  * projections that the engine fuses are adjacent: per encoder layer [Wq;Wk;Wv]
    as one [3d, d] matrix, per stack all 6 decoder cross-attention [Wk_i;Wv_i] as
    one [12d, d] matrix (the 6 decoder layers read the same encoder output);
  * "dead" parameters (never receive a gradient in the reference: v_mlp, input_proj,
    q_mlp, the unused position tables, MIL_NCE.R / rel_mlp / bilinear / marco_mlp,
    mcb sketches, cls_mcb) follow, so Adam and the all-reduce touch only
    [0, n_live).
Every parameter starts on a 64-float (256 B) boundary.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Tuple

import torch
import torch.nn as nn

ALIGN = 64

# The 407000 x 300 GloVe tables (AttModel_x3.py:36-41, :168-171, :295): only the rows of the
# step's token ids receive gradient, so their zero-fill and Adam run row by row.
ROW_TABLES = ("att_vis_grid.syb_emb.weight", "att_syb.syb_emb.weight", "MIL_NCE.syb_emb.weight")


def _live_order(num_blocks: int, only_obj: bool = True) -> List[str]:
    """Live parameter names in backward-completion order (see module docstring). With the
    relation branch (only_obj=False) MIL_NCE.R receives a gradient too (AttModel_x3.py:
    393-401) and joins the live range, last."""
    out: List[str] = []
    for head in ("cls", "cls_vis", "cls_syb"):
        out += [f"{head}.3.weight", f"{head}.3.bias", f"{head}.0.weight", f"{head}.0.bias"]
    for pre in ("att_vis_grid", "att_syb"):
        for i in reversed(range(num_blocks)):
            f = f"{pre}.dec_feed_forward_{i}"
            out += [f"{f}.normalization.gamma", f"{f}.normalization.beta", f"{f}.conv2.weight",
                    f"{f}.conv2.bias", f"{f}.conv1.0.weight", f"{f}.conv1.0.bias"]
            c = f"{pre}.dec_vanilla_attention_{i}"
            out += [f"{c}.normalization.gamma", f"{c}.normalization.beta", f"{c}.Q_proj.0.weight",
                    f"{c}.Q_proj.0.bias"]
            s = f"{pre}.dec_self_attention_{i}"
            out += [f"{s}.normalization.gamma", f"{s}.normalization.beta", f"{s}.V_proj.0.weight",
                    f"{s}.V_proj.0.bias", f"{s}.Q_proj.0.weight", f"{s}.Q_proj.0.bias",
                    f"{s}.K_proj.0.weight", f"{s}.K_proj.0.bias"]
        out += [f"{pre}.dec_emb.lookup_table", f"{pre}.dec_positional_encoding.lookup_table"]
        # fused decoder cross-attention K/V of all layers: weights then biases
        for i in range(num_blocks):
            c = f"{pre}.dec_vanilla_attention_{i}"
            out += [f"{c}.K_proj.0.weight", f"{c}.V_proj.0.weight"]
        for i in range(num_blocks):
            c = f"{pre}.dec_vanilla_attention_{i}"
            out += [f"{c}.K_proj.0.bias", f"{c}.V_proj.0.bias"]
        for i in reversed(range(num_blocks)):
            f = f"{pre}.enc_feed_forward_{i}"
            out += [f"{f}.normalization.gamma", f"{f}.normalization.beta", f"{f}.conv2.weight",
                    f"{f}.conv2.bias", f"{f}.conv1.0.weight", f"{f}.conv1.0.bias"]
            a = f"{pre}.enc_self_attention_{i}"
            out += [f"{a}.normalization.gamma", f"{a}.normalization.beta",
                    f"{a}.Q_proj.0.weight", f"{a}.K_proj.0.weight", f"{a}.V_proj.0.weight",
                    f"{a}.Q_proj.0.bias", f"{a}.K_proj.0.bias", f"{a}.V_proj.0.bias"]
        pos = (f"{pre}.syb_positional_encoding.0.lookup_table" if pre == "att_vis_grid"
               else f"{pre}.syb_positional_encoding.lookup_table")
        out += [pos, f"{pre}.syb_mlp2.weight", f"{pre}.syb_mlp2.bias", f"{pre}.syb_mlp.0.weight",
                f"{pre}.syb_mlp.0.bias", f"{pre}.syb_emb.weight"]
    m = "MIL_NCE"
    out += [f"{m}.ipt_mlp.0.weight", f"{m}.ipt_mlp.0.bias", f"{m}.syb_mlp.0.weight",
            f"{m}.syb_mlp.0.bias", f"{m}.vis_mlp.0.weight", f"{m}.vis_mlp.0.bias",
            f"{m}.syb_emb.weight"]
    if not only_obj:
        out.append(f"{m}.R")
    return out


class ParamArena:
    """Owns the flat parameter and gradient buffers of an AttModel."""

    def __init__(self, model: nn.Module, num_blocks: int, device=None):
        named = OrderedDict(model.named_parameters())
        order = _live_order(num_blocks, bool(getattr(model, "only_obj", True)))
        live = [n for n in order if n in named]
        missing = set(order) - set(named)
        if missing:
            raise RuntimeError(f"ParamArena: model lacks live params {sorted(missing)[:4]}")
        dead = [n for n in named if n not in set(live)]
        self.order = live + dead
        self.offsets: Dict[str, Tuple[int, torch.Size]] = {}
        off = 0
        for n in self.order:
            self.offsets[n] = (off, named[n].shape)
            off += (named[n].numel() + ALIGN - 1) // ALIGN * ALIGN
        self.total = off
        self.n_live = self.offsets[dead[0]][0] if dead else off
        self.live_names = live
        self.params = named
        dev = device if device is not None else next(iter(named.values())).device
        flat = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.flat = flat
        self.grad = None  # allocated on first backward (device of flat)
        self.generation = 0  # bumped by every optimizer update (raw-pointer writes)
        # row tracking of the GloVe tables (savqa_mark_rows / savqa_zero_rows / savqa_adam_rows):
        # name -> uint8 flag per row (bit 0: has Adam state, bit 1: touched since the last zero)
        self.row_tracking = True
        self.row_flags: Dict[str, torch.Tensor] = {}
        if flat.device.type == "meta":  # layout-only arena (host-side tests)
            return
        with torch.no_grad():
            for n in self.order:
                o, shp = self.offsets[n]
                flat[o:o + named[n].numel()].copy_(named[n].detach().reshape(-1))
        self._bind()

    # ------------------------------------------------------------------ views
    def view(self, name: str, buf=None) -> torch.Tensor:
        o, shp = self.offsets[name]
        b = self.flat if buf is None else buf
        n = 1
        for s in shp:
            n *= s
        return b[o:o + n].view(shp)

    def span(self, first: str, last: str, shape, buf=None) -> torch.Tensor:
        """View over the contiguous range first..last (must be adjacent in the arena)."""
        o0, _ = self.offsets[first]
        o1, s1 = self.offsets[last]
        n = 1
        for s in shape:
            n *= s
        if o0 + n != o1 + int(torch.Size(s1).numel()):
            raise RuntimeError(f"ParamArena.span: {first}..{last} is not contiguous")
        b = self.flat if buf is None else buf
        return b[o0:o0 + n].view(shape)

    def _bind(self):
        for n, p in self.params.items():
            p.data = self.view(n)

    def apply(self, fn):
        new = fn(self.flat)
        if new.dtype != torch.float32:
            raise RuntimeError("savqa AttModel parameters are fp32 (flat arena); dtype casts unsupported")
        self.flat = new
        if self.grad is not None and self.grad.device != new.device:
            self.grad = None
            self.row_flags = {}  # recreated with the gradient (optimizer state restarts too)
        self._bind()
        for n in self.live_names:
            self.params[n].grad = None

    # ------------------------------------------------------------------ grads
    def ensure_grads(self):
        """Attach .grad views of the flat gradient buffer to every live parameter.

        If a caller reset grads to None (torch's default zero_grad), the live range is
        zeroed and re-attached, so accumulation semantics match autograd's."""
        if self.grad is None or self.grad.device != self.flat.device:
            self.grad = torch.zeros(self.n_live, dtype=torch.float32, device=self.flat.device)
            reattach = True
        else:
            p0 = self.params[self.live_names[0]]
            reattach = p0.grad is None or p0.grad.data_ptr() != self.grad.data_ptr() + \
                self.offsets[self.live_names[0]][0] * 4
        if reattach:
            self.grad.zero_()
            for n in self.live_names:
                self.params[n].grad = self.view(n, self.grad)
            self._clear_touched()
        if self.row_tracking and not self.row_flags:
            for n in ROW_TABLES:
                if n in self.offsets and n in set(self.live_names):
                    self.row_flags[n] = torch.zeros(self.offsets[n][1][0], dtype=torch.uint8,
                                                    device=self.flat.device)
        return self.grad

    # ------------------------------------------------------------------ row tracking
    def table_width(self, name: str) -> int:
        return int(self.offsets[name][1][1])

    def mark_rows(self, name: str, ids: torch.Tensor):
        """Flag the rows `ids` of table `name` as touched this step (gradient rows written)."""
        f = self.row_flags.get(name)
        if f is not None:
            from . import ops
            ops.mark_rows(ids, f.numel(), f)

    def mark_table_rows(self, offset: int, ids: torch.Tensor):
        """mark_rows for the table that starts at arena offset `offset` (ddp's row exchange)."""
        for n, f in self.row_flags.items():
            if self.offsets[n][0] == offset:
                self.mark_rows(n, ids)

    def mark_all_rows(self, name: str):
        """After a dense update of `name` (its gradient came from an exchange the flags do not
        see): every row may hold Adam state AND a non-zero gradient, so the next zero_grad
        clears the whole table and a later row-tracked step reads every row's gradient."""
        f = self.row_flags.get(name)
        if f is not None:
            f.fill_(3)

    def _clear_touched(self):
        # the whole gradient was just zeroed densely: clear the touched bits with it
        from . import ops
        for n, f in self.row_flags.items():
            o, shp = self.offsets[n]
            ops.zero_rows(self.grad[o:o + shp.numel()], shp[1], shp[0], f)

    def gview(self, name: str) -> torch.Tensor:
        return self.view(name, self.grad)

    def gspan(self, first: str, last: str, shape) -> torch.Tensor:
        return self.span(first, last, shape, self.grad)

    def zero_grad(self):
        """Zero the live gradient range: one memset per dense span, and only the rows touched
        since the last zero in the row-tracked tables."""
        if self.grad is None:
            return
        from . import ops
        lo = 0
        for n, f in sorted(self.row_flags.items(), key=lambda kv: self.offsets[kv[0]][0]):
            o, shp = self.offsets[n]
            if o > lo:
                self.grad[lo:o].zero_()
            ops.zero_rows(self.grad[o:o + shp.numel()], shp[1], shp[0], f)
            lo = o + shp.numel()
        if lo < self.grad.numel():
            self.grad[lo:].zero_()

    def state_key(self):
        """Changes whenever parameter values may have changed: torch in-place edits of the flat
        buffer bump its version counter, optimizer kernels bump `generation`, and in-place
        writes through the Parameters themselves (load_state_dict's copy_, init_params_, any
        stock torch optimizer) bump each Parameter's OWN version counter -- `p.data = view`
        does not share the flat buffer's -- so their sum is part of the key."""
        return (self.flat.data_ptr(), self.flat._version, self.generation,
                sum(p._version for p in self.params.values()))

    def table_ranges(self):
        """Arena ranges of the live 407000 x 300 GloVe tables (row-gathered, never GEMM B
        operands of the low-precision path)."""
        out = []
        for n in self.live_names:
            if n.endswith("syb_emb.weight"):
                o, shp = self.offsets[n]
                out.append((o, o + int(torch.Size(shp).numel())))
        return sorted(out)
