"""Fused Adam over the flat parameter arena (torch.optim.Adam semantics, main:206/:366).

One HIP launch updates every live parameter: the arena keeps them contiguous, and the
gradient all-reduce's 1/world scaling is folded into the same pass (grad_scale).
Parameters that never receive a gradient (the reference's Adam skips grad=None) lie
outside the live range and are untouched. The three 407000 x 300 GloVe tables run row by
row (savqa_adam_rows): rows never touched have m = v = 0 and no gradient, where
torch.optim.Adam's update is exactly zero, so they are skipped bit-exactly.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import ops

# optim.Adam refreshes the low-precision modes' bf16 weight image in its own pass
# (SAVQA_ADAM_SHADOW=0: leave it to the forward's cast, for A/B runs)
ADAM_SHADOW = os.environ.get("SAVQA_ADAM_SHADOW", "1") != "0"


class Adam(torch.optim.Optimizer):
    def __init__(self, model, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if weight_decay != 0.0:
            raise NotImplementedError("weight_decay (the reference uses none)")
        arena = model._arena
        params = [arena.params[n] for n in arena.live_names]
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0.0))
        self.arena = arena
        self.step_count = 0
        self.m = None
        self.v = None
        self.grad_scale = 1.0

    @torch.no_grad()
    def step(self, closure=None, reducer=None):
        """reducer (ddp.GradReducer): update bucket by bucket as each all-reduce lands,
        with the reducer's 1/world factor; otherwise one launch over the live range."""
        loss = closure() if closure is not None else None
        a = self.arena
        g = a.grad
        if g is None:
            return loss
        if self.m is None or self.m.device != a.flat.device:
            self.m = torch.zeros(a.n_live, dtype=torch.float32, device=a.flat.device)
            self.v = torch.zeros_like(self.m)
        self.step_count += 1
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        t = self.step_count
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        ranges = [(None, 0, a.n_live)]
        scale = self.grad_scale
        active = reducer is not None and getattr(reducer, "active", reducer.world > 1)
        if active:
            works, scale = reducer.drain()
            ranges = works + self._coverage_gaps(reducer, works, a.n_live)
        rows = self._row_tables(reducer if active else None)
        lr, eps = grp["lr"], grp["eps"]
        # the low-precision modes' bf16 weight image (engine.LpShadow over [0, n_live)), written
        # by the same pass when it is current: its refresh then skips the cast of the arena
        sh = getattr(a, "lp_shadow", None) if ADAM_SHADOW else None
        shbuf = sh.buf if sh is not None and sh.current() else None
        for w, lo, hi in ranges:
            if w is not None:
                w.wait()   # this stream waits for this bucket's all-reduce only
            for plo, phi in self._dense_pieces(lo, hi, rows):
                ops.adam(a.flat[plo:phi], g[plo:phi], self.m[plo:phi], self.v[plo:phi], phi - plo,
                         lr, b1, b2, eps, bc1, bc2, scale,
                         shadow=None if shbuf is None else shbuf[plo:phi])
        # row-tracked tables last: every bucket covering them has been waited for by now
        for n in rows:
            o, shp = a.offsets[n]
            e = o + shp.numel()
            ops.adam_rows(a.flat[o:e], g[o:e], self.m[o:e], self.v[o:e], shp[1], shp[0],
                          a.row_flags[n], lr, b1, b2, eps, bc1, bc2, scale)
        for n in a.row_flags:
            if n not in rows:
                a.mark_all_rows(n)  # updated densely: every row may hold Adam state now
        a.generation += 1  # low-precision weight shadows are stale now
        if shbuf is not None:
            sh.arena_updated()  # ... except the bf16 image of the arena, written above
        return loss

    def _row_tables(self, reducer):
        """Tables whose Adam runs row by row this step. The touched-row flags are
        set by the engine's backward from the token ids; a table is row-updated only when
        those flags cover every row whose gradient can be non-zero: on one rank always; with
        GradReducer only the tables it exchanges by rows (it flags the union of all ranks'
        ids); under another data-parallel exchange (e.g. torch DDP) none -- the all-reduced
        gradient has rows other ranks touched."""
        a = self.arena
        if not a.row_flags:
            return ()
        if reducer is not None:
            return tuple(n for n in a.row_flags if reducer.rows_tracked(a.offsets[n][0]))
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            return ()
        return tuple(a.row_flags)

    def _dense_pieces(self, lo, hi, rows):
        """[lo, hi) minus the row-tracked tables."""
        a = self.arena
        out = []
        for n in sorted(rows, key=lambda n: a.offsets[n][0]):
            o, shp = a.offsets[n]
            e = o + shp.numel()
            if e <= lo or o >= hi:
                continue
            if o > lo:
                out.append((lo, o))
            lo = e
        if hi > lo:
            out.append((lo, hi))
        return out

    @staticmethod
    def _coverage_gaps(reducer, works, n_live):
        """All-reduce (densely) every live span the backward never declared final, so no
        rank applies a local-only gradient; overlapping declarations are a bug."""
        gaps, pos = [], 0
        for lo, hi in sorted((lo, hi) for _, lo, hi in works):
            if lo < pos:
                raise RuntimeError(f"gradient ranges declared twice: [{lo}, {hi}) overlaps "
                                   f"[.., {pos})")
            if lo > pos:
                gaps.append((pos, lo))
            pos = hi
        if pos < n_live:
            gaps.append((pos, n_live))
        for lo, hi in gaps:
            reducer._dense(lo, hi)
        extra = reducer.works
        reducer.works = []
        return extra

    def zero_grad(self, set_to_none: bool = False):
        # keep the arena views attached; zero the live gradient range (the row-tracked tables:
        # only the rows touched since the last zero)
        self.arena.zero_grad()
