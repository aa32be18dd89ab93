"""Fused Adam over the flat parameter arena (torch.optim.Adam semantics, main:206/:366).

One HIP launch updates every live parameter: the arena keeps them contiguous, and the
gradient all-reduce's 1/world scaling is folded into the same pass (grad_scale).
Parameters that never receive a gradient (the reference's Adam skips grad=None) lie
outside the live range and are untouched.
"""
from __future__ import annotations

import torch

from . import ops


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
        if reducer is not None and reducer.world > 1:
            works, scale = reducer.drain()
            ranges = works + self._coverage_gaps(reducer, works, a.n_live)
        for w, lo, hi in ranges:
            if w is not None:
                w.wait()   # this stream waits for this bucket's all-reduce only
            ops.adam(a.flat[lo:hi], g[lo:hi], self.m[lo:hi], self.v[lo:hi], hi - lo, grp["lr"], b1,
                     b2, grp["eps"], bc1, bc2, scale)
        a.generation += 1  # low-precision weight shadows are stale now
        return loss

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
        # keep the arena views attached; zero the live gradient range in one memset
        self.arena.zero_grad()
