"""Training loss of main_itp_ddp_tar_super_node.py:335-361 as one fused kernel.

  lsm  = (log_softmax(vis) + log_softmax(syb) + log_softmax(concat)) / 3
  y    = label_smoothing(onehot(answer))          (modules.py:461-463, eps = 0.1)
  loss = mean_b(-sum_c y * lsm) - mil_nce_obj      (with_MILNCE_loss)
The forward kernel also writes d loss / d logits, so the backward is a scale by the
(device-side) upstream gradient: no host synchronisation anywhere.
"""
from __future__ import annotations

import torch

from . import ops


class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lc, lv, ls, answer, mil, with_mil, eps):
        B, Cc = lc.shape
        dev = lc.device
        loss = torch.empty((), dtype=torch.float32, device=dev)
        dlog = torch.empty(3, B, Cc, dtype=torch.float32, device=dev)
        lsm = torch.empty(B, Cc, dtype=torch.float32, device=dev)
        ws = torch.empty(B, dtype=torch.float32, device=dev)
        milt = mil if torch.is_tensor(mil) else torch.zeros((), device=dev)
        ops.loss_fwd(lc.contiguous(), lv.contiguous(), ls.contiguous(),
                     answer.to(device=dev, dtype=torch.int64).contiguous(), B, Cc, eps,
                     milt.contiguous(), with_mil, loss, dlog, lsm, ws)
        ctx.save_for_backward(dlog)
        ctx.with_mil = with_mil and torch.is_tensor(mil)
        ctx.mark_non_differentiable(lsm)
        return loss, lsm

    @staticmethod
    def backward(ctx, gloss, glsm):
        (dlog,) = ctx.saved_tensors
        g = gloss.contiguous()
        out = torch.empty_like(dlog)
        ops.scale_by(dlog, g, dlog.numel(), out)
        dmil = None
        if ctx.with_mil:
            dmil = torch.empty((), dtype=torch.float32, device=g.device)
            ops.affine(g, 1, -1.0, 0.0, dmil)
        return out[0], out[1], out[2], None, dmil, None, None


class _Sum2Fn(torch.autograd.Function):
    """mil_nce_obj + mil_nce_rel on the device (main:326-329: loss += -obj - rel)."""

    @staticmethod
    def forward(ctx, a, b):
        out = torch.empty((), dtype=torch.float32, device=a.device)
        ops.axpby(a.contiguous(), b.contiguous(), 1, 1.0, 1.0, out)
        return out

    @staticmethod
    def backward(ctx, g):
        return g, g


def smoothed_loss(logits_concat, logits_vis, logits_syb, answer, mil_nce_obj=None,
                  with_milnce=True, epsilon=0.1, mil_nce_rel=None):
    """Returns (loss, lsm). lsm is the averaged log-softmax the reference uses for accuracy.
    mil_nce_rel (relation branch, a tensor) is subtracted too, as main:326-329 does."""
    mil = mil_nce_obj
    if mil is not None and torch.is_tensor(mil_nce_rel):
        mil = _Sum2Fn.apply(mil_nce_obj, mil_nce_rel)
    return _LossFn.apply(logits_concat, logits_vis, logits_syb, answer, mil,
                         bool(with_milnce and mil is not None), float(epsilon))
