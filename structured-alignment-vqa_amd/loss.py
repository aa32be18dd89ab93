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


def smoothed_loss(logits_concat, logits_vis, logits_syb, answer, mil_nce_obj=None,
                  with_milnce=True, epsilon=0.1):
    """Returns (loss, lsm). lsm is the averaged log-softmax the reference uses for accuracy."""
    return _LossFn.apply(logits_concat, logits_vis, logits_syb, answer, mil_nce_obj,
                         bool(with_milnce and mil_nce_obj is not None), float(epsilon))
