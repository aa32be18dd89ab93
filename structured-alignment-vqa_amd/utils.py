"""Small host utilities: device-side parameter init, checkpoint key conventions, meters."""
from __future__ import annotations

import math
from collections import OrderedDict

import torch


@torch.no_grad()
def init_params_(model, seed: int = 0):
    """Reference-like random init written straight into the device arena (xavier-normal
    for matrices / tables, LN gamma=1 beta=0, small biases); avoids a ~1.1B-parameter
    CPU init + copy on every bench start. Same distributions as the reference's
    constructors, different RNG stream (values never need to match for throughput)."""
    g = torch.Generator(device=model._arena.flat.device)
    g.manual_seed(seed)
    for name, p in model.named_parameters():
        leaf = name.rsplit(".", 1)[-1]
        if leaf == "gamma":
            p.fill_(1.0)
        elif leaf == "beta":
            p.zero_()
        elif p.dim() >= 2:
            fan_out, fan_in = p.shape[0], p.shape[1] * (p[0][0].numel() if p.dim() > 2 else 1)
            std = math.sqrt(2.0 / (fan_in + fan_out))
            p.normal_(0.0, std, generator=g)
            if name.endswith("dec_emb.lookup_table"):
                p[0].zero_()  # embedding(zeros_pad=True), modules.py:30-31
        else:
            bound = 1.0 / math.sqrt(max(1, p.numel()))
            p.uniform_(-bound, bound, generator=g)


def strip_module_prefix(state_dict):
    """DDP checkpoints carry a `module.` prefix (main:428); the eval script strips it
    (eval_itp_grid_ddp_tar_gt.py:107-116)."""
    out = OrderedDict()
    for k, v in state_dict.items():
        out[k[7:] if k.startswith("module.") else k] = v
    return out


def add_module_prefix(state_dict):
    return OrderedDict(("module." + k, v) for k, v in state_dict.items())


class AverageMeter:
    """models/misc.py:46-63."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count
