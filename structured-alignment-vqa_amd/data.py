"""Synthetic batches with the tensor contract of the reference's collate_fn
(models/data_loader_itp_bbox_super_node_onlyobj.py:341-445), generated on device.

The GQA tar/npz/json data is not available offline, so throughput runs use this
generator: relu(N(0,1)) 2048-d region features (pooled
Faster-RCNN features are non-negative), all-valid masks, Bernoulli question /
scene graphs, uniform GloVe ids, macro_obj_loc = region index, uniform answers.
"""
from __future__ import annotations

import torch

PAD = 400000


def synthetic_batch(B: int, Nv: int = 36, Lq: int = 14, Ns: int = 59, topN: int = 5,
                    num_classes: int = 914, seed: int = 1234, device="cuda"):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    dev = device

    def ri(low, high, shape):
        return torch.randint(low, high, shape, generator=g, device=dev, dtype=torch.int64)

    vis = torch.randn(B, Nv, 2048, generator=g, device=dev).clamp_min_(0)
    batch = {
        "vis_fea": vis,
        "vis_mask": torch.ones(B, Nv, Nv, dtype=torch.int32, device=dev),
        "q_ipt": ri(0, PAD, (B, Lq)),
        "q_mask": torch.ones(B, Lq, Lq, dtype=torch.int32, device=dev),
        "q_graph": (torch.rand(B, Lq, Lq, generator=g, device=dev) < 0.2).to(torch.int32),
        "macro_ipt": ri(0, PAD, (B, Ns)),
        "macro_mask": torch.ones(B, Ns, Ns, dtype=torch.int32, device=dev),
        "macro_graph": (torch.rand(B, Ns, Ns, generator=g, device=dev) < 0.05).to(torch.int32),
        "macro_obj_loc": torch.arange(Nv, device=dev, dtype=torch.int64).repeat(B, 1),
        "micro_positive_obj": ri(0, PAD, (B, Nv, topN)),
        "micro_negative_obj": ri(0, PAD, (B, Nv, topN)),
        "micro_obj_mask": torch.ones(B, Nv, topN, dtype=torch.int32, device=dev),
        "answer": ri(1, num_classes, (B,)),
    }
    return batch


MODEL_INPUTS = ("vis_fea", "vis_mask", "q_ipt", "q_mask", "q_graph", "macro_ipt", "macro_mask",
                "macro_graph", "macro_obj_loc", "micro_positive_obj", "micro_negative_obj",
                "micro_obj_mask")


def model_args(batch):
    """Positional args of AttModel.forward (the 4 relation tensors are empty, main:290-308)."""
    B = batch["vis_fea"].shape[0]
    empty = torch.empty((B, 0), device=batch["vis_fea"].device)
    return [batch[k] for k in MODEL_INPUTS] + [empty, empty, empty, empty]
