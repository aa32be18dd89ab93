"""Model API mirroring the reference's models/AttModel_x3.py (model_v=3).

Same classes (AttModel_vis_grid, AttModel_syb, MIL_NCE, CompactBilinearPooling,
AttModel), constructor signatures, attribute names and parameter registration
order, so the 498 state_dict keys are identical and checkpoints interchange both
ways (DDP's `module.` prefix is handled by utils.strip_module_prefix).

AttModel.forward(16 tensors, decMask, mcb) returns (logits_concat, logits_vis,
logits_syb, mil_nce_obj, mil_nce_rel) exactly like AttModel_x3.py:512-542, but the
whole forward is ONE autograd node whose body is the libsavqa kernel chain in
engine.py; parameters live in one flat fp32 arena (params.py).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
from torch.nn.parameter import Parameter

from .engine import ModelEngine
from .modules import embedding, feedforward, label_smoothing, multihead_attention, \
    new_multihead_attention
from .params import ParamArena

PAD = 400000          # AttModel_x3.py:13
UNK = 400001
END = 400003
INVALID = 400003
VIS_PAD = -1
LOC_PAD = -1
VOCAB = 407000        # AttModel_x3.py:36 (GloVe 400k + 7000 extra rows)


def _glove_table(glove, init: bool):
    t = torch.empty(VOCAB, 300)
    if init:
        nn.init.xavier_normal_(t)
        if glove is not None and getattr(glove, "vectors", None) is not None:
            v = glove.vectors
            t[:v.shape[0], :] = v
    return t


class AttModel_vis_grid(nn.Module):
    """AttModel_x3.py:20-156 (parameters; the forward runs inside AttModel's engine)."""

    def __init__(self, glove, hidden_size, maxlen, maxlen_q, num_blocks, num_heads, dropout_rate,
                 maxlen_v, num_classes, _init=True):
        super().__init__()
        self.hidden_size = hidden_size
        self.num_blocks = num_blocks
        self.num_heads = num_heads
        self.maxlen_q = maxlen_q
        self.maxlen = maxlen
        self.dropout_rate = dropout_rate
        self.enc_dropout = nn.Dropout(dropout_rate)
        self.dec_dropout = nn.Dropout(dropout_rate)
        self.syb_emb = nn.Embedding.from_pretrained(_glove_table(glove, _init), freeze=False)
        self.syb_mlp = nn.Sequential(nn.Linear(300, 2048), nn.ReLU(inplace=True))
        self.syb_mlp2 = nn.Linear(2048, hidden_size)
        self.v_mlp = nn.Sequential(nn.Linear(2048, hidden_size), nn.ReLU(inplace=True),
                                   nn.Linear(hidden_size, hidden_size))
        self.v_positional_encoding = nn.Sequential(
            embedding(maxlen_v, hidden_size, zeros_pad=False, scale=False), nn.Dropout(dropout_rate))
        self.input_proj = nn.Linear(2048, hidden_size)
        for i in range(num_blocks):
            self.__setattr__('enc_self_attention_%d' % i, new_multihead_attention(
                num_units=hidden_size, num_heads=num_heads, dropout_rate=0, causality=False))
            self.__setattr__('enc_feed_forward_%d' % i, feedforward(hidden_size, [4 * hidden_size,
                                                                                 hidden_size]))
        self.q_mlp = nn.Sequential(nn.Linear(300, hidden_size), nn.ReLU(inplace=True),
                                   nn.Linear(hidden_size, hidden_size))
        self.q_positional_encoding = nn.Sequential(
            embedding(maxlen_q, hidden_size, zeros_pad=False, scale=False), nn.Dropout(dropout_rate))
        self.syb_positional_encoding = nn.Sequential(
            embedding(maxlen, hidden_size, zeros_pad=False, scale=False), nn.Dropout(dropout_rate))
        self.dec_emb = embedding(num_classes, hidden_size, scale=True)
        self.dec_positional_encoding = embedding(maxlen, hidden_size, zeros_pad=False, scale=False)
        for i in range(num_blocks):
            self.__setattr__('dec_self_attention_%d' % i, multihead_attention(
                num_units=hidden_size, num_heads=num_heads, dropout_rate=0, causality=True))
            self.__setattr__('dec_vanilla_attention_%d' % i, new_multihead_attention(
                num_units=hidden_size, num_heads=num_heads, dropout_rate=0, causality=False))
            self.__setattr__('dec_feed_forward_%d' % i, feedforward(hidden_size, [4 * hidden_size,
                                                                                 hidden_size]))

    def forward(self, *a, **k):
        raise RuntimeError("AttModel_vis_grid runs inside AttModel.forward (savqa engine)")


class AttModel_syb(nn.Module):
    """AttModel_x3.py:158-282."""

    def __init__(self, glove, hidden_size, maxlen, maxlen_q, num_blocks, num_heads, dropout_rate,
                 num_classes, _init=True):
        super().__init__()
        self.num_blocks = num_blocks
        self.num_heads = num_heads
        self.hidden_size = hidden_size
        self.dropout_rate = dropout_rate
        self.maxlen = maxlen
        self.maxlen_q = maxlen_q
        self.syb_emb = nn.Embedding.from_pretrained(_glove_table(glove, _init), freeze=False)
        self.syb_mlp = nn.Sequential(nn.Linear(300, 2048), nn.ReLU(inplace=True))
        self.syb_mlp2 = nn.Linear(2048, hidden_size)
        self.enc_dropout = nn.Dropout(dropout_rate)
        self.syb_positional_encoding = embedding(maxlen + maxlen_q, hidden_size, zeros_pad=False,
                                                 scale=False)
        self.q_mlp = nn.Sequential(nn.Linear(300, hidden_size), nn.Linear(hidden_size, hidden_size))
        self.q_positional_encoding = nn.Sequential(
            embedding(maxlen_q, hidden_size, zeros_pad=False, scale=False), nn.Dropout(dropout_rate))
        self.dec_emb = embedding(num_classes, hidden_size, scale=True)
        self.dec_positional_encoding = embedding(maxlen + maxlen_q, hidden_size, zeros_pad=False,
                                                 scale=False)
        self.dec_dropout = nn.Dropout(dropout_rate)
        for i in range(num_blocks):
            self.__setattr__('dec_self_attention_%d' % i, multihead_attention(
                num_units=hidden_size, num_heads=num_heads, dropout_rate=0, causality=True))
            self.__setattr__('dec_vanilla_attention_%d' % i, new_multihead_attention(
                num_units=hidden_size, num_heads=num_heads, dropout_rate=0, causality=False))
            self.__setattr__('dec_feed_forward_%d' % i, feedforward(hidden_size, [4 * hidden_size,
                                                                                 hidden_size]))
        for i in range(num_blocks):
            self.__setattr__('enc_self_attention_%d' % i, new_multihead_attention(
                num_units=hidden_size, num_heads=num_heads, dropout_rate=0, causality=False))
            self.__setattr__('enc_feed_forward_%d' % i, feedforward(hidden_size, [4 * hidden_size,
                                                                                 hidden_size]))

    def forward(self, *a, **k):
        raise RuntimeError("AttModel_syb runs inside AttModel.forward (savqa engine)")


class MIL_NCE(nn.Module):
    """AttModel_x3.py:285-443 (parameters; both the only_obj branch :352-380 and the relation
    branch :382-440 run inside AttModel's engine -- engine.mil_forward / csrc/rel.hip)."""

    def __init__(self, glove, hidden_size, dropout_rate, num_relations, only_obj, _init=True):
        super().__init__()
        self.only_obj = only_obj
        self.dropout_rate = dropout_rate
        self.num_relations = num_relations
        self.hidden_size = hidden_size
        self.R = Parameter(torch.empty(num_relations, hidden_size, hidden_size))
        if _init:
            nn.init.xavier_normal_(self.R)
        self.syb_emb = nn.Embedding.from_pretrained(_glove_table(glove, _init), freeze=False)
        self.marco_mlp = nn.Sequential(nn.Linear(300, hidden_size), nn.ReLU(inplace=True))
        self.syb_mlp = nn.Sequential(nn.Linear(300, hidden_size), nn.ReLU(inplace=True))
        self.vis_mlp = nn.Sequential(nn.Linear(2048, hidden_size), nn.ReLU(inplace=True))
        self.rel_mlp = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.ReLU(inplace=True),
                                     nn.Linear(hidden_size, 1))
        self.softmax = torch.nn.Softmax(dim=2)
        self.softmax_bilinear = torch.nn.Softmax(dim=0)
        self.bilinear = nn.Bilinear(hidden_size, hidden_size, num_relations, bias=False)
        self.ipt_mlp = nn.Sequential(nn.Linear(hidden_size, 2048), nn.ReLU(inplace=True))

    def forward(self, *a, **k):
        raise RuntimeError("MIL_NCE runs inside AttModel.forward (savqa engine)")


class CompactBilinearPooling(nn.Module):
    """AttModel_x3.py:444-469. Parameters only: the mcb path needs torch.rfft (removed
    from torch >= 1.8) and is off in the published config; forward raises."""

    def __init__(self, input_dims, output_dim):
        super().__init__()
        self.output_dim = output_dim

        def sketch(input_dim):
            h = torch.randint(output_dim, size=(input_dim,))
            s = (2 * torch.randint(2, size=(input_dim,)) - 1).float()
            m = torch.zeros(input_dim, output_dim)
            m[torch.arange(input_dim), h] = s
            return m

        self.sketch1 = nn.Parameter(sketch(input_dims), requires_grad=False)
        self.sketch2 = nn.Parameter(sketch(input_dims), requires_grad=False)

    def forward(self, x1, x2):
        raise NotImplementedError("mcb=True (CompactBilinearPooling) is out of scope")


class _AttModelFn(torch.autograd.Function):
    """The whole AttModel.forward as one autograd node. Its inputs are the batch tensors AND
    every live Parameter: the backward writes the parameter gradients straight into the
    flat gradient arena (the Parameters' .grad views) and returns None for them, but having
    the Parameters as inputs puts their AccumulateGrad nodes into the graph, so everything
    that hooks gradient accumulation sees each parameter become ready after the backward:
    torch's DistributedDataParallel (main:203, find_unused_parameters=True) then averages
    the arena's gradients in place (its bucket copies read and write .grad): DDP hooks the
    AccumulateGrad NODES, whose hooks the engine runs after each. Per-tensor
    register_post_accumulate_grad_hook hooks do NOT fire: AccumulateGrad returns before
    them for an undefined incoming gradient -- read .grad after backward() instead."""

    @staticmethod
    def forward(ctx, model, decMask, drop, ntensors, *args):
        tensors = args[:ntensors]
        inp = dict(zip(_INPUT_NAMES + _REL_NAMES, tensors))
        if model.__dict__.get("_vis_scale") is not None:
            inp["vis_fea_scale"] = model._vis_scale
        (lc, lv, ls, mil, mil_rel), saved = model._engine.forward(inp, decMask, drop)
        ctx.model = model
        ctx.saved = saved
        ctx.nargs = len(args)
        ctx.rel = mil_rel is not None
        if mil_rel is None:
            mil_rel = torch.zeros((), device=mil.device)
            ctx.mark_non_differentiable(mil_rel)
        return lc, lv, ls, mil, mil_rel

    @staticmethod
    def backward(ctx, dlc, dlv, dls, dmil, dmil_rel):
        model = ctx.model
        dev = model._arena.flat.device

        def z(g, shape):
            return g.contiguous() if g is not None else torch.zeros(shape, device=dev)

        B = ctx.saved[1].B
        Cc = model.num_classes
        red = model.__dict__.get("_reducer")
        if red is not None:
            red.prepare_rows()           # on the backward's main stream
        model._engine.backward(ctx.saved, z(dlc, (B, Cc)), z(dlv, (B, Cc)), z(dls, (B, Cc)),
                               z(dmil, ()), on_range=red.reduce_range if red else None,
                               dmil_rel=z(dmil_rel, ()) if ctx.rel else None)
        ctx.saved = None
        return (None, None, None, None) + (None,) * ctx.nargs


_INPUT_NAMES = ("vis_fea", "vis_mask", "q_ipt", "q_mask", "q_graph", "macro_ipt", "macro_mask",
                "macro_graph", "macro_obj_loc", "micro_positive_obj", "micro_negative_obj",
                "micro_obj_mask")
_REL_NAMES = ("micro_positive_rel", "micro_positive_rel_loc", "micro_negative_rel_loc")


class AttModel(nn.Module):
    """AttModel_x3.py:471-542."""

    def __init__(self, glove, hidden_size, hidden_size_mil, num_classes, maxlen_q, maxlen, maxlen_v,
                 num_blocks, num_heads, dropout_rate, dropout_rate_mcb, num_relations, only_obj,
                 device=None, init=True, gemm_precision="fp32"):
        super().__init__()
        self.only_obj = only_obj
        self.num_classes = num_classes
        self.maxlen_q = maxlen_q
        self.hidden_size = hidden_size
        self.num_blocks = num_blocks
        self.num_heads = num_heads
        self.dropout_rate = dropout_rate
        self.att_vis_grid = AttModel_vis_grid(glove, hidden_size, maxlen, maxlen_q, num_blocks,
                                              num_heads, dropout_rate, maxlen_v, num_classes, init)
        self.att_syb = AttModel_syb(glove, hidden_size, maxlen, maxlen_q, num_blocks, num_heads,
                                    dropout_rate, num_classes, init)
        self.MIL_NCE = MIL_NCE(glove, hidden_size_mil, dropout_rate, num_relations, self.only_obj,
                               init)
        self.cls = nn.Sequential(nn.Linear(hidden_size * 2, hidden_size), nn.ReLU(),
                                 nn.Dropout(dropout_rate, inplace=True),
                                 nn.Linear(hidden_size, num_classes))
        self.cls_vis = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.ReLU(),
                                     nn.Dropout(dropout_rate, inplace=True),
                                     nn.Linear(hidden_size, num_classes))
        self.cls_syb = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.ReLU(),
                                     nn.Dropout(dropout_rate, inplace=True),
                                     nn.Linear(hidden_size, num_classes))
        self.mcb_out = 16000
        self.mcb = CompactBilinearPooling(hidden_size, self.mcb_out)
        self.mcb_dropout = nn.Dropout(dropout_rate_mcb)
        self.cls_mcb = nn.Sequential(nn.Linear(self.mcb_out, hidden_size), nn.ReLU(),
                                     nn.Dropout(dropout_rate, inplace=True),
                                     nn.Linear(hidden_size, num_classes))
        self.label_smoothing = label_smoothing()
        # flatten every parameter into the arena (state_dict keys unchanged)
        object.__setattr__(self, "_arena", ParamArena(self, num_blocks, device=device))
        # gemm_precision (engine.ModelEngine): "fp32" (default, fp32 GEMMs; "fp32_native" forces
        # the v_mfma_f32_16x16x4_f32 kernel),
        # "bf16x3" (three bf16 MFMAs per product, ~2^-16 relative), "bf16" (BASELINE cfg 3:
        # bf16-resident GEMM / attention operands, fp32 accumulation, residual stream, LN,
        # softmax, loss and master weights) or "fp8" (cfg 5: "bf16" + fp8-e4m3 region
        # features on block-scaled fp8 MFMA; forward(..., vis_fea_scale=) for fp8 inputs)
        object.__setattr__(self, "_engine", ModelEngine(self._arena, num_blocks, hidden_size,
                                                        num_heads, gemm_precision))

    def attach_reducer(self, reducer, batch_size: Optional[int] = None):
        """Stream the data-parallel gradient all-reduce out of the backward (ddp.GradReducer).
        The two stacks' syb_emb tables only get question-token rows (AttModel_x3.py:96-99,
        :216-219), so they are exchanged by rows (ddp.GradReducer.add_sparse_table).
        batch_size (the per-rank batch every rank is configured with): the row lists are then
        padded to the static bound batch_size * maxlen_q, so no rank waits for the others'
        counts in the forward (without it the counts are agreed on the host each step)."""
        object.__setattr__(self, "_reducer", reducer)
        object.__setattr__(self, "_rows_cap", None if batch_size is None
                           else int(batch_size) * int(self.maxlen_q))
        active = reducer is not None and getattr(reducer, "active", getattr(reducer, "world", 1) > 1)
        self._engine.multi_rank = active
        if active:
            for pre in ("att_vis_grid", "att_syb"):
                o, shp = self._arena.offsets[f"{pre}.syb_emb.weight"]
                reducer.add_sparse_table(o, o + shp.numel(), shp[1])

    # parameters live in the arena: moving the module moves the arena
    def _apply(self, fn, recurse=True):
        arena = self.__dict__.get("_arena")
        if arena is None:
            return super()._apply(fn, recurse)
        arena.apply(fn)
        self._engine.rebind()
        return self

    def forward(self, vis_fea, vis_mask, q_ipt, q_mask, q_graph,
                macro_ipt, macro_mask, macro_graph, macro_obj_loc,
                micro_positive_obj, micro_negative_obj, micro_obj_mask,
                micro_positive_rel, micro_negative_rel, micro_positive_rel_loc,
                micro_negative_rel_loc, decMask=True, mcb=False, vis_fea_scale=None):
        """AttModel_x3.py:512-542. vis_fea may be float8_e4m3fn (fp8 mode, BASELINE cfg 5) with
        its e8m0 block scales vis_fea_scale [B, Nv, 2048/32] (savqa_quant_fp8's layout)."""
        if mcb:
            raise NotImplementedError("mcb=True needs torch.rfft (removed in torch>=1.8); out of scope")
        drop = None
        if self.training and self.dropout_rate > 0:
            # one 63-bit step seed per forward from torch's CPU generator (torch.manual_seed
            # makes it reproducible); the backward regenerates the same masks from it
            seed = int(torch.randint(0, 2 ** 63 - 1, (1,), dtype=torch.int64).item())
            drop = (seed, float(self.dropout_rate))
        object.__setattr__(self, "_last_dropout", drop)
        dev = self._arena.flat.device
        if dev.type != "cuda":
            raise RuntimeError("savqa AttModel runs on a HIP device: call model.cuda() first")

        def f32(t):
            return t.to(device=dev, dtype=torch.float32).contiguous()

        def i32(t):
            return t.to(device=dev, dtype=torch.int32).contiguous()

        def i64(t):
            return t.to(device=dev, dtype=torch.int64).contiguous()

        fp8_in = vis_fea.dtype == torch.float8_e4m3fn
        if fp8_in and self._engine.gemm_precision != "fp8":
            raise ValueError("fp8 region features need AttModel(..., gemm_precision='fp8')")
        vis_t = vis_fea.to(device=dev).contiguous() if fp8_in else f32(vis_fea)
        object.__setattr__(self, "_vis_scale", vis_fea_scale.to(device=dev).contiguous()
                           if (fp8_in and vis_fea_scale is not None) else None)
        tensors = (vis_t, i32(vis_mask), i64(q_ipt), i32(q_mask), i32(q_graph), i64(macro_ipt),
                   i32(macro_mask), i32(macro_graph), i64(macro_obj_loc), i64(micro_positive_obj),
                   i64(micro_negative_obj), i32(micro_obj_mask))
        # a check left over from a forward that raised must never answer for this one
        self._engine.pending_rel_check = None
        if not self.only_obj:  # relation branch inputs (micro_negative_rel ids are unused, :391)
            tensors = tensors + (i64(micro_positive_rel), i64(micro_positive_rel_loc),
                                 i64(micro_negative_rel_loc))
            # the bounds check runs on a side stream; the engine waits for its verdict only
            # before launching the first kernel that reads these tables
            self._engine.pending_rel_check = self._check_relation_locs(
                tensors[-2], tensors[-1], vis_fea.shape[1], macro_ipt.shape[1],
                tensors[-3].shape[1])
        live = self._live_params()
        red = self.__dict__.get("_reducer")
        if red is not None and live:
            red.set_rows(tensors[2], cap=self.__dict__.get("_rows_cap"))  # q_ipt: touched rows
        lc, lv, ls, mil, mil_rel = _AttModelFn.apply(self, bool(decMask), drop, len(tensors),
                                                     *tensors, *live)
        return lc, lv, ls, mil, (mil_rel if not self.only_obj else 0)

    def _check_relation_locs(self, pos, neg, n_obj, n_macro, n_rel):
        """The reference indexes rels_bilinear / new_macro_ipt with these columns
        (AttModel_x3.py:401-437) and fails with IndexError on a bad one; the kernels would
        read outside their buffers instead, so the listed rows are bounds-checked: one device
        reduction on a side stream (after the producers of the tables on the caller's stream)
        into pinned host memory. Returns the wait: it raises IndexError for a bad table and
        synchronises with that reduction only -- a host read of the flag right here stalled the
        host until the GPU had drained the previous step, ~1.6 ms of the relation workload's
        step of launches the GPU then waited for. Shape errors raise at once."""
        nrel = self.MIL_NCE.num_relations
        dev = pos.device
        cur = torch.cuda.current_stream(dev)
        st = self.__dict__.get("_rel_check_stream")
        if st is None or st.device != dev:
            st = torch.cuda.Stream(device=dev)
            object.__setattr__(self, "_rel_check_stream", st)
            object.__setattr__(self, "_rel_check_host", torch.zeros(1, dtype=torch.bool,
                                                                  pin_memory=True))
        flag = self._rel_check_host
        bad = []
        for loc, w in ((pos, 5), (neg, 4)):
            if loc.numel() == 0:
                continue
            if loc.dim() != 3 or loc.shape[2] < w:
                raise IndexError(f"relation locations need shape (B, L, >={w}), got {tuple(loc.shape)}")
            bad.append((loc, w))
        if not bad:
            return lambda: None
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            flags = []
            for loc, w in bad:
                loc.record_stream(st)
                v = loc[..., 3] >= 0
                b = (loc[..., 0] < 0) | (loc[..., 0] >= n_obj) | (loc[..., 1] < 0) | \
                    (loc[..., 1] >= n_obj) | (loc[..., 2] < 0) | (loc[..., 2] >= nrel) | \
                    (loc[..., 3] >= n_macro)
                if w == 5:
                    b = b | (loc[..., 4] < 0) | (loc[..., 4] >= n_rel)
                flags.append((v & b).any())
            flag.copy_(torch.stack(flags).any().reshape(1), non_blocking=True)
            done = torch.cuda.Event()
            done.record(st)

        def wait():
            done.synchronize()
            if bool(flag[0]):
                raise IndexError("relation location out of range (objects / categories "
                                 f"< {nrel} / macro nodes / positive words)")
        return wait

    def _live_params(self):
        """The live Parameters (those the backward writes gradients for) when a graph is being
        recorded, else () -- they link the autograd node to their AccumulateGrad nodes."""
        if not torch.is_grad_enabled():
            return ()
        a = self._arena
        live = [a.params[n] for n in a.live_names]
        return tuple(p for p in live if p.requires_grad)
