"""Block-level API mirroring the reference's models/modules.py.

Same class names, constructor signatures, parameter names and forward semantics as
/root/reference/models/modules.py (embedding :13-46, layer_normalization :49-65,
multihead_attention :119-207, new_multihead_attention :210-311, feedforward
:405-447, label_smoothing :450-463), so state_dicts interchange. Forward/backward
run on libsavqa HIP kernels through autograd Functions; there is no torch-op
fallback (CPU tensors raise). Inside AttModel the stacks do not call these
forwards -- engine.py drives the same kernels over the flat arena with fused
projections -- but the modules own the parameters and the names.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
from torch.nn.parameter import Parameter

from . import ops
from .engine import _empty

__all__ = ["embedding", "layer_normalization", "multihead_attention", "new_multihead_attention",
           "feedforward", "label_smoothing"]


def _acc(p: Parameter) -> torch.Tensor:
    """p.grad, materialised as zeros if absent (kernels accumulate into it)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


def _rows(x: torch.Tensor, d: int) -> int:
    return x.numel() // d


# ------------------------------------------------------------------------------ embedding
class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, table, scale, padding_idx, mod):
        idx_c = idx.reshape(-1).contiguous()
        out = _empty(*idx.shape, table.shape[1], dev=table.device)
        ops.gather_rows(table, idx_c, idx_c.numel(), table.shape[1], scale, out)
        ctx.save_for_backward(idx_c)
        ctx.scale, ctx.pad, ctx.mod = scale, padding_idx, mod
        return out

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        p = ctx.mod.lookup_table
        pad = ctx.pad if ctx.pad >= 0 else p.shape[0] + ctx.pad
        ops.scatter_rows(g.contiguous(), idx, idx.numel(), p.shape[1], ctx.scale, pad, _acc(p))
        return None, None, None, None, None


class embedding(nn.Module):
    """modules.py:13-46."""

    def __init__(self, vocab_size, num_units, zeros_pad=True, scale=True):
        super().__init__()
        self.vocab_size = vocab_size
        self.num_units = num_units
        self.zeros_pad = zeros_pad
        self.scale = scale
        self.lookup_table = Parameter(torch.empty(vocab_size, num_units))
        nn.init.xavier_normal_(self.lookup_table.data)
        if self.zeros_pad:
            self.lookup_table.data[0, :].fill_(0)

    def forward(self, inputs):
        self.padding_idx = 0 if self.zeros_pad else -1
        scale = (self.num_units ** 0.5) if self.scale else 1.0
        return _EmbeddingFn.apply(inputs, self.lookup_table, scale, self.padding_idx, self)


# ------------------------------------------------------------------------------ LN
class _LNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps, mod):
        d = gamma.numel()
        xc = x.contiguous()
        y = torch.empty_like(xc)
        R = _rows(xc, d)
        st = (_empty(R, dev=x.device), _empty(R, dev=x.device), _empty(R, dev=x.device))
        ops.ln_fwd(xc, gamma, beta, y, *st, eps=eps)
        ctx.save_for_backward(xc, *st)
        ctx.mod = mod
        return y

    @staticmethod
    def backward(ctx, g):
        xc, m, r, s = ctx.saved_tensors
        mod = ctx.mod
        dz = torch.empty_like(xc)
        ops.ln_bwd(g.contiguous(), xc, m, r, s, mod.gamma, dz, _acc(mod.gamma), _acc(mod.beta))
        return dz, None, None, None, None


class layer_normalization(nn.Module):
    """modules.py:49-65 (unbiased std, eps added to std)."""

    def __init__(self, features, epsilon=1e-8):
        super().__init__()
        self.epsilon = epsilon
        self.gamma = nn.Parameter(torch.ones(features))
        self.beta = nn.Parameter(torch.zeros(features))

    def forward(self, x):
        return _LNFn.apply(x, self.gamma, self.beta, self.epsilon, self)


# ------------------------------------------------------------------------------ attention
def _proj(x2d, lin: nn.Linear, out):
    ops.linear(x2d, lin.weight, lin.bias, out, relu=True)


class _MHAFn(torch.autograd.Function):
    """Q/K/V projections + graph attention core + residual + LN (modules.py:236-311)."""

    @staticmethod
    def forward(ctx, queries, keys, values, graph, mod, want_att, *params):
        d, H = mod.num_units, mod.num_heads
        B, Tq, _ = queries.shape
        Tk = keys.shape[1]
        dev = queries.device
        q2, k2, v2 = (t.contiguous().reshape(-1, d) for t in (queries, keys, values))
        Q, K, V = _empty(B * Tq, d, dev=dev), _empty(B * Tk, d, dev=dev), _empty(B * Tk, d, dev=dev)
        _proj(q2, mod.Q_proj[0], Q)
        _proj(k2, mod.K_proj[0], K)
        _proj(v2, mod.V_proj[0], V)
        kf, qf = _empty(B * Tk, dev=dev), _empty(B * Tq, dev=dev)
        ops.rowflag(k2, B * Tk, d, d, kf)
        ops.rowflag(q2, B * Tq, d, d, qf)
        G = graph.to(torch.float32).contiguous()
        o = _empty(B * Tq, d, dev=dev)
        att = _empty(H * B, Tq, Tk, dev=dev) if want_att else None
        flash = ops.use_flash(Tq, Tk)
        if flash:
            if want_att:
                raise NotImplementedError("return_att=True needs T <= 128 (full-row kernels)")
            ast = _empty(B * H * Tq * 4, dev=dev)
            ops.gattn_fwd_flash(Q, d, K, d, V, d, G, kf, qf, B, Tq, Tk, H, o, d, ast)
        else:
            ast = o.new_empty(0)
            ops.gattn_fwd(Q, d, K, d, V, d, G, kf, qf, B, Tq, Tk, H, o, d, att)
        z, y = _empty(B * Tq, d, dev=dev), _empty(B * Tq, d, dev=dev)
        st = tuple(_empty(B * Tq, dev=dev) for _ in range(3))
        ln = mod.normalization
        ops.ln_fwd(o, ln.gamma, ln.beta, y, *st, r=q2, z_out=z, eps=ln.epsilon)
        ctx.save_for_backward(q2, k2, v2, Q, K, V, kf, qf, G, z, *st, ast)
        ctx.flash = flash
        ctx.mod, ctx.shape = mod, (B, Tq, Tk)
        ctx.same_kv = keys is values
        ctx.same_qk = queries is keys
        y = y.view(B, Tq, d)
        if want_att:
            ctx.mark_non_differentiable(att)
            return y, att
        return y

    @staticmethod
    def backward(ctx, gy, *rest):
        q2, k2, v2, Q, K, V, kf, qf, G, z, m, r, s, ast = ctx.saved_tensors
        mod = ctx.mod
        d, H = mod.num_units, mod.num_heads
        B, Tq, Tk = ctx.shape
        dev = gy.device
        ln = mod.normalization
        dz = _empty(B * Tq, d, dev=dev)
        ops.ln_bwd(gy.contiguous(), z, m, r, s, ln.gamma, dz, _acc(ln.gamma), _acc(ln.beta))
        dQ, dK, dV = _empty(B * Tq, d, dev=dev), _empty(B * Tk, d, dev=dev), _empty(B * Tk, d, dev=dev)
        if ctx.flash:
            ops.gattn_bwd_flash(Q, d, K, d, V, d, G, kf, qf, B, Tq, Tk, H, dz, d, ast, dQ, d,
                                dK, d, dV, d)
        else:
            ops.gattn_bwd(Q, d, K, d, V, d, G, kf, qf, B, Tq, Tk, H, dz, d, dQ, d, dK, d, dV, d)
        dq = _empty(B * Tq, d, dev=dev)
        dk = _empty(B * Tk, d, dev=dev)
        dv = _empty(B * Tk, d, dev=dev)
        for dP, x2, lin, dx, res in ((dQ, q2, mod.Q_proj[0], dq, dz), (dK, k2, mod.K_proj[0], dk, None),
                                     (dV, v2, mod.V_proj[0], dv, None)):
            ops.linear_dw(dP, x2, _acc(lin.weight), _acc(lin.bias), rows=x2.shape[0])
            ops.linear_dx(dP, lin.weight, dx, rows=x2.shape[0], resid=res)
        dq, dk, dv = dq.view(B, Tq, d), dk.view(B, Tk, d), dv.view(B, Tk, d)
        # autograd sums the grads of aliased inputs (queries is keys is values)
        return (dq, dk, dv, None, None, None) + (None,) * len(ctx.needs_input_grad[6:])


class new_multihead_attention(nn.Module):
    """modules.py:210-311 (graph-guided attention)."""

    def __init__(self, num_units, num_heads=8, dropout_rate=0, causality=False, return_att=False):
        super().__init__()
        self.num_units = num_units
        self.num_heads = num_heads
        self.dropout_rate = dropout_rate
        self.causality = causality
        self.return_att = return_att
        self.Q_proj = nn.Sequential(nn.Linear(num_units, num_units), nn.ReLU())
        self.K_proj = nn.Sequential(nn.Linear(num_units, num_units), nn.ReLU())
        self.V_proj = nn.Sequential(nn.Linear(num_units, num_units), nn.ReLU())
        self.output_dropout = nn.Dropout(p=dropout_rate)
        self.normalization = layer_normalization(num_units)

    def _check(self):
        if self.training and self.dropout_rate > 0:
            raise NotImplementedError("attention-probability dropout > 0 (the reference hard-codes 0)")

    def forward(self, queries, keys, values, graph):
        self._check()
        if self.causality:
            Tq, Tk = queries.shape[1], keys.shape[1]
            tril = torch.tril(torch.ones(Tq, Tk, device=queries.device))
            graph = graph * tril
        params = [p for p in self.parameters()]
        out = _MHAFn.apply(queries, keys, values, graph, self, self.return_att, *params)
        return out


class multihead_attention(new_multihead_attention):
    """modules.py:119-207: the same core with graph = causal tril (or all ones).

    Masking the future after the softmax and renormalising (what the graph path does)
    equals the reference's pre-softmax -2^32 fill up to fp32 rounding; the model
    only uses it with T_q = T_k = 1, where both are exactly 1."""

    def __init__(self, num_units, num_heads=8, dropout_rate=0, causality=False):
        super().__init__(num_units, num_heads, dropout_rate, causality, False)
        del self.return_att
        self.return_att = False

    def forward(self, queries, keys, values):
        self._check()
        B, Tq, Tk = queries.shape[0], queries.shape[1], keys.shape[1]
        g = torch.ones(B, Tq, Tk, device=queries.device)
        if self.causality:
            g = torch.tril(g)
        params = [p for p in self.parameters()]
        return _MHAFn.apply(queries, keys, values, g, self, False, *params)


# ------------------------------------------------------------------------------ FFN
class _FFNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, *params):
        d = mod.in_channels
        dh = mod.num_units[0]
        dev = x.device
        x2 = x.contiguous().reshape(-1, d)
        R = x2.shape[0]
        h = _empty(R, dh, dev=dev)
        ops.linear(x2, mod.conv1[0].weight, mod.conv1[0].bias, h, relu=True)
        z = _empty(R, mod.num_units[1], dev=dev)
        ops.linear(h, mod.conv2.weight, mod.conv2.bias, z, resid=x2)
        y = torch.empty_like(z)
        st = tuple(_empty(R, dev=dev) for _ in range(3))
        ln = mod.normalization
        ops.ln_fwd(z, ln.gamma, ln.beta, y, *st, eps=ln.epsilon)
        ctx.save_for_backward(x2, h, z, *st)
        ctx.mod = mod
        return y.view(x.shape[:-1] + (mod.num_units[1],))

    @staticmethod
    def backward(ctx, gy):
        x2, h, z, m, r, s = ctx.saved_tensors
        mod = ctx.mod
        ln = mod.normalization
        R = x2.shape[0]
        dz = torch.empty_like(z)
        ops.ln_bwd(gy.contiguous(), z, m, r, s, ln.gamma, dz, _acc(ln.gamma), _acc(ln.beta))
        ops.linear_dw(dz, h, _acc(mod.conv2.weight), _acc(mod.conv2.bias), rows=R)
        dh = torch.empty_like(h)
        ops.linear_dx(dz, mod.conv2.weight, dh, rows=R, mask=h, ldmask=h.shape[1])
        ops.linear_dw(dh, x2, _acc(mod.conv1[0].weight), _acc(mod.conv1[0].bias), rows=R)
        dx = torch.empty_like(x2)
        ops.linear_dx(dh, mod.conv1[0].weight, dx, rows=R, resid=dz)
        return (dx.view(gy.shape[:-1] + (x2.shape[1],)), None) + (None,) * (len(ctx.needs_input_grad) - 2)


class feedforward(nn.Module):
    """modules.py:405-447 (Linear path; the Conv1d path is disabled in the reference, :419)."""

    def __init__(self, in_channels, num_units=[2048, 512]):
        super().__init__()
        self.in_channels = in_channels
        self.num_units = num_units
        self.conv = False
        self.conv1 = nn.Sequential(nn.Linear(in_channels, num_units[0]), nn.ReLU())
        self.conv2 = nn.Linear(num_units[0], num_units[1])
        self.normalization = layer_normalization(in_channels)

    def forward(self, inputs):
        return _FFNFn.apply(inputs, self, *list(self.parameters()))


# ------------------------------------------------------------------------------ misc
class _AffineFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, a, b):
        xc = x.contiguous()
        out = torch.empty_like(xc)
        ops.affine(xc, xc.numel(), a, b, out)
        ctx.a = a
        return out

    @staticmethod
    def backward(ctx, g):
        gc = g.contiguous()
        out = torch.empty_like(gc)
        ops.affine(gc, gc.numel(), ctx.a, 0.0, out)
        return out, None, None


class label_smoothing(nn.Module):
    """modules.py:450-463."""

    def __init__(self, epsilon=0.1):
        super().__init__()
        self.epsilon = epsilon

    def forward(self, inputs):
        K = inputs.size()[-1]
        return _AffineFn.apply(inputs, 1 - self.epsilon, self.epsilon / K)
