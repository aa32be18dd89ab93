"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the SA-VQA model_v=3 hot path.

This module is the parity oracle (task rule: only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may use it; the product path never does).

It restates, in plain fp32 PyTorch-CPU tensor ops over a flat dict of the
reference's state_dict keys, the algorithm of
  /root/reference/models/modules.py      (layer_normalization, multihead_attention,
                                          new_multihead_attention, feedforward,
                                          label_smoothing)
  /root/reference/models/AttModel_x3.py  (AttModel_vis_grid, AttModel_syb, MIL_NCE
                                          only_obj branch, AttModel heads)
  /root/reference/models/main_itp_ddp_tar_super_node.py:335-366 (loss, Adam step),
                                          :42-142, :380-404 (eval metrics + gather)
Each function cites the reference lines it follows. Backward is torch autograd
over these ops.

Pinning: tests/test_oracle_golden.py checks this restatement against the golden
vectors in tests/golden/, which tools/make_golden.py produced by importing and
running the reference itself in the build container.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

PAD = 400000          # AttModel_x3.py:13
PAD_NEG = -2 ** 32 + 1  # modules.py:261 (becomes -4294967296.0 in fp32)


# --------------------------------------------------------------------------- dropout
# nn.Dropout sites of model_v=3 (p = dropout_rate in training): torch draws masks from its
# Philox stream, which no other implementation can reproduce, so parity with p > 0 uses
# the build's documented counter-hash stream (include/savqa.h, "Dropout") on both sides:
# everything except WHICH elements are dropped is then checked against this restatement.
VIS_SITES = (1, 2, 3)    # vis position-table dropout (:71-72), enc_dropout (:102), dec (:147)
SYB_SITES = (-1, 4, 5)   # syb: no position dropout (:178), enc_dropout (:227), dec (:274)
HEAD_SITES = {"cls": 6, "cls_vis": 7, "cls_syb": 8}   # heads (:482-500)

_K1, _K2 = np.uint64(0xD1B54A32D192ED03), np.uint64(0x9E3779B97F4A7C15)
_M1, _M2 = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)


def dropout_keep(seed: int, site: int, n: int, p: float) -> np.ndarray:
    """Keep mask (bool[n]) of elements 0..n-1 at dropout site `site` (SplitMix64 of
    counter seed + site*K1 + (idx+1)*K2, keep iff the high 32 bits >= floor(p*2^32))."""
    with np.errstate(over="ignore"):
        idx = np.arange(n, dtype=np.uint64)
        z = np.uint64(seed) + np.uint64(site) * _K1 + (idx + np.uint64(1)) * _K2
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    if p >= 1:
        return np.zeros(n, dtype=bool)
    thr = min(int(p * 4294967296.0), 0xFFFFFFFF) if p > 0 else 0
    return (z >> np.uint64(32)) >= np.uint64(thr)


def dropout(x, drop, site):
    """nn.Dropout(p)(x) with the counter-hash mask; drop = (seed, p) or None (identity)."""
    if drop is None or site < 0:
        return x
    seed, p = drop
    keep = torch.from_numpy(dropout_keep(seed, site, x.numel(), p)).reshape(x.shape)
    scale = 0.0 if p >= 1 else float(np.float32(1.0) / (np.float32(1.0) - np.float32(p)))
    return x * keep.to(x.dtype) * scale


# --------------------------------------------------------------------------- blocks
def layer_norm(x, gamma, beta, eps=1e-8):
    """modules.py:62-65 -- unbiased std, eps added to std."""
    mean = x.mean(-1, keepdim=True)
    std = x.std(-1, keepdim=True)
    return gamma * (x - mean) / (std + eps) + beta


# Test hook, branch-aligned references: {(site, call): bool mask} -- the ReLU of the call-th
# call of Linear `site` keeps exactly the units the mask marks (y * mask: the same piecewise-
# linear branch as the computation the masks came from), so an fp64 run follows the fp32
# path's ReLU decisions and the two differ by rounding alone, not by units within rounding of
# 0 that land on the other side (tests/branch_masks.py). Sites without a mask use F.relu.
RELU_BRANCHES = None
_relu_calls = {}


def linear(x, P, name, relu=False):
    y = F.linear(x, P[name + ".weight"], P[name + ".bias"])
    if not relu:
        return y
    if RELU_BRANCHES is not None:
        k = _relu_calls.get(name, 0)
        _relu_calls[name] = k + 1
        if RELU_BRANCHES.get("_record"):     # record this run's own decisions instead
            RELU_BRANCHES[(name, k)] = (y > 0).detach()
            if RELU_BRANCHES.get("_pre") is not None:  # and the pre-activations themselves
                RELU_BRANCHES["_pre"][(name, k)] = y.detach()
            return F.relu(y)
        m = RELU_BRANCHES.get((name, k))
        if m is not None:
            return y * m.reshape(y.shape).to(device=y.device, dtype=y.dtype)
    return F.relu(y)


class relu_branches:
    """Context manager: run the oracle with the given ReLU branch masks (RELU_BRANCHES)."""

    def __init__(self, masks):
        self.masks = masks

    def __enter__(self):
        global RELU_BRANCHES
        RELU_BRANCHES = self.masks
        _relu_calls.clear()
        return self

    def __exit__(self, *exc):
        global RELU_BRANCHES
        RELU_BRANCHES = None
        _relu_calls.clear()
        return False


def _heads(X, h):
    """torch.cat(torch.chunk(X, h, 2), 0): (N,T,C) -> (h*N, T, C/h), head-major."""
    return torch.cat(torch.chunk(X, h, dim=2), dim=0)


def _unheads(X, h):
    return torch.cat(torch.chunk(X, h, dim=0), dim=2)


def _mask_scores(S, keys, h, Tq):
    """modules.py:257-263 key masking by exact-zero feature sums."""
    km = torch.sign(torch.abs(torch.sum(keys, dim=-1)))          # (N, Tk)
    km = km.repeat(h, 1).unsqueeze(1).repeat(1, Tq, 1)           # (hN, Tq, Tk)
    cond = km.eq(0.).float()
    pad = torch.ones_like(S) * PAD_NEG
    return pad * cond + S * (1. - cond)


def _query_mask(queries, h, Tk):
    qm = torch.sign(torch.abs(torch.sum(queries, dim=-1)))       # (N, Tq)
    return qm.repeat(h, 1).unsqueeze(2).repeat(1, 1, Tk)


def graph_mha(P, pre, queries, keys, values, graph, h=8, return_att=False):
    """new_multihead_attention.forward, modules.py:236-311 (dropout p=0)."""
    Q = linear(queries, P, pre + ".Q_proj.0", relu=True)
    K = linear(keys, P, pre + ".K_proj.0", relu=True)
    V = linear(values, P, pre + ".V_proj.0", relu=True)
    Q_, K_, V_ = _heads(Q, h), _heads(K, h), _heads(V, h)
    S = torch.bmm(Q_, K_.permute(0, 2, 1)) / (K_.size(-1) ** 0.5)
    S = _mask_scores(S, keys, h, queries.size(1))
    A = F.softmax(S, dim=-1)
    A = graph.repeat(h, 1, 1) * A                                # :280-284
    A = F.normalize(A, p=1, dim=-1)                              # :285
    att = A.clone()
    A = A * _query_mask(queries, h, keys.size(1))                # :289-292
    O = _unheads(torch.bmm(A, V_), h)                            # :298-301
    O = O + queries                                              # :304
    out = layer_norm(O, P[pre + ".normalization.gamma"], P[pre + ".normalization.beta"])
    return (out, att) if return_att else out


def causal_mha(P, pre, queries, keys, values, h=8):
    """multihead_attention.forward with causality, modules.py:143-207."""
    Q = linear(queries, P, pre + ".Q_proj.0", relu=True)
    K = linear(keys, P, pre + ".K_proj.0", relu=True)
    V = linear(values, P, pre + ".V_proj.0", relu=True)
    Q_, K_, V_ = _heads(Q, h), _heads(K, h), _heads(V, h)
    S = torch.bmm(Q_, K_.permute(0, 2, 1)) / (K_.size(-1) ** 0.5)
    S = _mask_scores(S, keys, h, queries.size(1))
    tril = torch.tril(torch.ones(S.shape[1:], dtype=S.dtype))
    cond = tril.unsqueeze(0).repeat(S.size(0), 1, 1).eq(0.).float()
    S = torch.ones_like(S) * PAD_NEG * cond + S * (1. - cond)
    A = F.softmax(S, dim=-1)
    A = A * _query_mask(queries, h, keys.size(1))
    O = _unheads(torch.bmm(A, V_), h) + queries
    return layer_norm(O, P[pre + ".normalization.gamma"], P[pre + ".normalization.beta"])


def feedforward(P, pre, x):
    """feedforward.forward, Linear path, modules.py:432-447."""
    hdn = linear(x, P, pre + ".conv1.0", relu=True)
    out = linear(hdn, P, pre + ".conv2") + x
    return layer_norm(out, P[pre + ".normalization.gamma"], P[pre + ".normalization.beta"])


# --------------------------------------------------------------------------- graphs
def build_graphs(node_mask, q_mask, q_graph, node_graph=None, decMask=True):
    """Per-sample graph construction, AttModel_x3.py:103-122 (vis) / :229-247 (syb).

    Returns (graph_diag, graph, dec_mask). graph_cross is the same tensor as
    graph in the reference (alias at :118-120 / :244-245), so layers 2-5 all
    use `graph`.
    """
    B, Nn = node_mask.shape[:2]
    Lq = q_mask.shape[1]
    T = Nn + Lq
    mask = torch.zeros((B, T, T))
    graph_diag = torch.zeros((B, T, T))
    dec_mask = torch.zeros((B, 1, T))
    for i in range(B):
        mask[i] = torch.block_diag(node_mask[i], q_mask[i])
        graph_diag[i, -Lq:, -Lq:] = q_mask[i].float()
        if decMask:
            rs = torch.sum(mask[i], dim=1)
            rs[rs.nonzero()] = 1
            dec_mask[i, 0, :] = rs
    graph = 1 - mask
    if node_graph is None:
        graph[:, :Nn, :Nn] = 1
    else:
        graph[:, :Nn, :Nn] = node_graph.float()
    graph[:, Nn:, Nn:] = q_graph.float()
    return graph_diag, graph, dec_mask


# --------------------------------------------------------------------------- stacks
def _encoder_decoder(P, pre, fea, graph_diag, graph, dec_mask, num_blocks=6, h=8, drop=None,
                     dec_site=-1):
    """Encoder schedule AttModel_x3.py:127-139 and decoder :141-154."""
    x = fea
    for i in range(num_blocks):
        g = graph_diag if i < 2 else graph
        x = graph_mha(P, f"{pre}.enc_self_attention_{i}", x, x, x, g, h)
        x = feedforward(P, f"{pre}.enc_feed_forward_{i}", x)
    B = fea.size(0)
    d = fea.size(2)
    dec_in = torch.full((B, 1), 2, dtype=torch.long)
    dec = F.embedding(dec_in, P[f"{pre}.dec_emb.lookup_table"], 0) * (d ** 0.5)  # modules.py:40-43
    dec = dec + F.embedding(torch.zeros((B, 1), dtype=torch.long),
                            P[f"{pre}.dec_positional_encoding.lookup_table"], -1)
    dec = dropout(dec, drop, dec_site)                                       # dec_dropout
    for i in range(num_blocks):
        dec = causal_mha(P, f"{pre}.dec_self_attention_{i}", dec, dec, dec, h)
        dec = graph_mha(P, f"{pre}.dec_vanilla_attention_{i}", dec, x, x, dec_mask, h)
        dec = feedforward(P, f"{pre}.dec_feed_forward_{i}", dec)
    return dec


def vis_grid_forward(P, vis_fea, vis_mask, q_ipt, q_graph, q_mask, decMask=True,
                     num_blocks=6, h=8, pre="att_vis_grid", drop=None):
    """AttModel_vis_grid.forward, AttModel_x3.py:91-156."""
    q = F.embedding(q_ipt, P[f"{pre}.syb_emb.weight"])
    q = linear(q, P, f"{pre}.syb_mlp.0", relu=True)
    fea = linear(torch.cat([vis_fea, q], dim=1), P, f"{pre}.syb_mlp2")
    T = fea.size(1)
    pos = torch.arange(T).unsqueeze(0).repeat(fea.size(0), 1)
    pe = F.embedding(pos, P[f"{pre}.syb_positional_encoding.0.lookup_table"], -1)
    fea = fea + dropout(pe, drop, VIS_SITES[0])              # Sequential(embedding, Dropout)
    fea = dropout(fea, drop, VIS_SITES[1])                   # enc_dropout (:102)
    gd, g, dm = build_graphs(vis_mask, q_mask, q_graph, None, decMask)
    return _encoder_decoder(P, pre, fea, gd, g, dm, num_blocks, h, drop, VIS_SITES[2])


def syb_forward(P, syb_ipt, syb_mask, syb_graph, q_ipt, q_graph, q_mask, decMask=True,
                num_blocks=6, h=8, pre="att_syb", drop=None):
    """AttModel_syb.forward, AttModel_x3.py:214-282."""
    q = F.embedding(q_ipt, P[f"{pre}.syb_emb.weight"])
    q = linear(q, P, f"{pre}.syb_mlp.0", relu=True)
    fea = linear(torch.cat([syb_ipt, q], dim=1), P, f"{pre}.syb_mlp2")
    T = fea.size(1)
    pos = torch.arange(T).unsqueeze(0).repeat(fea.size(0), 1)
    fea = fea + F.embedding(pos, P[f"{pre}.syb_positional_encoding.lookup_table"], -1)
    fea = dropout(fea, drop, SYB_SITES[1])                   # enc_dropout (:227)
    gd, g, dm = build_graphs(syb_mask, q_mask, q_graph, syb_graph, decMask)
    return _encoder_decoder(P, pre, fea, gd, g, dm, num_blocks, h, drop, SYB_SITES[2])


def mil_nce_forward(P, vis_fea, macro_ipt, macro_obj_loc, pos_obj, neg_obj, obj_mask,
                    pre="MIL_NCE", eps=1e-6, rel=None):
    """MIL_NCE.forward, AttModel_x3.py:338-441: the only_obj branch (:338-380), plus the
    relation branch (:382-437) when rel = (pos_rel, neg_rel, pos_rel_loc, neg_rel_loc)."""
    E = P[f"{pre}.syb_emb.weight"]
    macro = linear(F.embedding(macro_ipt, E), P, f"{pre}.marco_mlp.0", relu=True).detach()
    Pf = linear(F.embedding(pos_obj, E), P, f"{pre}.syb_mlp.0", relu=True)   # (B,Nv,K,H)
    Nf = linear(F.embedding(neg_obj, E), P, f"{pre}.syb_mlp.0", relu=True)
    v = linear(vis_fea, P, f"{pre}.vis_mlp.0", relu=True).unsqueeze(3)       # (B,Nv,H,1)
    m4 = obj_mask.unsqueeze(3)
    sp = m4 * torch.matmul(Pf, v)                                             # (B,Nv,K,1)
    sn = m4 * torch.matmul(Nf, v)
    zeros = torch.zeros(sn.size())
    mil = torch.mean(torch.logsumexp(torch.cat((sp.clamp(min=eps), zeros.clamp(min=eps)), 1), 2)
                     - torch.logsumexp(torch.cat((sp.clamp(min=eps), sn.clamp(min=eps)), 1), 2))
    w = F.softmax(torch.matmul(Pf, v), dim=2)                                 # :372-374
    obj = torch.sum(w * Pf, dim=2)                                            # (B,Nv,H)
    valid = (macro_obj_loc >= 0).nonzero()                                    # :377-380
    macro[valid[:, 0], macro_obj_loc[valid[:, 0], valid[:, 1]].long(), :] = \
        obj[valid[:, 0], valid[:, 1], :].to(macro.dtype)  # (dtype cast: autocast runs)
    mil_rel = 0
    if rel is not None:
        macro, mil_rel = mil_nce_relations(P, macro, obj, *rel, pre=pre, eps=eps)
    out = linear(macro, P, f"{pre}.ipt_mlp.0", relu=True)
    return out, mil, mil_rel


def mil_nce_relations(P, macro, obj, pos_rel, neg_rel, pos_loc, neg_loc, pre="MIL_NCE", eps=1e-6):
    """Relation branch of MIL_NCE.forward, AttModel_x3.py:382-437.

    loc rows: [obj_i, obj_j, rel_category, macro_rel_loc, micro_rel_loc] (negatives have
    the first four); rows with macro_rel_loc < 0 are padding. bilinear(b, r, i, j) =
    obj[b,i]^T R[r] obj[b,j] (the einsum pair at :398-401, only at the listed entries).
    The softmax over ALL positives of the batch (:420) is indexed by the per-sample
    micro_rel_loc (:426-436), exactly as the reference does."""
    E = P[f"{pre}.syb_emb.weight"]
    R = P[f"{pre}.R"]
    relf = linear(F.embedding(pos_rel, E), P, f"{pre}.syb_mlp.0", relu=True)  # (B, maxrel, H)

    def bilinear(loc):
        v = (loc[:, :, 3] >= 0).nonzero()
        b, k = v[:, 0], v[:, 1]
        xi = obj[b, loc[b, k, 0]]
        xj = obj[b, loc[b, k, 1]]
        Rr = R[loc[b, k, 2]]
        return torch.einsum("pl,plk,pk->p", xi, Rr, xj), v

    sp, vpos = bilinear(pos_loc)
    sn, _ = bilinear(neg_loc)
    mil_rel = torch.logsumexp(sp.clamp(min=eps), dim=0) - torch.logsumexp(
        torch.cat((sp.clamp(min=eps), sn.clamp(min=eps)), dim=0), dim=0)
    b, k = vpos[:, 0], vpos[:, 1]
    macro = macro.clone()
    macro[b, pos_loc[b, k, 3]] = 0                                            # :418
    w = F.softmax(sp, dim=0)                                                  # :420
    for bb, kk in vpos.tolist():                                              # :421-436
        m4 = int(pos_loc[bb, kk, 4])
        r3 = int(pos_loc[bb, kk, 3])
        macro[bb, r3] = macro[bb, r3] + w[m4] * relf[bb, m4]
    return macro, mil_rel


def heads(P, fea_vis, fea_syb, drop=None):
    """AttModel.forward heads, AttModel_x3.py:531-541 (mcb=False)."""
    def head(x, name):
        hdn = dropout(linear(x, P, f"{name}.0", relu=True), drop, HEAD_SITES[name])
        return linear(hdn, P, f"{name}.3")
    logits_vis = head(fea_vis, "cls_vis").squeeze(1)
    logits_syb = head(fea_syb, "cls_syb").squeeze(1)
    fea = torch.cat((fea_syb.squeeze(1), fea_vis.squeeze(1)), 1)
    logits_concat = head(fea, "cls")
    return logits_concat, logits_vis, logits_syb


def attmodel_forward(P, inp: Dict[str, torch.Tensor], decMask=True, num_blocks=6, h=8,
                     drop=None, only_obj=True):
    """AttModel.forward, AttModel_x3.py:512-542 (only_obj, mcb=False); drop = (seed, p)
    applies the training-mode dropout sites with the counter-hash masks."""
    rel = None if only_obj else (inp["micro_positive_rel"], inp["micro_negative_rel"],
                                 inp["micro_positive_rel_loc"], inp["micro_negative_rel_loc"])
    new_macro, mil_obj, mil_rel = mil_nce_forward(
        P, inp["vis_fea"], inp["macro_ipt"], inp["macro_obj_loc"],
        inp["micro_positive_obj"], inp["micro_negative_obj"], inp["micro_obj_mask"], rel=rel)
    f_vis = vis_grid_forward(P, inp["vis_fea"], inp["vis_mask"], inp["q_ipt"], inp["q_graph"],
                             inp["q_mask"], decMask, num_blocks, h, drop=drop)
    f_syb = syb_forward(P, new_macro, inp["macro_mask"], inp["macro_graph"], inp["q_ipt"],
                        inp["q_graph"], inp["q_mask"], decMask, num_blocks, h, drop=drop)
    lc, lv, ls = heads(P, f_vis, f_syb, drop)
    return lc, lv, ls, mil_obj, mil_rel


# --------------------------------------------------------------------------- loss / optim
def train_loss(logits_concat, logits_vis, logits_syb, answer, mil_nce_obj,
               with_milnce=True, epsilon=0.1, mil_nce_rel=0):
    """main_itp_ddp_tar_super_node.py:326-361 with label_smoothing modules.py:461-463
    (mil_nce_loss = -mil_nce_obj - mil_nce_rel when the relation branch runs)."""
    lsm = (F.log_softmax(logits_vis, -1) + F.log_softmax(logits_syb, -1)
           + F.log_softmax(logits_concat, -1)) / 3
    oh = torch.zeros_like(logits_concat)
    oh.scatter_(1, answer.view(-1, 1), 1)
    oh = (1 - epsilon) * oh + epsilon / oh.size(-1)
    loss = (-(oh * lsm).sum(-1)).mean()
    if with_milnce:
        loss = loss + (-mil_nce_obj - mil_nce_rel)
    return loss, lsm


def eval_batch(logits_concat, logits_vis, logits_syb, answer, mil_nce_obj, mil_nce_rel=0,
               with_milnce=False, epsilon=0.1):
    """One batch of eval(), main_itp_ddp_tar_super_node.py:103-133: the label-smoothed loss
    (+ the MIL-NCE loss if --with_MILNCE_loss, :129-131), cnt_correct over NON-ZERO answers
    (:125-126, torch.max = first maximal index), cnt += batch_size (:127: every sample).
    Returns (loss, correct, batch_size, mil_nce_loss) as Python numbers."""
    loss, lsm = train_loss(logits_concat, logits_vis, logits_syb, answer, mil_nce_obj,
                           with_milnce=with_milnce, epsilon=epsilon, mil_nce_rel=mil_nce_rel)
    _, pred = torch.max(lsm, dim=1)
    nz = torch.nonzero(answer)
    correct = int((pred[nz] == answer[nz]).long().sum())
    mil_loss = -mil_nce_obj - mil_nce_rel
    return float(loss), correct, int(answer.shape[0]), float(mil_loss)


def eval_epoch(batch_stats):
    """eval()'s return value (main:42-142): (loss_meter.avg, cnt_correct, cnt) over the
    batches' eval_batch() results (AverageMeter weighted by batch size, misc.py:46-63)."""
    tot = sum(b for _, _, b, _ in batch_stats)
    avg = sum(l * b for l, _, b, _ in batch_stats) / tot if tot else 0.0
    return avg, sum(c for _, c, _, _ in batch_stats), tot


def gather_epoch_metrics(per_rank):
    """main:383-404: the 3-float (loss, cnt_correct, cnt) vectors of every rank are
    all-gathered; loss = mean over ranks, counts summed; accuracy = correct / cnt."""
    loss = sum(v[0] for v in per_rank) / len(per_rank)
    corr = sum(v[1] for v in per_rank)
    cnt = sum(v[2] for v in per_rank)
    return loss, corr, cnt, (corr / cnt if cnt else 0.0)


def adam_step(params, grads, state, step, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8):
    """torch.optim.Adam single-tensor update (main:206, :366), restated."""
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    for k, p in params.items():
        g = grads.get(k)
        if g is None:
            continue
        m, v = state.setdefault(k, (torch.zeros_like(p), torch.zeros_like(p)))
        m.mul_(beta1).add_(g, alpha=1 - beta1)
        v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(m, denom, value=-(lr / bc1))


# --------------------------------------------------------------------------- params
def model_param_shapes(hidden=512, hidden_mil=1024, num_classes=914, maxlen_q=40, maxlen=450,
                       maxlen_v=49, num_blocks=6, num_relations=311, vocab=407000, emb=300):
    """Reference state_dict keys and shapes in registration order (AttModel_x3.py:20-510)."""
    d = hidden
    out = []

    def lin(name, i, o):
        out.append((f"{name}.weight", (o, i)))
        out.append((f"{name}.bias", (o,)))

    def ln(name):
        out.append((f"{name}.gamma", (d,)))
        out.append((f"{name}.beta", (d,)))

    def mha(name):
        for p in ("Q_proj", "K_proj", "V_proj"):
            lin(f"{name}.{p}.0", d, d)
        ln(f"{name}.normalization")

    def ffn(name):
        lin(f"{name}.conv1.0", d, 4 * d)
        lin(f"{name}.conv2", 4 * d, d)
        ln(f"{name}.normalization")

    v = "att_vis_grid"
    out.append((f"{v}.syb_emb.weight", (vocab, emb)))
    lin(f"{v}.syb_mlp.0", emb, 2048)
    lin(f"{v}.syb_mlp2", 2048, d)
    lin(f"{v}.v_mlp.0", 2048, d)
    lin(f"{v}.v_mlp.2", d, d)
    out.append((f"{v}.v_positional_encoding.0.lookup_table", (maxlen_v, d)))
    lin(f"{v}.input_proj", 2048, d)
    for i in range(num_blocks):
        mha(f"{v}.enc_self_attention_{i}")
        ffn(f"{v}.enc_feed_forward_{i}")
    lin(f"{v}.q_mlp.0", emb, d)
    lin(f"{v}.q_mlp.2", d, d)
    out.append((f"{v}.q_positional_encoding.0.lookup_table", (maxlen_q, d)))
    out.append((f"{v}.syb_positional_encoding.0.lookup_table", (maxlen, d)))
    out.append((f"{v}.dec_emb.lookup_table", (num_classes, d)))
    out.append((f"{v}.dec_positional_encoding.lookup_table", (maxlen, d)))
    for i in range(num_blocks):
        mha(f"{v}.dec_self_attention_{i}")
        mha(f"{v}.dec_vanilla_attention_{i}")
        ffn(f"{v}.dec_feed_forward_{i}")

    s = "att_syb"
    out.append((f"{s}.syb_emb.weight", (vocab, emb)))
    lin(f"{s}.syb_mlp.0", emb, 2048)
    lin(f"{s}.syb_mlp2", 2048, d)
    out.append((f"{s}.syb_positional_encoding.lookup_table", (maxlen + maxlen_q, d)))
    lin(f"{s}.q_mlp.0", emb, d)
    lin(f"{s}.q_mlp.1", d, d)
    out.append((f"{s}.q_positional_encoding.0.lookup_table", (maxlen_q, d)))
    out.append((f"{s}.dec_emb.lookup_table", (num_classes, d)))
    out.append((f"{s}.dec_positional_encoding.lookup_table", (maxlen + maxlen_q, d)))
    for i in range(num_blocks):
        mha(f"{s}.dec_self_attention_{i}")
        mha(f"{s}.dec_vanilla_attention_{i}")
        ffn(f"{s}.dec_feed_forward_{i}")
    for i in range(num_blocks):
        mha(f"{s}.enc_self_attention_{i}")
        ffn(f"{s}.enc_feed_forward_{i}")

    m = "MIL_NCE"
    H = hidden_mil
    out.append((f"{m}.R", (num_relations, H, H)))
    out.append((f"{m}.syb_emb.weight", (vocab, emb)))
    lin(f"{m}.marco_mlp.0", emb, H)
    lin(f"{m}.syb_mlp.0", emb, H)
    lin(f"{m}.vis_mlp.0", 2048, H)
    lin(f"{m}.rel_mlp.0", H, H)
    lin(f"{m}.rel_mlp.2", H, 1)
    out.append((f"{m}.bilinear.weight", (num_relations, H, H)))
    lin(f"{m}.ipt_mlp.0", H, 2048)

    lin("cls.0", 2 * d, d)
    lin("cls.3", d, num_classes)
    lin("cls_vis.0", d, d)
    lin("cls_vis.3", d, num_classes)
    lin("cls_syb.0", d, d)
    lin("cls_syb.3", d, num_classes)
    out.append(("mcb.sketch1", (d, 16000)))
    out.append(("mcb.sketch2", (d, 16000)))
    lin("cls_mcb.0", 16000, d)
    lin("cls_mcb.3", d, num_classes)
    return out
