"""ReLU branch masks of one HIP forward (fp32 mode), keyed as the oracle's Linear calls
(oracle.savqa_oracle.relu_branches): the unit of every ReLU site is on when the HIP path's saved
post-ReLU value is > 0. Running the oracle in fp64 under these masks gives the exact gradient of
the same piecewise-linear branch the HIP forward took, so HIP-vs-fp64 differences are rounding
alone: units whose pre-activation sits within fp32 rounding of 0 (and flip between any two fp32
summation orders) no longer decide the comparison.

Sites the HIP path does not compute have no mask (the oracle's own ReLU runs there): the
decoder self-attention's Q / K (one key: softmax == 1, exactly zero gradient) and the detached
macro projection (AttModel_x3.py:354). In encoder layers 0-1 the node rows' Q / V are not
computed either (their attention weights are exactly 0: engine.PRUNE_L01); their mask is 0."""
import re

import torch

_PRUNED = re.compile(r"enc_self_attention_[01]\.(Q|V)_proj")


def capture(model):
    """Wrap model._engine.forward so the next forward's saved state is kept: returns a list that
    receives (ms, sv, ss, hs)."""
    eng = model._engine
    box = []
    orig = eng.forward

    def fwd(*a, **k):
        out = orig(*a, **k)
        box.append(out[1])
        eng.forward = orig
        return out
    eng.forward = fwd
    return box


def hip_masks(saved, d=512, nb=6):
    """{(site, call): bool mask shaped like the oracle's pre-activation} from (ms, sv, ss, hs)."""
    ms, sv, ss, hs = saved
    m = {}
    for pre, s in (("att_vis_grid", sv), ("att_syb", ss)):
        B, T, Nn, Lq = s.B, s.T, s.Nn, s.Lq
        cat = s.cat.view(B, T, -1)
        m[(f"{pre}.syb_mlp.0", 0)] = cat[:, Nn:] > 0
        for i, e in enumerate(s.enc):
            a = f"{pre}.enc_self_attention_{i}"
            if e.get("qkv") is not None:
                q, k, v = e["qkv"][:, :d], e["qkv"][:, d:2 * d], e["qkv"][:, 2 * d:]
            else:
                q, k, v = e["qv"][:, :d], e["kb"], e["qv"][:, d:]
            for name, t in (("Q", q), ("K", k), ("V", v)):
                m[(f"{a}.{name}_proj.0", 0)] = (t > 0).reshape(B, T, d)
            m[(f"{pre}.enc_feed_forward_{i}.conv1.0", 0)] = (e["h"] > 0).reshape(B, T, -1)
        for i, e in enumerate(s.dec):
            m[(f"{pre}.dec_self_attention_{i}.V_proj.0", 0)] = (e["v"] > 0).reshape(B, 1, d)
            c = f"{pre}.dec_vanilla_attention_{i}"
            m[(f"{c}.Q_proj.0", 0)] = (e["qc"] > 0).reshape(B, 1, d)
            m[(f"{c}.K_proj.0", 0)] = (s.kv[:, 2 * i * d:(2 * i + 1) * d] > 0).reshape(B, T, d)
            m[(f"{c}.V_proj.0", 0)] = (s.kv[:, (2 * i + 1) * d:(2 * i + 2) * d] > 0).reshape(B, T, d)
            m[(f"{pre}.dec_feed_forward_{i}.conv1.0", 0)] = (e["h"] > 0).reshape(B, 1, -1)
    B, Nv, K = ms.B, ms.Nv, ms.K
    m[("MIL_NCE.syb_mlp.0", 0)] = (ms.Pf > 0).reshape(B, Nv, K, -1)
    m[("MIL_NCE.syb_mlp.0", 1)] = (ms.Nf > 0).reshape(B, Nv, K, -1)
    m[("MIL_NCE.vis_mlp.0", 0)] = (ms.vv > 0).reshape(B, Nv, -1)
    m[("MIL_NCE.ipt_mlp.0", 0)] = ss.cat.view(ss.B, ss.T, -1)[:, :ss.Nn] > 0
    for name in ("cls", "cls_vis", "cls_syb"):
        m[(f"{name}.0", 0)] = hs[name] > 0
    return {k: v.detach().clone() for k, v in m.items()}


def oracle_grads(O, params, batch, masks, dtype, device, names, decMask=True, **kw):
    """The oracle's gradients of `names` (and its outputs) in `dtype` on `device` under the ReLU
    branch masks (None: its own ReLUs); kw: attmodel_forward's num_blocks / h."""
    P = {n: p.detach().to(device=device, dtype=dtype).clone().requires_grad_(n in names)
         for n, p in params.items()}
    inp = {k: (v.to(device=device, dtype=dtype) if v.is_floating_point() else v.to(device))
           for k, v in batch.items()}
    # ({"_record": True}: the run records its own decisions into that dict)
    mk = masks if masks is None or masks.get("_record") else {k: v.to(device)
                                                              for k, v in masks.items()}
    old = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        with torch.device(device), O.relu_branches(mk) if mk is not None else _null():
            rc, rv, rs, rmil, _ = O.attmodel_forward(P, inp, decMask=decMask, **kw)
            rloss, _ = O.train_loss(rc, rv, rs, inp["answer"], rmil)
            rloss.backward()
    finally:
        torch.set_default_dtype(old)
    return {n: P[n].grad.detach() for n in names}, (rc.detach(), rv.detach(), rs.detach(),
                                                   rmil.detach(), rloss.detach())


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def mask_disagreement(O, params, batch, hip, names, tol=1e-4, **kw):
    """The HIP forward's ReLU decisions against the fp64 oracle's OWN (an unaligned fp64 run
    that records its pre-activations): per site, the units where they differ must sit within
    tol x the site's largest |pre-activation| of 0 (rounding can flip those, a wrong gate flips
    units anywhere) and be rare. Returns {site: (flips, units, worst |pre| / max |pre|)}."""
    rec = {"_record": True, "_pre": {}}
    oracle_grads(O, params, batch, rec, torch.float64, "cuda", names, **kw)
    pre = rec["_pre"]
    out = {}
    for key, m in hip.items():
        y = pre.get(key)
        if y is None or _PRUNED.search(key[0]):  # node rows of layers 0-1: masks are "don't
            continue                             # care" zeros there (module docstring)
        y = y.reshape(m.shape).to(m.device)
        flip = m != (y > 0)
        n = int(flip.sum())
        scale = float(y.abs().max())
        worst = float(y[flip].abs().max()) / max(scale, 1e-300) if n else 0.0
        out[key] = (n, m.numel(), worst)
    bad = {k: v for k, v in out.items() if v[2] > tol or v[0] > max(8, v[1] // 1000)}
    assert not bad, bad
    assert out, "no site compared"
    return out
