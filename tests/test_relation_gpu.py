"""MIL-NCE relation branch (only_obj=False, AttModel_x3.py:382-437) on the HIP path against
the reference's own outputs on super-node batches (tests/golden/full_rel_{b2,sn}.npz, produced
by tools/make_golden.py running the reference): logits, mil_nce_obj, mil_nce_rel, loss and
the gradients of every trained parameter, MIL_NCE.R included (north-star tolerance 1e-3).
full_rel_sn has T_syb = 211 > 128, so the semantic stack runs the key-tiled attention
(csrc/attn_flash.hip) inside the parity case. full_rel_big is the reference's relation
configuration at the benched super-node size: hidden_size_mil 64 (submit.py:101), maxlen 1600
(:87), 311 relation categories, T_syb = 1313 (36 objects: 1260 relation nodes), ~5.7k listed
positive relations in the first sample."""
import os

import numpy as np
import pytest
import torch

from oracle import hashfill

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
INPUTS = ("vis_fea", "vis_mask", "q_ipt", "q_mask", "q_graph", "macro_ipt", "macro_mask",
          "macro_graph", "macro_obj_loc", "micro_positive_obj", "micro_negative_obj",
          "micro_obj_mask", "micro_positive_rel", "micro_negative_rel", "micro_positive_rel_loc",
          "micro_negative_rel_loc")


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("case", ["full_rel_b2", "full_rel_sn", "full_rel_big"])
def test_relation_branch_against_reference_golden(case):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.backends.cuda.matmul.allow_tf32 = False
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    g = np.load(os.path.join(GOLD, f"{case}.npz"))
    hm = int(g["hidden_mil"]) if "hidden_mil" in g else 1024
    maxlen = int(g["maxlen"]) if "maxlen" in g else 450
    m = AttModel(None, 512, hm, 914, 40, maxlen, 49, int(g["num_blocks"]), 8, 0.0, 0.0,
                 int(g["num_relations"]), False, device="cuda", init=False)
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.copy_(torch.from_numpy(hashfill.param_value(n, tuple(p.shape))))
    m.train()
    assert "MIL_NCE.R" in m._arena.live_names
    t = {k: torch.from_numpy(g[k]).cuda() for k in INPUTS + ("answer",)}
    lc, lv, ls, mil, mil_rel = m(*[t[k] for k in INPUTS], decMask=True, mcb=False)
    for name, out in (("logits_concat", lc), ("logits_vis", lv), ("logits_syb", ls)):
        o = out.detach().cpu().numpy()
        assert rel(o, g[name]) < 1e-3, name
        assert (o.argmax(-1) == g[name].argmax(-1)).all(), name
    assert abs(float(mil) - float(g["mil_nce_obj"])) < 1e-3 * max(1.0, abs(float(g["mil_nce_obj"])))
    assert abs(float(mil_rel) - float(g["mil_nce_rel"])) < 1e-3 * max(1.0, abs(float(g["mil_nce_rel"])))
    loss, _ = smoothed_loss(lc, lv, ls, t["answer"], mil, mil_nce_rel=mil_rel)
    assert abs(float(loss) - float(g["loss"])) < 1e-4 * abs(float(g["loss"]))
    opt = Adam(m, lr=1e-4)
    opt.zero_grad()
    loss.backward()
    params = dict(m.named_parameters())
    worst = []
    for n in [str(x) for x in g["grad_names"]]:
        gr = params[n].grad
        assert gr is not None, n
        flat = gr.reshape(-1).cpu().double().numpy()
        ref = g[f"g:{n}:val"].astype(np.float64)
        idx = g[f"g:{n}:idx"]
        scale = max(np.abs(ref).max(), float(g[f"g:{n}:abssum"]) / flat.size, 1e-20)
        worst.append((np.abs(flat[idx] - ref).max() / scale, n))
        asum = float(g[f"g:{n}:abssum"])
        assert abs(flat.sum() - float(g[f"g:{n}:sum"])) <= 1e-3 * max(asum, 1e-12) + 1e-9, n
    worst.sort(reverse=True)
    print(case, "per-gradient worst-element error, top 8 / 1st percentile / median:", worst[:8],
          worst[len(worst) // 100], worst[len(worst) // 2])
    # north-star bar for every case: at T_syb = 1313 (full_rel_big) the worst gradient element
    # lands 2.2e-4 from the reference (round 4: x6 GEMMs, base-2 softmax; 2.1e-3 in round 3,
    # when this case had a 1e-2 bar), the reference's own fp32 lands <= 2.8e-5 from the fp64
    # oracle (tests/golden/full_rel_big_fp64dev.json, tools/rel_fp64_check.py)
    assert worst[0][0] < 1e-3, worst[:5]
    assert worst[len(worst) // 2][0] < 1e-4, worst[len(worst) // 2]
    used = torch.from_numpy(g["R_used"]).cuda()
    assert rel(params["MIL_NCE.R"].grad[used, :4].cpu().numpy(), g["R_grad_used"]) < 1e-3
    opt.step()
    torch.cuda.synchronize()


@pytest.mark.parametrize("col,value", [(2, 4), (0, 99), (3, 10 ** 6), (4, 10 ** 6)])
def test_relation_locations_out_of_range_raise(col, value):
    """A relation row the reference would fail to index (IndexError) raises before any
    kernel reads outside its buffers."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.data import model_args_rel, synthetic_relation_batch
    from savqa_amd.utils import init_params_
    m = AttModel(None, 256, 64, 12, 16, 80, 10, 2, 4, 0.0, 0.0, 4, False, device="cuda",
                 init=False)
    init_params_(m, seed=2)
    b = synthetic_relation_batch(2, Nv=4, Lq=5, topN=2, num_relations=4, num_classes=12,
                                 seed=3, device="cuda")
    m(*model_args_rel(b), decMask=True, mcb=False)  # in range: runs
    keep = int(b["micro_positive_rel_loc"][1, 3, col])
    b["micro_positive_rel_loc"][1, 3, col] = value
    with pytest.raises(IndexError):
        m(*model_args_rel(b), decMask=True, mcb=False)
    # the check is per forward (asynchronous, AttModel._check_relation_locs): a valid batch
    # after the failed one runs
    b["micro_positive_rel_loc"][1, 3, col] = keep
    lc, *_ = m(*model_args_rel(b), decMask=True, mcb=False)
    assert bool(torch.isfinite(lc).all())
