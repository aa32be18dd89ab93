import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
exec(open(os.path.join(os.path.dirname(__file__), 'cpu_fp32_vs_fp64.py')).read().split("go(P, inp, torch.float32)")[0])
import torch.nn.functional as F
def run(PP, ii, dt):
    torch.set_default_dtype(dt)
    cap = {}
    orig_emb = F.embedding
    def emb(idx, table, *a, **k):
        out = orig_emb(idx, table, *a, **k)
        if table.shape[0] == 476 and out.requires_grad and idx.shape[1] == 449:
            out.retain_grad(); cap["pos"] = out
        return out
    orig = O.graph_mha
    def spy(P_, pre, queries, keys, values, graph, h=8, return_att=False):
        if pre == "att_syb.dec_vanilla_attention_0":
            keys.retain_grad(); cap["xenc"] = keys
        if pre == "att_syb.enc_self_attention_1":
            queries.retain_grad(); cap["x1"] = queries
        return orig(P_, pre, queries, keys, values, graph, h, return_att)
    O.F.embedding = emb; O.graph_mha = spy
    rc, rv, rs, rmil, _ = O.attmodel_forward(PP, ii, decMask=True, num_blocks=L, h=H)
    rl, _ = O.train_loss(rc, rv, rs, ii["answer"], rmil); rl.backward()
    O.F.embedding = orig_emb; O.graph_mha = orig
    torch.set_default_dtype(torch.float32)
    return {k: v.grad.double() for k, v in cap.items()}
a = run(P, inp, torch.float32)
b = run(P64, inp64, torch.float64)
for k in ("xenc", "x1", "pos"):
    e = (a[k] - b[k]).abs().amax(-1)  # (B, T)
    m = b[k].abs().amax()
    print(k, "max err/max", float(e.max() / m), "worst (b,t)", divmod(int(e.argmax()), e.shape[1]), "row331 err/max", [float(e[bb, 331] / m) for bb in range(B)])
