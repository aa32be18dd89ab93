"""The C ABI's ownership contract (include/savqa.h: caller-owned memory, no allocation, no
host synchronisation, async on the caller's stream) makes a whole training step capturable:
forward (both stacks on their side streams), loss, backward and Adam are captured into one
hipGraph (torch.cuda.graph) and replayed. A replay from a saved state must reproduce the
eager step (same kernels in the same order; split-K dW atomics may add in another order,
hence 1e-5), and a second replay from the same state must reproduce the first."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_training_step_captured_into_a_hip_graph(prec):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    from savqa_amd.utils import init_params_
    m = AttModel(None, 256, 128, 40, 16, 80, 40, 2, 4, 0.0, 0.0, 2, True, device="cuda",
                 init=False, gemm_precision=prec)
    init_params_(m, seed=5)
    m.train()
    batch = synthetic_batch(16, Nv=36, Lq=14, Ns=40, topN=5, num_classes=40, seed=9,
                            device="cuda")
    args = model_args(batch)
    opt = Adam(m, lr=1e-3)
    a = m._arena
    out = {}

    def step():
        lc, lv, ls, mil, _ = m(*args, decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
        opt.zero_grad()
        loss.backward()
        opt.step()
        out["loss"] = loss

    # warm-up on a side stream (lazy allocations: gradient arena, Adam moments, streams,
    # low-precision weight shadow), as torch.cuda.graph requires
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()

    def save():
        return (a.flat.clone(), opt.m.clone(), opt.v.clone(), opt.step_count)

    def load(st):
        a.flat.copy_(st[0])
        opt.m.copy_(st[1])
        opt.v.copy_(st[2])
        opt.step_count = st[3]
        a.generation += 1

    st = save()
    eager = []
    for _ in range(2):   # the eager step twice from the same state (determinism check)
        load(st)
        torch.cuda.synchronize()
        step()
        torch.cuda.synchronize()
        eager.append((a.flat[:a.n_live].clone(), a.grad.clone(), float(out["loss"])))
    eager_p, eager_g, eager_loss = eager[0]

    load(st)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    static_loss = out["loss"]
    rep = []
    for _ in range(2):
        load(st)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        rep.append((a.flat[:a.n_live].clone(), a.grad.clone(), float(static_loss)))

    def rel(x, y):
        return float((x - y).abs().max() / y.abs().max())

    def worst(x, y):
        out = []
        for n in a.live_names:
            o, shp = a.offsets[n]
            yy = y[o:o + shp.numel()]
            e = float((x[o:o + shp.numel()] - yy).abs().max() / yy.abs().max().clamp_min(1e-30))
            out.append((e, n))
        return sorted(out, reverse=True)[:12]

    diag = {"eager_p": rel(eager[1][0], eager_p), "eager_g": rel(eager[1][1], eager_g),
            "rep_p": rel(rep[1][0], rep[0][0]), "rep_g": rel(rep[1][1], rep[0][1]),
            "rep_vs_eager_p": rel(rep[0][0], eager_p), "rep_vs_eager_g": rel(rep[0][1], eager_g),
            "worst_g": worst(rep[0][1], eager_g), "worst_eager_g": worst(eager[1][1], eager_g)}
    print("graph-capture diagnostics:", diag)
    for p, gr, loss in rep:
        assert abs(loss - eager_loss) <= 1e-5 * abs(eager_loss), (loss, eager_loss)
        assert rel(gr, eager_g) <= 1e-5, diag
        assert rel(p, eager_p) <= 1e-5, diag
        assert not torch.equal(p, st[0][:a.n_live])   # the replay did update the parameters
    assert diag["rep_p"] <= 1e-5, diag
