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
    batch = synthetic_batch(16, Nv=36, Lq=14, Ns=30, topN=5, num_classes=40, seed=9,
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
    step()
    torch.cuda.synchronize()
    eager_p, eager_loss = a.flat[:a.n_live].clone(), float(out["loss"])

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
        rep.append((a.flat[:a.n_live].clone(), float(static_loss)))
    for p, loss in rep:
        assert abs(loss - eager_loss) <= 1e-5 * abs(eager_loss), (loss, eager_loss)
        d = (p - eager_p).abs().max() / eager_p.abs().max()
        assert float(d) <= 1e-5, float(d)
        assert not torch.equal(p, st[0][:a.n_live])   # the replay did update the parameters
    assert float((rep[0][0] - rep[1][0]).abs().max() / rep[0][0].abs().max()) <= 1e-5
