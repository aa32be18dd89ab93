"""Single-query graph attention split over keys (csrc/attn_q1s.hip: the decoder cross-attention
at T_k > 128, AttModel_x3.py:279 -> modules.py:246-301 with T_q = 1) against the fp64 torch
restatement of the core (forward output; dQ / dK / dV through the ReLU masks), at the relation
workload's T_k = 1314, cfg 4's 449 (d = 1024, 16 heads) and the short / ragged edges (one key,
a partial last split, exactly one split), with the parity traps: masked keys, a sample whose
keys are all masked (uniform softmax), a sample whose graph row is empty, F.normalize's clamped
branch (neighbour mass < 1e-12), a zero query flag, negative and non-unit graph weights. Also
bit-identical reruns (fixed-order split sums) and agreement with the key-tiled kernels."""
import pytest
import torch

from tests.test_kernels_gpu import _attn_ref, g, rel

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def ops():
    from savqa_amd import ops as O
    return O


def _case(B, Tk, H, D, seed):
    Q = g(B, D, seed=seed, relu=True)
    kv = g(B * Tk, 2 * D, seed=seed + 1, relu=True)
    K, V = kv[:, :D], kv[:, D:]
    G = (torch.rand(B, 1, Tk, generator=torch.Generator().manual_seed(seed + 2)) < 0.5).float()
    G[0, 0, : min(3, Tk)] = torch.tensor([2.0, -1.0, 0.5])[: min(3, Tk)]  # non-unit / negative
    G = G.to(dev)
    kf = torch.ones(B, Tk, device=dev)
    kf[0, min(5, Tk - 1)] = 0.0
    qf = torch.ones(B, device=dev)
    if B >= 2:
        qf[-1] = 0.0                     # zero query flag
    if B >= 3:
        kf[1] = 0.0                      # every key masked: uniform softmax
    if B >= 4:
        G[2] = 0.0                       # empty graph row: output 0, no gradient
    if B >= 5 and Tk > 8:
        # clamped branch: sample 3 neighbours only key 7, ~40 below the row max
        with torch.no_grad():
            Q[3] = 2.3
            K[3 * Tk + 4] = 2.3
            K[3 * Tk + 7] = 0.0
        G[3] = 0.0
        G[3, 0, 7] = 1.0
    return Q, K, V, kv, G, kf, qf


CASES = [(4, 1314, 8, 512), (5, 1314, 8, 512), (3, 449, 16, 1024), (5, 129, 4, 256),
         (2, 64, 8, 512), (2, 65, 8, 512), (3, 1, 8, 512), (6, 73, 8, 512)]


@pytest.mark.parametrize("B,Tk,H,D", CASES)
def test_q1s_fwd_bwd_against_fp64(B, Tk, H, D):
    O = ops()
    Q, K, V, kv, G, kf, qf = _case(B, Tk, H, D, 70 + Tk)
    out = torch.empty(B, D, device=dev)
    stats = torch.empty(B * H * 4, device=dev)
    O.gattn_fwd_q1s(Q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, Tk, H, out, D, stats)
    Qr = Q.reshape(B, 1, D).double().cpu().requires_grad_(True)
    Kr = K.reshape(B, Tk, D).double().cpu().requires_grad_(True)
    Vr = V.reshape(B, Tk, D).double().cpu().requires_grad_(True)
    ref, _ = _attn_ref(Qr, Kr, Vr, G.double().cpu(), kf.double().cpu(),
                       qf.double().cpu().view(B, 1), h=H)
    assert rel(out.view(B, 1, D), ref) < 2e-5
    dO = g(B, D, seed=77)
    (ref * dO.view(B, 1, D).double().cpu()).sum().backward()
    res = []
    for _ in range(2):
        dq = torch.empty(B, D, device=dev)
        dkv = torch.full((B * Tk, 2 * D), float("nan"), device=dev)
        O.gattn_bwd_q1s(Q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, Tk, H, dO, D, stats,
                        dq, D, dkv, 2 * D, dkv[:, D:], 2 * D)
        torch.cuda.synchronize()
        res.append((dq.clone(), dkv.clone()))
    (dq, dkv), (dq2, dkv2) = res
    assert torch.equal(dq, dq2) and torch.equal(dkv, dkv2)  # fixed-order split sums
    assert bool(torch.isfinite(dkv).all())                   # every key row written
    mq, mk, mv = (Qr > 0), (Kr > 0), (Vr > 0)
    assert rel(dq.view(B, 1, D), Qr.grad * mq) < 5e-5
    assert rel(dkv[:, :D].view(B, Tk, D), Kr.grad * mk) < 5e-5
    assert rel(dkv[:, D:].view(B, Tk, D), Vr.grad * mv) < 5e-5


def test_q1s_matches_key_tiled_kernels():
    """The relation workload's shape through both long-key paths: same outputs and gradients to
    fp32 rounding."""
    O = ops()
    B, Tk, H, D = 4, 1314, 8, 512
    Q, K, V, kv, G, kf, qf = _case(B, Tk, H, D, 90)
    o1, o2 = torch.empty(B, D, device=dev), torch.empty(B, D, device=dev)
    s1, s2 = torch.empty(B * H * 4, device=dev), torch.empty(B * H * 4, device=dev)
    O.gattn_fwd_q1s(Q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, Tk, H, o1, D, s1)
    O.gattn_fwd_flash(Q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, 1, Tk, H, o2, D, s2)
    assert rel(o1, o2) < 1e-5
    dO = g(B, D, seed=91)
    d1q, d2q = torch.empty(B, D, device=dev), torch.empty(B, D, device=dev)
    d1 = torch.empty(B * Tk, 2 * D, device=dev)
    d2 = torch.empty(B * Tk, 2 * D, device=dev)
    O.gattn_bwd_q1s(Q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, Tk, H, dO, D, s1, d1q, D, d1, 2 * D,
                    d1[:, D:], 2 * D)
    O.gattn_bwd_flash(Q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, 1, Tk, H, dO, D, s2, d2q, D, d2,
                      2 * D, d2[:, D:], 2 * D)
    assert rel(d1q, d2q) < 1e-4
    assert rel(d1, d2) < 1e-4
