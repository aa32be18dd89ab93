"""Key-tiled (flash) graph attention (csrc/attn_flash.hip) against an fp64 torch
restatement of modules.py:246-301 (forward output, dQ/dK/dV with the ReLU masks), at the
long sequence lengths the full-row kernels cannot take (cfg 4: T = 114 / 449 with d = 1024,
16 heads; super-node relation graphs: T = 1600), plus the parity traps: masked keys,
fully masked samples, rows with no neighbours, rows whose neighbours' softmax mass is
below F.normalize's 1e-12 clamp, zero query flags."""
import pytest
import torch

from tests.test_kernels_gpu import _attn_ref, g, rel

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.backends.cuda.matmul.allow_tf32 = False


def ops():
    from savqa_amd import ops as O
    return O


CASES = [(2, 73, 73, "self", 8, 512), (2, 449, 449, "self", 16, 1024), (3, 114, 114, "self", 16, 1024),
         (1, 1600, 1600, "self", 8, 512), (3, 1, 449, "cross", 16, 1024), (4, 1, 1600, "cross", 8, 512),
         (2, 200, 7, "cross", 8, 512), (2, 5, 300, "cross", 8, 512), (2, 17, 129, "cross", 4, 256)]


@pytest.mark.parametrize("B,Tq,Tk,kind,H,D", CASES)
def test_flash_attention_fwd_bwd(B, Tq, Tk, kind, H, D):
    O = ops()
    if kind == "self":
        qkv = g(B * Tk, 3 * D, seed=50, relu=True)
        Q, K, V = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
        ldq = ldk = ldv = 3 * D
    else:
        Q = g(B * Tq, D, seed=51, relu=True)
        kv = g(B * Tk, 2 * D, seed=52, relu=True)
        K, V = kv[:, :D], kv[:, D:]
        ldq, ldk, ldv = D, 2 * D, 2 * D
    G = (torch.rand(B, Tq, Tk, generator=torch.Generator().manual_seed(53)) < 0.3).float().to(dev)
    G[0, :min(3, Tq)] = 0.0                      # rows that attend to nothing
    kf = torch.ones(B, Tk, device=dev)
    kf[0, min(2, Tk - 1)] = 0.0
    kf[-1, -1] = 0.0
    qf = torch.ones(B, Tq, device=dev)
    qf[-1, 0] = 0.0
    if B >= 3:
        kf[1] = 0.0                              # a sample whose keys are all masked
    if Tq > 5 and Tk > 8:
        # clamped branch: query 5 of sample 0 only neighbours key 7, whose score sits
        # ~40 below the row max (key 3 amplified) -> sum|A*G| < 1e-12
        with torch.no_grad():
            K[3] = 2.3    # score(5, 3) = 64 * 2.3^2 / 8 ~ 42 per head
            Q[5] = 2.3
            K[7] = 0.0    # score(5, 7) = 0
        G[0, 5] = 0.0
        G[0, 5, 7] = 1.0
    out = torch.empty(B * Tq, D, device=dev)
    stats = torch.empty(B * H * Tq * 4, device=dev)
    O.gattn_fwd_flash(Q, ldq, K, ldk, V, ldv, G, kf, qf, B, Tq, Tk, H, out, D, stats)
    Qr = Q.reshape(B, Tq, D).double().cpu().requires_grad_(True)
    Kr = K.reshape(B, Tk, D).double().cpu().requires_grad_(True)
    Vr = V.reshape(B, Tk, D).double().cpu().requires_grad_(True)
    ref, _ = _attn_ref(Qr, Kr, Vr, G.double().cpu(), kf.double().cpu(), qf.double().cpu(), h=H)
    assert rel(out.view(B, Tq, D), ref) < 2e-5
    dO = g(B * Tq, D, seed=54)
    (ref * dO.view(B, Tq, D).double().cpu()).sum().backward()
    dq = torch.empty(B * Tq, D, device=dev)
    dk = torch.empty(B * Tk, D, device=dev)
    dv = torch.empty(B * Tk, D, device=dev)
    O.gattn_bwd_flash(Q, ldq, K, ldk, V, ldv, G, kf, qf, B, Tq, Tk, H, dO, D, stats,
                      dq, D, dk, D, dv, D)
    mq, mk, mv = (Qr > 0), (Kr > 0), (Vr > 0)
    assert rel(dq.view(B, Tq, D), Qr.grad * mq) < 5e-5
    assert rel(dk.view(B, Tk, D), Kr.grad * mk) < 5e-5
    assert rel(dv.view(B, Tk, D), Vr.grad * mv) < 5e-5


def test_flash_matches_full_row_kernels():
    """At T = 73 both paths exist: same outputs to fp32 rounding."""
    O = ops()
    B, T, H, D = 3, 73, 8, 512
    qkv = g(B * T, 3 * D, seed=60, relu=True)
    Q, K, V = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
    G = (torch.rand(B, T, T, generator=torch.Generator().manual_seed(61)) < 0.2).float().to(dev)
    kf = torch.ones(B, T, device=dev)
    qf = torch.ones(B, T, device=dev)
    o1 = torch.empty(B * T, D, device=dev)
    o2 = torch.empty(B * T, D, device=dev)
    stats = torch.empty(B * H * T * 4, device=dev)
    O.gattn_fwd(Q, 3 * D, K, 3 * D, V, 3 * D, G, kf, qf, B, T, T, H, o1, D)
    O.gattn_fwd_flash(Q, 3 * D, K, 3 * D, V, 3 * D, G, kf, qf, B, T, T, H, o2, D, stats)
    assert rel(o2, o1) < 1e-5
    dO = g(B * T, D, seed=62)
    d1 = torch.empty(B * T, 3 * D, device=dev)
    d2 = torch.empty(B * T, 3 * D, device=dev)
    O.gattn_bwd(Q, 3 * D, K, 3 * D, V, 3 * D, G, kf, qf, B, T, T, H, dO, D, d1, 3 * D,
                d1[:, D:], 3 * D, d1[:, 2 * D:], 3 * D)
    O.gattn_bwd_flash(Q, 3 * D, K, 3 * D, V, 3 * D, G, kf, qf, B, T, T, H, dO, D, stats,
                      d2, 3 * D, d2[:, D:], 3 * D, d2[:, 2 * D:], 3 * D)
    assert rel(d2, d1) < 1e-4


@pytest.mark.parametrize("B,Tq,Tk,H,D", [(2, 449, 449, 8, 512), (2, 17, 129, 4, 256),
                                         (1, 1314, 1314, 8, 512), (3, 200, 7, 8, 512)])
def test_flash_presplit_planes_bit_identical(B, Tq, Tk, H, D, monkeypatch):
    """savqa_gattn_{fwd,bwd}_flash_ws (Q / K / V / dO split once into bf16 plane tiles, DMA'd
    by the kernels) against the kernels splitting their own tiles (ws = NULL): the same splits
    meet the same MFMAs in the same order, so outputs, dQ / dK / dV and the stats are
    bit-identical -- ragged T (rows past T zero in the last tile), T_q != T_k, one tile."""
    O = ops()
    Q = g(B * Tq, D, seed=71, relu=True)
    kv = g(B * Tk, 2 * D, seed=72, relu=True)
    K, V = kv[:, :D], kv[:, D:]
    G = (torch.rand(B, Tq, Tk, generator=torch.Generator().manual_seed(73)) < 0.3).float().to(dev)
    kf = torch.ones(B, Tk, device=dev)
    kf[0, -1] = 0.0
    qf = torch.ones(B, Tq, device=dev)
    dO = g(B * Tq, D, seed=74)
    res = []
    for mode in ("0", "1"):
        monkeypatch.setattr(O, "FLASH_PLANES", mode)
        out = torch.empty(B * Tq, D, device=dev)
        st = torch.empty(B * H * Tq * 4, device=dev)
        O.gattn_fwd_flash(Q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, Tq, Tk, H, out, D, st)
        dq = torch.empty(B * Tq, D, device=dev)
        dkv = torch.empty(B * Tk, 2 * D, device=dev)
        O.gattn_bwd_flash(Q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, Tq, Tk, H, dO, D, st,
                          dq, D, dkv, 2 * D, dkv[:, D:], 2 * D)
        res.append((out, st, dq, dkv))
    for a, b in zip(*res):
        assert torch.equal(a, b)
