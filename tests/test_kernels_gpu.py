"""Kernel-level parity of libsavqa (HIP, gfx950) against plain PyTorch fp32 references
and the CPU oracle. Each test calls through the C ABI (savqa_amd.ops -> libsavqa.so)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.backends.cuda.matmul.allow_tf32 = False
    import savqa_amd._lib as L
    L.load()


def ops():
    from savqa_amd import ops as O
    return O


@pytest.fixture(params=["fp32_native", "fp32x6"])
def fp32k(request):
    """The two fp32 GEMM kernels of the 128x128-tile shapes: v_mfma_f32_16x16x4_f32
    (gemm.hip) and exact three-term bf16 splits on the bf16 matrix cores (gemm_x6.hip, the
    engine's default); the skinny kernels are the same under both."""
    with ops().gemm_precision(request.param):
        yield request.param


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def g(*shape, seed=0, relu=False):
    t = torch.randn(*shape, generator=torch.Generator().manual_seed(seed))
    if relu:
        t = t.clamp_min(0)
    return t.to(dev)


@pytest.mark.parametrize("M,N,K", [(77, 130, 300), (256, 512, 512), (1000, 1536, 512), (300, 2048, 64)])
def test_gemm_nt_epilogues(M, N, K, fp32k):
    O = ops()
    X, W, b = g(M, K, seed=1), g(N, K, seed=2), g(N, seed=3)
    pos = g(7, N, seed=4)
    res = g(M, N, seed=5)
    out = torch.empty(M, N, device=dev)
    O.linear(X, W, b, out, relu=True, rowvec=pos, rowvec_period=7, resid=res)
    ref = torch.relu(X @ W.t() + b + pos[torch.arange(M, device=dev) % 7]) + res
    assert rel(out, ref) < 2e-6


def test_gemm_gather_scatter_and_maps(fp32k):
    O = ops()
    table = g(1000, 300, seed=6)
    idx = torch.randint(0, 1000, (90,), generator=torch.Generator().manual_seed(7)).to(dev)
    W, b = g(64, 300, seed=8), g(64, seed=9)
    # gathered rows written into a (B=10, T=13) "cat" layout at rows [4, 13)
    out = torch.zeros(10 * 13, 64, device=dev)
    O.linear(table, W, b, out, relu=True, a_rows=idx, c_group=9, c_stride=13, c_offset=4)
    ref = torch.relu(table[idx] @ W.t() + b)
    got = out.view(10, 13, 64)[:, 4:].reshape(90, 64)
    assert rel(got, ref) < 2e-6
    assert float(out.view(10, 13, 64)[:, :4].abs().max()) == 0.0
    # scatter-add back (embedding grad): dtable[idx] += dY W
    dY = g(90, 64, seed=10)
    dtab = torch.zeros_like(table)
    O.linear_dx(dY, W, dtab, rows=90, c_rows=idx, atomic=True)
    ref = torch.zeros_like(table).index_add_(0, idx, dY @ W)
    assert rel(dtab, ref) < 2e-6


@pytest.mark.parametrize("M,N,K", [(77, 130, 300), (4000, 512, 1536)])
def test_gemm_dx_dw(M, N, K, fp32k):
    O = ops()
    dY, W, X = g(M, N, seed=11), g(N, K, seed=12), g(M, K, seed=13)
    H = g(M, K, seed=14, relu=True)
    res = g(M, K, seed=15)
    dX = torch.empty(M, K, device=dev)
    O.linear_dx(dY, W, dX, rows=M, mask=H, ldmask=K, resid=res)
    ref = (dY @ W) * (H > 0) + res
    assert rel(dX, ref) < 2e-6
    dW = g(N, K, seed=16)
    db = g(N, seed=17)
    dW0, db0 = dW.clone(), db.clone()
    O.linear_dw(dY, X, dW, db, rows=M)
    assert rel(dW, dW0 + dY.t() @ X) < 1e-5
    assert rel(db, db0 + dY.sum(0)) < 1e-5
    # b_rows gather on the TN layout
    table = g(500, K, seed=18)
    idx = torch.randint(0, 500, (M,), generator=torch.Generator().manual_seed(19)).to(dev)
    dW2 = torch.zeros(N, K, device=dev)
    O.linear_dw(dY, table, dW2, None, rows=M, x_rows=idx)
    assert rel(dW2, dY.t() @ table[idx]) < 1e-5


@pytest.mark.parametrize("M,N,K", [(16640, 512, 512), (16600, 512, 2048), (18688, 512, 1536),
                                   (5256, 512, 2048), (5256, 512, 512)])
def test_gemm_tail_split(M, N, K, fp32k):
    """More 128x128 tiles than one wave of workgroups: the partial last wave is split
    over K (zero-fill + atomics) when the epilogue is linear; relu/beta keep one pass.
    (5256 rows x 512: 168 tiles, fewer than the chip's CUs -- the relation workload's
    B = 4 x T_syb = 1314 stack.)"""
    O = ops()
    X, W, b = g(M, K, seed=30), g(N, K, seed=31), g(N, seed=32)
    if fp32k == "fp32_native" and M == 5256:
        # the fewer-tiles-than-CUs split: every tile split over K at K = 2048, none at K = 512
        # (zero fill and atomics outweigh it there); counted on the device's CU count
        plan = O.gemm(X, W, b, M, N, K, lda=K, ldb=K, ldc=N, b_trans=True, bias=b,
                      plan_only=True)
        if torch.cuda.get_device_properties(0).multi_processor_count > 168:
            assert (plan[2] >= 2) if K == 2048 else (plan[2] == 0), plan
    res = g(M, N, seed=33)
    H = g(M, N, seed=34, relu=True)
    out = torch.full((M, N), float("nan"), device=dev)
    O.gemm(X, W, out, M, N, K, lda=K, ldb=K, ldc=N, b_trans=True, bias=b, resid=res, ldr=N,
           mask=H, ldmask=N)
    ref = (X.double() @ W.double().t() + b.double()) * (H > 0).double() + res.double()
    tol = 1e-5  # fp32 accumulation over K <= 2048 against an fp64 reference
    assert rel(out, ref) < tol
    out2 = torch.full((M, N), float("nan"), device=dev)
    O.linear(X, W, b, out2, relu=True)
    assert rel(out2, torch.relu(X.double() @ W.double().t() + b.double())) < tol


@pytest.mark.parametrize("N,K,rows", [(1536, 512, 18688), (6144, 512, 18688), (512, 2048, 12800)])
def test_gemm_dw_auto_split(N, K, rows, fp32k):
    O = ops()
    dY, X = g(rows, N, seed=35), g(rows, K, seed=36)
    dW = g(N, K, seed=37)
    dW0 = dW.clone()
    O.linear_dw(dY, X, dW, None, rows=rows)
    assert rel(dW, dW0.double() + dY.double().t() @ X.double()) < 1e-5


@pytest.mark.parametrize("M,N,K", [(33, 65, 37), (256, 512, 2048), (256, 914, 1024), (1, 7, 3),
                                   (512, 512, 520), (16, 1024, 256)])
@pytest.mark.parametrize("at,bt", [(False, True), (False, False), (True, False), (True, True)])
def test_gemm_skinny_layouts(M, N, K, at, bt):
    """Few-tile problems run the skinny kernel (32x32 tiles, K split over 8 waves): every
    operand layout, K tails, an m/n gather and the fused bias-gradient column sum."""
    O = ops()
    A = g(K, M, seed=40) if at else g(M, K, seed=40)
    B = g(N, K, seed=41) if bt else g(K, N, seed=41)
    Ar = A.t() if at else A
    Br = B.t() if bt else B
    bias = g(N, seed=42)
    out = torch.full((M, N), float("nan"), device=dev)
    cs = torch.zeros(M, device=dev) if at else None
    O.gemm(A, B, out, M, N, K, lda=M if at else K, ldb=K if bt else N, ldc=N, a_trans=at,
           b_trans=bt, bias=bias, relu=True, colsum_a=cs)
    ref = torch.relu(Ar.double() @ Br.double() + bias.double())
    assert rel(out, ref) < 1e-5
    if at:
        assert rel(cs, Ar.double().sum(1)) < 1e-5
    if not at:  # gather rows of A through a_rows (embedding-style)
        idx = torch.randint(0, M, (M,), generator=torch.Generator().manual_seed(43)).to(dev)
        out2 = torch.empty(M, N, device=dev)
        O.gemm(A, B, out2, M, N, K, lda=K, ldb=K if bt else N, ldc=N, b_trans=bt, a_rows=idx)
        assert rel(out2, Ar.double()[idx] @ Br.double()) < 1e-5


def test_gemm_mask_arows_rowscale(fp32k):
    O = ops()
    M, N, K = 50, 96, 64
    src = g(200, N, seed=20, relu=True)       # mask source in gathered-row space
    A = g(200, K, seed=21)
    idx = torch.randperm(200, generator=torch.Generator().manual_seed(22))[:M].to(dev)
    W = g(K, N, seed=23)                       # B stored [K][N]
    out = torch.empty(M, N, device=dev)
    O.gemm(A, W, out, M, N, K, lda=K, ldb=N, ldc=N, a_rows=idx, mask=src, ldmask=N, mask_arows=True)
    ref = (A[idx] @ W) * (src[idx] > 0)
    assert rel(out, ref) < 2e-6
    rs = (torch.arange(M, device=dev) % 3 != 0).float()
    W2 = g(N, K, seed=24)
    O.linear(A, W2, None, out, relu=True, rows=M, a_rows=idx, rowscale=rs)
    ref = torch.relu(A[idx] @ W2.t()) * rs[:, None]
    assert rel(out, ref) < 2e-6


def _ln_ref(z, gam, bet):
    m = z.mean(-1, keepdim=True)
    return gam * (z - m) / (z.std(-1, keepdim=True) + 1e-8) + bet


def test_layernorm_fwd_bwd():
    O = ops()
    R, Cc = 333, 512
    x, r = g(R, Cc, seed=30), g(R, Cc, seed=31)
    gam, bet = g(Cc, seed=32) * 0.2 + 1, g(Cc, seed=33) * 0.2
    y, z = torch.empty_like(x), torch.empty_like(x)
    mean, rden, std, flag = (torch.empty(R, device=dev) for _ in range(4))
    xs = (torch.arange(R, device=dev) % 5 != 0).float()
    O.ln_fwd(x, gam, bet, y, mean, rden, std, r=r, z_out=z, flag=flag, xscale=xs)
    zz = (x * xs[:, None] + r)
    ref = _ln_ref(zz.double(), gam.double(), bet.double())
    assert rel(y, ref) < 5e-6
    assert torch.equal(flag.cpu(), (ref.sum(-1) != 0).float().cpu())
    dy = g(R, Cc, seed=34)
    dz = torch.empty_like(x)
    dg, db = torch.zeros(Cc, device=dev), torch.zeros(Cc, device=dev)
    O.ln_bwd(dy, z, mean, rden, std, gam, dz, dg, db)
    zd = zz.double().cpu().requires_grad_(True)
    gd, bd = gam.double().cpu().requires_grad_(True), bet.double().cpu().requires_grad_(True)
    (_ln_ref(zd, gd, bd) * dy.double().cpu()).sum().backward()
    assert rel(dz, zd.grad) < 1e-5
    assert rel(dg, gd.grad) < 1e-5
    assert rel(db, bd.grad) < 1e-5


@pytest.mark.parametrize("R,Cc", [(18688, 512), (4099, 1024), (7, 256)])
def test_layernorm_bwd_param_grads_fixed_order(R, Cc):
    """dgamma/dbeta: per-workgroup partials added in block order (512 partial rows at the
    cfg-2 shape), accumulated into the caller's buffers, and bit-identical run to run."""
    O = ops()
    x = g(R, Cc, seed=40)
    gam, bet = g(Cc, seed=41) * 0.2 + 1, g(Cc, seed=42) * 0.2
    y, z = torch.empty_like(x), torch.empty_like(x)
    mean, rden, std = (torch.empty(R, device=dev) for _ in range(3))
    O.ln_fwd(x, gam, bet, y, mean, rden, std, z_out=z)
    dy = g(R, Cc, seed=43)
    g0, b0 = g(Cc, seed=44), g(Cc, seed=45)
    outs = []
    for _ in range(3):
        dz = torch.empty_like(x)
        dg, db = g0.clone(), b0.clone()
        O.ln_bwd(dy, z, mean, rden, std, gam, dz, dg, db)
        outs.append((dz, dg, db))
    for o in outs[1:]:
        for a, b in zip(o, outs[0]):
            assert torch.equal(a, b)
    zd = x.double()
    nrm = (zd - zd.mean(-1, keepdim=True)) / (zd.std(-1, keepdim=True) + 1e-8)
    dyd = dy.double()
    assert rel(outs[0][1], g0.double() + (dyd * nrm).sum(0)) < 1e-5
    assert rel(outs[0][2], b0.double() + dyd.sum(0)) < 1e-5


def _attn_ref(Q, K, V, G, kf, qf, h=8):
    """modules.py:246-301 core on already-projected (post-ReLU) Q, K, V."""
    B, Tq, D = Q.shape
    Tk = K.shape[1]
    cat = lambda X: torch.cat(torch.chunk(X, h, 2), 0)
    S = torch.bmm(cat(Q), cat(K).permute(0, 2, 1)) / 8.0
    km = kf.repeat(h, 1).unsqueeze(1).repeat(1, Tq, 1)
    cond = km.eq(0).to(S.dtype)
    S = torch.ones_like(S) * (-2 ** 32 + 1) * cond + S * (1 - cond)
    A = F.softmax(S, -1) * G.repeat(h, 1, 1)
    N = F.normalize(A, p=1, dim=-1)
    P = N * qf.repeat(h, 1).unsqueeze(2)
    Oc = torch.bmm(P, cat(V))
    return torch.cat(torch.chunk(Oc, h, 0), 2), N


@pytest.mark.parametrize("B,Tq,Tk,kind", [(3, 50, 50, "self"), (2, 73, 73, "self"),
                                           (5, 1, 73, "cross"), (2, 20, 100, "self"),
                                           (2, 128, 128, "self"), (3, 17, 33, "cross"),
                                           (4, 1, 50, "cross"), (2, 16, 16, "self"),
                                           (1, 5, 3, "cross"), (2, 100, 7, "cross"),
                                           (3, 1, 128, "cross"), (2, 1, 5, "cross"),
                                           (2, 1, 3, "cross"), (3, 4, 33, "cross"),
                                           (3, 1, 17, "cross"), (2, 1, 65, "cross"),
                                           (2, 1, 16, "cross")])
def test_graph_attention_fwd_bwd(B, Tq, Tk, kind):
    O = ops()
    H, D = 8, 512
    qkv = g(B * Tk, 3 * D, seed=40, relu=True) if kind == "self" and Tq == Tk else None
    if qkv is not None:
        Q, K, V = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
        ldq = ldk = ldv = 3 * D
    else:
        Q = g(B * Tq, D, seed=41, relu=True)
        kv = g(B * Tk, 2 * D, seed=42, relu=True)
        K, V = kv[:, :D], kv[:, D:]
        ldq, ldk, ldv = D, 2 * D, 2 * D
    G = (torch.rand(B, Tq, Tk, generator=torch.Generator().manual_seed(43)) < 0.4).float().to(dev)
    G[0, :3] = 0.0  # rows that attend to nothing
    kf = torch.ones(B, Tk, device=dev)
    kf[0, 2] = 0.0
    kf[-1, -1] = 0.0
    qf = torch.ones(B, Tq, device=dev)
    qf[-1, 0] = 0.0
    out = torch.empty(B * Tq, D, device=dev)
    att = torch.empty(H * B, Tq, Tk, device=dev)
    O.gattn_fwd(Q, ldq, K, ldk, V, ldv, G, kf, qf, B, Tq, Tk, H, out, D, att)
    Qr = Q.reshape(B, Tq, D).double().cpu().requires_grad_(True)
    Kr = K.reshape(B, Tk, D).double().cpu().requires_grad_(True)
    Vr = V.reshape(B, Tk, D).double().cpu().requires_grad_(True)
    ref, Nref = _attn_ref(Qr, Kr, Vr, G.double().cpu(), kf.double().cpu(), qf.double().cpu())
    assert rel(out.view(B, Tq, D), ref) < 2e-5
    assert rel(att, Nref) < 2e-5
    dO = g(B * Tq, D, seed=44)
    (ref * dO.view(B, Tq, D).double().cpu()).sum().backward()
    dq = torch.empty(B * Tq, D, device=dev)
    dk = torch.empty(B * Tk, D, device=dev)
    dv = torch.empty(B * Tk, D, device=dev)
    O.gattn_bwd(Q, ldq, K, ldk, V, ldv, G, kf, qf, B, Tq, Tk, H, dO, D, dq, D, dk, D, dv, D)
    mq, mk, mv = (Qr > 0), (Kr > 0), (Vr > 0)
    assert rel(dq.view(B, Tq, D), Qr.grad * mq) < 5e-5
    assert rel(dk.view(B, Tk, D), Kr.grad * mk) < 5e-5
    assert rel(dv.view(B, Tk, D), Vr.grad * mv) < 5e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_single_query_attention_one_key_and_reruns(dt):
    """T_q = 1 kernels (one workgroup per (sample, head), keys split over its 4 waves): with one
    key the softmax weight is exactly 1, so dQ and dK are exactly 0 as in the reference (the
    cross-wave sums add exact zeros); at T_k = 73 / 128 reruns are bit-identical."""
    O = ops()
    H, D = 8, 512
    for B, Tk in ((3, 1), (4, 73), (2, 128)):
        Q = g(B, D, seed=70, relu=True)
        kv = g(B * Tk, 2 * D, seed=71, relu=True).to(dt)
        G = torch.ones(B, 1, Tk, device=dev)
        G[:, :, ::3] = 0.5
        kf, qf = torch.ones(B, Tk, device=dev), torch.ones(B, 1, device=dev)
        dO = g(B, D, seed=72)
        outs = []
        for _ in range(2):
            o = torch.empty(B, D, device=dev)
            dq = torch.empty(B, D, device=dev)
            dkv = torch.empty(B * Tk, 2 * D, device=dev, dtype=dt)
            O.gattn_fwd(Q, D, kv, 2 * D, kv[:, D:], 2 * D, G, kf, qf, B, 1, Tk, H, o, D)
            O.gattn_bwd(Q, D, kv, 2 * D, kv[:, D:], 2 * D, G, kf, qf, B, 1, Tk, H, dO, D, dq, D,
                        dkv, 2 * D, dkv[:, D:], 2 * D)
            outs.append((o, dq, dkv))
        for a, b_ in zip(*outs):
            assert torch.equal(a, b_)
        o, dq, dkv = outs[0]
        if Tk == 1:
            assert int((dq != 0).sum()) == 0 and int((dkv[:, :D] != 0).sum()) == 0
            assert torch.equal(o, kv[:, D:].float())   # P = 1 (G / |G| = 1) times V


@pytest.mark.parametrize("B,Tq,Tk,kind", [(3, 50, 50, "self"), (2, 73, 73, "self"),
                                           (5, 1, 73, "cross"), (4, 1, 50, "cross"),
                                           (2, 128, 128, "self"), (3, 17, 33, "cross")])
def test_graph_attention_bf16_storage(B, Tq, Tk, kind):
    """bf16-storage attention (savqa_gattn_{fwd,bwd}_bf16; cfg 3 / cfg 5) against the fp32
    kernels and the fp64 reference on the bf16-rounded inputs. T_q = 1 (single-query kernels):
    the same fp32 math, so O equals the fp32 kernel's to fp32 rounding. T_q > 1 (bf16 MFMA
    strip kernels): S = QK^T is exact (bf16 products, fp32 sums) and the softmax / graph / L1
    chain is fp32, but P, dS and dO enter their second products rounded to bf16 (as in a bf16
    attention), so O is within a few bf16 ulps (tolerance 4e-3 relative Frobenius, ~1 ulp =
    3.9e-3 per element, averaged down over 64-term sums); dQ/dK/dV carry one more rounding."""
    O = ops()
    H, D = 8, 512
    bf = torch.bfloat16
    if kind == "self":
        qkv = g(B * Tk, 3 * D, seed=50, relu=True).to(bf)
        Q, K, V = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
        ldq = ldk = ldv = 3 * D
    else:
        Q = g(B * Tq, D, seed=51, relu=True).to(bf)
        kv = g(B * Tk, 2 * D, seed=52, relu=True).to(bf)
        K, V = kv[:, :D], kv[:, D:]
        ldq, ldk, ldv = D, 2 * D, 2 * D
    G = (torch.rand(B, Tq, Tk, generator=torch.Generator().manual_seed(53)) < 0.4).float().to(dev)
    G[0, :3] = 0.0
    kf = torch.ones(B, Tk, device=dev)
    kf[0, 2] = 0.0
    qf = torch.ones(B, Tq, device=dev)
    qf[-1, 0] = 0.0
    Qf, Kf, Vf = (x.float().contiguous() for x in (Q, K, V))
    o16 = torch.empty(B * Tq, D, device=dev)
    o32 = torch.empty(B * Tq, D, device=dev)
    O.gattn_fwd(Q, ldq, K, ldk, V, ldv, G, kf, qf, B, Tq, Tk, H, o16, D)
    O.gattn_fwd(Qf, D, Kf, D, Vf, D, G, kf, qf, B, Tq, Tk, H, o32, D)
    tol_o = 1e-6 if Tq == 1 else 4e-3
    assert rel(o16, o32) < tol_o
    dO = g(B * Tq, D, seed=54)
    d16 = [torch.empty(B * n, D, device=dev, dtype=bf) for n in (Tq, Tk, Tk)]
    d32 = [torch.empty(B * n, D, device=dev) for n in (Tq, Tk, Tk)]
    O.gattn_bwd(Q, ldq, K, ldk, V, ldv, G, kf, qf, B, Tq, Tk, H, dO, D, d16[0], D, d16[1], D,
                d16[2], D)
    O.gattn_bwd(Qf, D, Kf, D, Vf, D, G, kf, qf, B, Tq, Tk, H, dO, D, d32[0], D, d32[1], D, d32[2], D)
    for a, b_ in zip(d16, d32):
        assert rel(a.float(), b_.to(bf).float()) < 1e-2   # one bf16 rounding (+ fp32 order)
        assert rel(a.float(), b_) < 1e-2
    Qr = Qf.reshape(B, Tq, D).double().cpu().requires_grad_(True)
    Kr = Kf.reshape(B, Tk, D).double().cpu().requires_grad_(True)
    Vr = Vf.reshape(B, Tk, D).double().cpu().requires_grad_(True)
    ref, _ = _attn_ref(Qr, Kr, Vr, G.double().cpu(), kf.double().cpu(), qf.double().cpu())
    assert rel(o16.view(B, Tq, D), ref) < (2e-5 if Tq == 1 else 4e-3)
    (ref * dO.view(B, Tq, D).double().cpu()).sum().backward()
    assert rel(d16[0].float().view(B, Tq, D), Qr.grad * (Qr > 0)) < 1e-2
    assert rel(d16[1].float().view(B, Tk, D), Kr.grad * (Kr > 0)) < 1e-2
    assert rel(d16[2].float().view(B, Tk, D), Vr.grad * (Vr > 0)) < 1e-2


@pytest.mark.parametrize("Tk", [50, 73, 128])
def test_graph_attention_fp32_query_bf16_kv(Tk):
    """The decoder's cross-attention in the bf16 mode: fp32 single query (and dQ), bf16 K/V
    (and dK/dV); equals the fp32 kernels on the bf16-rounded K/V."""
    O = ops()
    B, H, D = 6, 8, 512
    Q = g(B, D, seed=60, relu=True)
    kv = g(B * Tk, 2 * D, seed=61, relu=True).to(torch.bfloat16)
    K, V = kv[:, :D], kv[:, D:]
    Kf, Vf = K.float().contiguous(), V.float().contiguous()
    G = (torch.rand(B, 1, Tk, generator=torch.Generator().manual_seed(62)) < 0.5).float().to(dev)
    kf = torch.ones(B, Tk, device=dev)
    kf[1, 3] = 0.0
    qf = torch.ones(B, 1, device=dev)
    o16, o32 = torch.empty(B, D, device=dev), torch.empty(B, D, device=dev)
    O.gattn_fwd(Q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, 1, Tk, H, o16, D)
    O.gattn_fwd(Q, D, Kf, D, Vf, D, G, kf, qf, B, 1, Tk, H, o32, D)
    assert rel(o16, o32) < 1e-6
    dO = g(B, D, seed=63)
    dq16, dq32 = torch.empty(B, D, device=dev), torch.empty(B, D, device=dev)
    dkv16 = torch.empty(B * Tk, 2 * D, device=dev, dtype=torch.bfloat16)
    dk32, dv32 = torch.empty(B * Tk, D, device=dev), torch.empty(B * Tk, D, device=dev)
    O.gattn_bwd(Q, D, K, 2 * D, V, 2 * D, G, kf, qf, B, 1, Tk, H, dO, D, dq16, D, dkv16, 2 * D,
                dkv16[:, D:], 2 * D)
    O.gattn_bwd(Q, D, Kf, D, Vf, D, G, kf, qf, B, 1, Tk, H, dO, D, dq32, D, dk32, D, dv32, D)
    assert rel(dq16, dq32) < 1e-6
    assert rel(dkv16[:, :D].float(), dk32) < 1e-2
    assert rel(dkv16[:, D:].float(), dv32) < 1e-2


def test_graph_build_matches_oracle():
    from oracle import savqa_oracle as OR
    O = ops()
    B, Nn, Lq = 3, 9, 5
    gen = torch.Generator().manual_seed(50)
    nm = torch.zeros(B, Nn, Nn, dtype=torch.int32)
    qm = torch.zeros(B, Lq, Lq, dtype=torch.int32)
    for b, (n, l) in enumerate([(9, 5), (4, 3), (0, 5)]):
        nm[b, :n, :n] = 1
        qm[b, :l, :l] = 1
    qg = (torch.rand(B, Lq, Lq, generator=gen) < 0.3).int()
    ng = (torch.rand(B, Nn, Nn, generator=gen) < 0.3).int()
    T = Nn + Lq
    for node_graph in (None, ng):
        for dec in (True, False):
            gd, gr, dm = (torch.empty(B, T, T, device=dev), torch.empty(B, T, T, device=dev),
                          torch.empty(B, 1, T, device=dev))
            O.graph_build(nm.to(dev), qm.to(dev), qg.to(dev),
                          None if node_graph is None else node_graph.to(dev), B, Nn, Lq, dec, gd, gr, dm)
            rgd, rg, rdm = OR.build_graphs(nm, qm, qg, node_graph, dec)
            assert torch.equal(gd.cpu(), rgd) and torch.equal(gr.cpu(), rg) and torch.equal(dm.cpu(), rdm)


@pytest.mark.parametrize("K,H", [(5, 64), (5, 1024), (8, 1000), (1, 512), (9, 64), (5, 1028)])
def test_mil_core_fwd_bwd(K, H):
    """MIL-NCE core (AttModel_x3.py:358-373) against fp64 autograd: the single-pass
    one-workgroup-per-row kernels (topN <= 8, H <= 1024; their scores are summed in the one-wave
    kernels' order: the same object features bit for bit) and the one-wave kernels past them."""
    O = ops()
    B, Nv, eps = 3, 7, 1e-6
    Pf = g(B * Nv * K, H, seed=60, relu=True) * 0.2
    Nf = g(B * Nv * K, H, seed=61, relu=True) * 0.2
    v = g(B * Nv, H, seed=62, relu=True) * 0.2
    mask = torch.ones(B, Nv, K, dtype=torch.int32)
    mask[1, 3:] = 0
    obj = torch.empty(B * Nv, H, device=dev)
    ws = torch.empty(B * Nv, device=dev)
    mil = torch.empty((), device=dev)
    O.mil_fwd(Pf, Nf, v, mask.to(dev), B * Nv, K, H, eps, obj, ws, mil)
    P4 = Pf.view(B, Nv, K, H).double().cpu().requires_grad_(True)
    N4 = Nf.view(B, Nv, K, H).double().cpu().requires_grad_(True)
    v4 = v.view(B, Nv, H).double().cpu().requires_grad_(True)
    m4 = mask.double().unsqueeze(3)
    vv = v4.unsqueeze(3)
    sp = m4 * torch.matmul(P4, vv)
    sn = m4 * torch.matmul(N4, vv)
    z = torch.zeros(sn.size(), dtype=torch.double)
    ref_mil = torch.mean(torch.logsumexp(torch.cat((sp.clamp(min=eps), z.clamp(min=eps)), 1), 2)
                         - torch.logsumexp(torch.cat((sp.clamp(min=eps), sn.clamp(min=eps)), 1), 2))
    ref_obj = torch.sum(F.softmax(torch.matmul(P4, vv), dim=2) * P4, dim=2)
    assert abs(float(mil) - float(ref_mil)) < 1e-5 * max(1.0, abs(float(ref_mil)))
    assert rel(obj.view(B, Nv, H), ref_obj) < 1e-5
    dobj = g(B * Nv, H, seed=63)
    dmil = torch.tensor(-1.7, device=dev)
    (ref_obj * dobj.view(B, Nv, H).double().cpu()).sum().add(ref_mil * -1.7).backward()
    dPf, dNf, dv = torch.empty_like(Pf), torch.empty_like(Nf), torch.empty_like(v)
    O.mil_bwd(Pf, Nf, v, mask.to(dev), B * Nv, K, H, eps, dobj, dmil, dPf, dNf, dv)
    assert rel(dPf.view(B, Nv, K, H), P4.grad * (P4 > 0)) < 1e-5
    assert rel(dNf.view(B, Nv, K, H), N4.grad * (N4 > 0)) < 1e-5
    assert rel(dv.view(B, Nv, H), v4.grad * (v4 > 0)) < 1e-5


def test_loss_matches_oracle():
    from oracle import savqa_oracle as OR
    O = ops()
    B, Cc = 6, 914
    lc, lv, ls = g(B, Cc, seed=70), g(B, Cc, seed=71), g(B, Cc, seed=72)
    ans = torch.randint(1, Cc, (B,), generator=torch.Generator().manual_seed(73))
    mil = torch.tensor(0.37, device=dev)
    loss = torch.empty((), device=dev)
    dl = torch.empty(3, B, Cc, device=dev)
    lsm = torch.empty(B, Cc, device=dev)
    ws = torch.empty(B, device=dev)
    O.loss_fwd(lc, lv, ls, ans.to(dev), B, Cc, 0.1, mil, True, loss, dl, lsm, ws)
    t = [x.double().cpu().requires_grad_(True) for x in (lc, lv, ls)]
    ref, ref_lsm = OR.train_loss(t[0], t[1], t[2], ans, torch.tensor(0.37, dtype=torch.double))
    ref.backward()
    assert abs(float(loss) - float(ref)) < 1e-5 * abs(float(ref))
    assert rel(lsm, ref_lsm) < 1e-6
    for i in range(3):
        assert rel(dl[i], t[i].grad) < 1e-5


def test_adam_matches_oracle():
    from oracle import savqa_oracle as OR
    O = ops()
    n = 10003
    p, gr = g(n, seed=80), g(n, seed=81)
    m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    P = {"x": p.cpu().clone()}
    st = {}
    for step in (1, 2, 3):
        gg = gr * step
        O.adam(p, gg, m, v, n, 1e-4, 0.9, 0.999, 1e-8, 1 - 0.9 ** step, 1 - 0.999 ** step)
        OR.adam_step(P, {"x": gg.cpu()}, st, step)
    assert rel(p, P["x"]) < 1e-6


@pytest.mark.parametrize("prec,tol", [(3, 1e-4), (6, 2e-6)])
@pytest.mark.parametrize("lay", ["NT", "NN", "TN"])
@pytest.mark.parametrize("M,N,K", [(2048, 2048, 512), (4100, 1280, 520), (2100, 1536, 96)])
def test_gemm_bf16_paths(prec, tol, lay, M, N, K):
    """3xbf16 (prec 3, the "bf16x3" mode) and x6 (prec 6, fp32 from exact three-term splits)
    MFMA GEMMs against fp64, with the
    same epilogues as the fp32 path (bias+ReLU forward, residual dX, split-K dW with the
    bias-gradient column sums), including edge tiles and k tails."""
    O = ops()
    if lay == "NT":
        X, W, b = g(M, K, seed=70), g(N, K, seed=71), g(N, seed=72)
        res = g(M, N, seed=73)
        out = torch.empty(M, N, device=dev)
        O.gemm(X, W, out, M, N, K, lda=K, ldb=K, ldc=N, b_trans=True, bias=b, relu=True,
               resid=res, ldr=N, prec=prec)
        ref = torch.relu(X.double() @ W.double().t() + b.double()) + res.double()
        scale = (X.double().abs() @ W.double().abs().t()).max()
    elif lay == "NN":
        A, W = g(M, K, seed=74), g(K, N, seed=75)
        out = torch.empty(M, N, device=dev)
        O.gemm(A, W, out, M, N, K, lda=K, ldb=N, ldc=N, prec=prec)
        ref = A.double() @ W.double()
        scale = (A.double().abs() @ W.double().abs()).max()
    else:
        A, X = g(K, M, seed=76), g(K, N, seed=77)
        out = torch.zeros(M, N, device=dev)
        cs = torch.zeros(M, device=dev)
        O.gemm(A, X, out, M, N, K, lda=M, ldb=N, ldc=N, a_trans=True, atomic=True, split_k=-1,
               colsum_a=cs, prec=prec)
        ref = A.double().t() @ X.double()
        scale = (A.double().abs().t() @ X.double().abs()).max()
        assert rel(cs, A.double().sum(0)) < 1e-5  # column sums stay fp32
    err = float((out.double() - ref).abs().max() / scale)
    assert err < tol, err
    if prec == 3:  # 3xbf16 is not plain bf16: at least 100x closer to fp64
        assert err < 1e-4


CFG2_SHAPES = [("NT", 18688, 1536, 512), ("NT", 18688, 2048, 512), ("NT", 18688, 512, 2048),
               ("NT", 18688, 6144, 512), ("NN", 18688, 2048, 512), ("NN", 18688, 512, 2048),
               ("NN", 18688, 512, 1536), ("NN", 18688, 512, 6144), ("TN", 1536, 512, 18688),
               ("TN", 2048, 512, 18688), ("TN", 512, 2048, 18688), ("TN", 6144, 512, 18688)]


@pytest.mark.parametrize("x6", [6])
@pytest.mark.parametrize("lay,M,N,K", CFG2_SHAPES)
def test_gemm_x6_error_at_most_native(lay, M, N, K, x6):
    """The x6 kernel is an fp32 GEMM: on every cfg-2 step shape (forward NT, dX NN, split-K
    dW TN with the bias-gradient column sums) its max error against fp64 is within 1.25x of
    the native fp32 MFMA kernel's on the same inputs (measured: at or below it). The split-K
    slices of both kernels are summed through slabs in a fixed order (ops.GEMM_SLABS), so
    the comparison no longer depends on the order fp32 atomics land in."""
    O = ops()
    if lay == "NT":
        A, B = g(M, K, seed=90), g(N, K, seed=91)
        kw = dict(lda=K, ldb=K, ldc=N, b_trans=True)
        ref = A.double() @ B.double().t()
    elif lay == "NN":
        A, B = g(M, K, seed=92), g(K, N, seed=93)
        kw = dict(lda=K, ldb=N, ldc=N)
        ref = A.double() @ B.double()
    else:
        A, B = g(K, M, seed=94), g(K, N, seed=95)
        kw = dict(lda=M, ldb=N, ldc=N, a_trans=True, atomic=True, split_k=-1)
        ref = A.double().t() @ B.double()
    errs = {}
    for prec in (0, x6):
        out = torch.zeros(M, N, device=dev)
        cs = torch.zeros(M, device=dev) if lay == "TN" else None
        O.gemm(A, B, out, M, N, K, colsum_a=cs, prec=prec, **kw)
        errs[prec] = float((out.double() - ref).abs().max() / ref.abs().max())
        if cs is not None:
            assert rel(cs, A.double().sum(0)) < 1e-5
    assert errs[x6] <= 1.25 * errs[0] + 1e-8, errs
    assert errs[x6] < 5e-6, errs


@pytest.mark.parametrize("prec", [0, 6])
@pytest.mark.parametrize("case", ["splitk_dw", "tail"])
def test_gemm_slabs_deterministic(prec, case, monkeypatch):
    """K splits through partial slabs (savqa_gemm_desc.ws, ops.GEMM_SLABS): the split-K
    weight gradient (with its fused bias-gradient column sums) and a tail-split forward with a
    residual are bit-identical run to run, and agree with the atomic form to fp32 rounding."""
    O = ops()
    if case == "splitk_dw":
        M, N, K = 2048, 512, 18688
        A, B = g(K, M, seed=31), g(K, N, seed=32)
        kw = dict(lda=M, ldb=N, ldc=N, a_trans=True, atomic=True, split_k=-1)
        ref = A.double().t() @ B.double()
    else:
        M, N, K = 18688, 512, 2048
        A, B = g(M, K, seed=33), g(N, K, seed=34)
        R = g(M, N, seed=35)
        kw = dict(lda=K, ldb=K, ldc=N, b_trans=True, resid=R, ldr=N)
        ref = A.double() @ B.double().t() + R.double()
    plan = O.gemm(A, B, None, M, N, K, prec=prec, plan_only=True, **kw)
    assert plan[0] == 128 and (plan[1] > 1 if case == "splitk_dw" else plan[2] > 1), plan

    # the weight gradient ACCUMULATES (the slab reduce's C += sum, colsum += sum branch, which
    # runs every step since GEMM_SLABS became the default): start from an existing gradient
    gen = torch.Generator(device=dev).manual_seed(36)
    c0 = torch.randn(M, N, generator=gen, device=dev) if case == "splitk_dw" else None
    s0 = torch.randn(M, generator=gen, device=dev) if case == "splitk_dw" else None

    def run():
        out = c0.clone() if c0 is not None else torch.zeros(M, N, device=dev)
        cs = s0.clone() if s0 is not None else None
        O.gemm(A, B, out, M, N, K, prec=prec, colsum_a=cs, **kw)
        torch.cuda.synchronize()
        return out, cs
    outs = [run() for _ in range(3)]
    for o, c in outs[1:]:
        assert torch.equal(o, outs[0][0])
        if c is not None:
            assert torch.equal(c, outs[0][1])
    if case == "splitk_dw":
        ref = ref + c0.double()
        assert rel(outs[0][1].double() - s0.double(), A.double().sum(0)) < 1e-5
    assert rel(outs[0][0], ref) < 5e-6
    monkeypatch.setattr(O, "GEMM_SLABS", False)
    atom, _ = run()
    assert rel(atom, outs[0][0]) < 5e-6


def _wide(shape, lo, hi, seed):
    """sign x 10^U(lo, hi): operands spanning many decades (fp32 normal range)."""
    gen = torch.Generator().manual_seed(seed)
    e = torch.empty(shape, dtype=torch.float64).uniform_(lo, hi, generator=gen)
    s = torch.randint(0, 2, shape, generator=gen).double() * 2 - 1
    return (s * torch.pow(10.0, e)).float().to(dev)


@pytest.mark.parametrize("x6", [6])
@pytest.mark.parametrize("lay", ["NT", "NN", "TN"])
@pytest.mark.parametrize("rng", ["wide", "tiny", "huge"])
def test_gemm_x6_wide_dynamic_range(lay, rng, x6):
    """The exact three-term split over operands far from N(0, 1): 'wide' spans 24 decades
    (a1 / a2 of the smallest values stay fp32-normal), 'tiny' puts A at 1e-37..1e-33, where
    a1 / a2 fall below the fp32 / bf16 normal range while every product stays normal, 'huge'
    puts A at 3.35e38..3.40e38, next to FLT_MAX, where a rounded bf16 a0 would be +-inf (the
    truncation split keeps every finite operand) and B at 1e-33..1e-31 (its terms stay normal). Per
    element the error against fp64 is measured relative to sum_k |a||b| (the fp32 GEMM's own
    error scale, meaningful whatever an element's magnitude); x6 within 1.25x of native."""
    O = ops()
    M, N, K = (2048, 2048, 1024) if lay != "TN" else (2048, 1024, 4096)
    alo, ahi, blo, bhi = {"wide": (-12, 12, -12, 12), "tiny": (-37, -33, 1, 5),
                          "huge": (38.525, 38.5315, -33, -31)}[rng]
    if lay == "NT":
        A, B = _wide((M, K), alo, ahi, 1), _wide((N, K), blo, bhi, 2)
        kw = dict(lda=K, ldb=K, ldc=N, b_trans=True)
        Am, Bm = A.double(), B.double().t()
    elif lay == "NN":
        A, B = _wide((M, K), alo, ahi, 3), _wide((K, N), blo, bhi, 4)
        kw = dict(lda=K, ldb=N, ldc=N)
        Am, Bm = A.double(), B.double()
    else:
        A, B = _wide((K, M), alo, ahi, 5), _wide((K, N), blo, bhi, 6)
        kw = dict(lda=M, ldb=N, ldc=N, a_trans=True, atomic=True, split_k=-1)
        Am, Bm = A.double().t(), B.double()
    ref = Am @ Bm
    scale = Am.abs() @ Bm.abs()
    assert O.gemm(A, B, None, M, N, K, prec=x6, plan_only=True, **kw)[0] == 128  # x6 kernel
    errs, rms = {}, {}
    for prec in (0, x6):
        out = torch.zeros(M, N, device=dev)
        O.gemm(A, B, out, M, N, K, prec=prec, **kw)
        assert bool(torch.isfinite(out).all())
        e = (out.double() - ref).abs() / scale
        errs[prec], rms[prec] = float(e.max()), float(e.pow(2).mean().sqrt())
    print(f"x6 wide-range {rng} {lay} prec {x6}: max {errs}, rms {rms}")
    assert rms[x6] <= 1.25 * rms[0] + 1e-10, (errs, rms)
    assert errs[x6] <= 1.25 * errs[0] + 1e-9, (errs, rms)
    assert errs[x6] < 1e-5, errs


def test_gemm_x6_infinite_operands():
    """Non-finite operands (gemm_x6.hip, Range): x6 cannot reproduce fp32's infinities -- the
    split of +-inf is (inf, NaN, NaN) -- but an output is non-finite exactly where the native
    fp32 kernel's is (NaN where fp32 gives +-inf), so overflow still surfaces, and every
    finite output agrees."""
    O = ops()
    M, N, K = 2048, 2048, 512
    A, B = g(M, K, seed=61), g(N, K, seed=62)
    A[3, 7] = float("inf")
    A[100, 300] = float("-inf")
    A[200, 10] = float("inf")
    A[200, 11] = float("-inf")           # row 200: +inf and -inf terms
    B[50, 400] = float("inf")            # column 50: inf in the other operand
    B[60, 5] = float("nan")
    outs = {}
    assert O.gemm(A, B, None, M, N, K, lda=K, ldb=K, ldc=N, b_trans=True, prec=6,
                  plan_only=True)[0] == 128
    for prec in (0, 6):
        out = torch.zeros(M, N, device=dev)
        O.gemm(A, B, out, M, N, K, lda=K, ldb=K, ldc=N, b_trans=True, prec=prec)
        outs[prec] = out.cpu()
    n, x = outs[0], outs[6]
    assert torch.equal(torch.isfinite(n), torch.isfinite(x))
    assert int((~torch.isfinite(n)).sum()) >= 4 * N - 4
    fin = torch.isfinite(n)
    assert rel(x[fin], n[fin]) < 1e-5


@pytest.mark.parametrize("gather", ["b", "a", "ab"])
@pytest.mark.parametrize("N", [300, 256])
def test_gemm_k_row_gathers(gather, N, fp32k):
    """dW-layout GEMMs whose k rows are gathered through token ids (the GloVe-table
    gradient of the micro-object projections: K = B*Nv*topN rows, N = 300): branch-free
    gathered loads on full k-tiles, a guarded last k-tile, clamped edge columns."""
    O = ops()
    M, K, V = 1024, 4612, 700
    gen = torch.Generator().manual_seed(41)
    ia = torch.randint(0, V, (K,), generator=gen).to(dev)
    ib = torch.randint(0, V, (K,), generator=gen).to(dev)
    A = g(V if "a" in gather else K, M, seed=42)  # A(m, k) = A[ra(k)][m]
    B = g(V if "b" in gather else K, N, seed=43)  # B(k, n) = B[rb(k)][n]
    out = torch.zeros(M, N, device=dev)
    O.gemm(A, B, out, M, N, K, lda=M, ldb=N, ldc=N, a_trans=True, atomic=True, split_k=-1,
           a_rows=ia if "a" in gather else None, b_rows=ib if "b" in gather else None)
    Ag = A[ia] if "a" in gather else A
    Bg = B[ib] if "b" in gather else B
    ref = Ag.double().t() @ Bg.double()
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("lay,M,N,K", [("NT", 512, 2048, 512), ("NN", 1024, 512, 2048),
                                       ("TN", 512, 2048, 512), ("NT", 300, 914, 1000),
                                       ("NN", 512, 1024, 914), ("TN", 914, 512, 520),
                                       ("TT", 512, 512, 512)])
def test_gemm_skinny_bf16_products(lay, M, N, K):
    """prec = 1 (ops.PREC "bf16sk", the low-precision modes' decoder / head chain): the skinny
    launches round both operands to bf16 (RNE) and accumulate the exact products in fp32
    (gemm_skinny_bf_kernel) -- held to the fp64 product of the bf16-rounded operands, incl. K
    not a multiple of 16 (the guarded last group), M / N edge tiles, the TN bias-gradient
    column sums (of the fp32 values) and a residual epilogue."""
    O = ops()
    at, bt = lay[0] == "T", lay[1] == "T"
    A = g(K, M, seed=71) if at else g(M, K, seed=71)
    B = g(N, K, seed=72) if bt else g(K, N, seed=72)
    kw = dict(lda=M if at else K, ldb=K if bt else N, ldc=N, a_trans=at, b_trans=bt)
    assert O.gemm(A, B, None, M, N, K, prec=1, plan_only=True, **kw)[0] == 32  # skinny
    Ar = (A.t() if at else A).to(torch.bfloat16).double()
    Br = (B.t() if bt else B).to(torch.bfloat16).double()
    R = torch.randn(M, N, device=dev)
    out = torch.empty(M, N, device=dev)
    cs = torch.zeros(M, device=dev) if at else None
    O.gemm(A, B, out, M, N, K, prec=1, resid=None if at else R, ldr=N, colsum_a=cs, **kw)
    ref = Ar @ Br + (0 if at else R.double())
    assert rel(out, ref) < 1e-5
    exact = (A.t() if at else A).double() @ (B.t() if bt else B).double()
    assert rel(out - (0 if at else R), exact) > 1e-4  # really bf16 products, not fp32 ones
    if cs is not None:
        assert rel(cs, A.double().sum(0)) < 1e-5


@pytest.mark.parametrize("prec", [6, 5])
@pytest.mark.parametrize("lay,M,N,K", [("NT", 18688, 2048, 512), ("NT", 1000, 300, 520),
                                       ("NN", 18688, 512, 2048), ("NN", 777, 1000, 300),
                                       ("NT", 18688, 512, 2048), ("NN", 18688, 512, 6144)])
def test_gemm_x6_weight_planes_bit_identical(lay, M, N, K, prec):
    """savqa_gemm_desc.b_planes (ops.weight_planes: the weight split into the x6 kernel's three
    bf16 plane images once, DMA'd into a double-buffered LDS image by the kernel): the same
    split values meet the same MFMAs, so the outputs are BIT-identical to the launch that
    splits B itself -- M / N / K edges, the tail split (N = 512 at 18688 rows), the two-level
    form (prec 5), an A row gather, a residual and a ReLU-backward mask."""
    O = ops()
    bt = lay == "NT"
    A = g(M, K, seed=81)
    B = g(N, K, seed=82) if bt else g(K, N, seed=82)
    kw = dict(lda=K, ldb=K if bt else N, ldc=N, b_trans=bt, prec=prec)
    R = g(M, N, seed=83)
    H = g(M, N, seed=84, relu=True)
    O.WP_KEY = ("test", lay, M, N, K, prec)
    outs = []
    for planes in (False, True):
        out = torch.empty(M, N, device=dev)
        O.gemm(A, B, out, M, N, K, resid=R, ldr=N, mask=H, ldmask=N, b_planes=planes, **kw)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])
    ref = (A.double() @ (B.double().t() if bt else B.double())) * (H > 0).double() + R.double()
    assert rel(outs[1], ref) < 5e-6
    idx = torch.randint(0, M, (M // 2,), generator=torch.Generator().manual_seed(85)).to(dev)
    gathered = []
    for planes in (False, True):
        out = torch.empty(M // 2, N, device=dev)
        O.gemm(A, B, out, M // 2, N, K, a_rows=idx, b_planes=planes, **kw)
        gathered.append(out)
    assert torch.equal(gathered[0], gathered[1])


def _planes_ref(Bv, N, K):
    """The x6 plane image of an [N][K] fp32 matrix (savqa_x6_weight_planes' layout, restated):
    per (128-row n tile, 32-k tile) three 128 x 32 bf16 planes, row r at 64 B, 16-B chunk
    (k / 8) XOR S[(r / 4) % 4] with S = {0, 2, 3, 1}; plane p holds the top 16 bits of the
    p-th truncation residue (a0 = a with its low 16 bits cleared, a1 of a - a0, ...)."""
    NT, KT = (N + 127) // 128, (K + 31) // 32
    P = torch.zeros(NT * 128, KT * 32, dtype=torch.float32, device=Bv.device)
    P[:N, :K] = Bv
    x = P.clone()
    terms = []
    for _ in range(3):
        hi = (x.view(torch.int32) & -65536).view(torch.float32)
        terms.append((hi.view(torch.int32) >> 16).to(torch.int16))
        x = x - hi
    img = torch.zeros(NT, KT, 3, 128, 32, dtype=torch.int16, device=Bv.device)
    r = torch.arange(128, device=Bv.device)
    swz = (0x1320 >> (4 * ((r >> 2) & 3))) & 3
    k = torch.arange(32, device=Bv.device)
    col = (((k[None, :] >> 3) ^ swz[:, None]) << 3) + (k[None, :] & 7)   # [128, 32] -> slot
    for p in range(3):
        t = terms[p].view(NT, 128, KT, 32).permute(0, 2, 1, 3)            # [NT, KT, 128, 32]
        img[:, :, p].scatter_(3, col.expand(NT, KT, 128, 32), t)
    return img.flatten().view(torch.uint8)


def test_x6_weight_planes_batch_matches_reference_layout():
    """savqa_x6_weight_planes_batch over 40 operands (two launches of <= 32 jobs): k-contiguous
    and n-contiguous B, ragged N / K, a leading dimension wider than the operand, an operand
    not 16-B aligned -- every image byte-equal to the layout restated in torch (_planes_ref),
    and to the one-operand entry point."""
    import ctypes as C
    from savqa_amd import _lib
    O = ops()
    shapes = [(512, 512), (300, 520), (2048, 512), (129, 33), (1000, 300), (64, 31), (6144, 512)]
    jobs, refs, keep = [], [], []
    for i in range(40):
        N, K = shapes[i % len(shapes)]
        bt = bool(i % 2)
        ld = (K if bt else N) + (7 if i % 3 == 0 else 0)
        off = 1 if i % 5 == 4 else 0
        rows = N if bt else K
        store = g(rows * ld + off, 1, seed=200 + i).flatten()
        W = store[off:]
        Bv = W[:rows * ld].view(rows, ld)[:, :(K if bt else N)]
        Bnk = Bv if bt else Bv.t()
        out = torch.zeros(int(_lib.load().savqa_x6_weight_planes_bytes(N, K)), dtype=torch.uint8,
                          device=dev)
        keep += [store, out]
        jobs.append((W, ld, bt, N, K, out))
        refs.append(_planes_ref(Bnk, N, K))
    arr = (_lib.PlanesJob * len(jobs))()
    for i, (W, ld, bt, N, K, out) in enumerate(jobs):
        arr[i].B, arr[i].ldb, arr[i].b_trans = W.data_ptr(), ld, int(bt)
        arr[i].N, arr[i].K, arr[i].out = N, K, out.data_ptr()
    O.call("savqa_x6_weight_planes_batch", O._stream(), C.cast(arr, C.c_void_p), len(jobs))
    torch.cuda.synchronize()
    for i, (W, ld, bt, N, K, out) in enumerate(jobs):
        assert torch.equal(out, refs[i]), (i, N, K, bt, ld)
        one = torch.full_like(out, 7)
        O.call("savqa_x6_weight_planes", O._stream(), W.data_ptr(), ld, int(bt), N, K,
               one.data_ptr())
        assert torch.equal(one, out), i


@pytest.mark.parametrize("M,N,K,tile", [(3584, 512, 1024, 128), (3584, 300, 2048, 128),
                                        (1024, 2048, 512, 32), (256, 2048, 512, 32)])
def test_gemm_planner_tall_launches(M, N, K, tile):
    """plan_gemm: 128x128-tile launches with < 160 tiles go to the skinny kernels (tuned on the
    M = B decoder rows) except tall ones (M >= 2048) with >= 80 tiles, which take the x6 kernel
    (the cfg-2 question-token dX / GloVe-row gradient shapes); results to fp32 accuracy either
    way, with an A row gather as the engine's dX launch has."""
    if "SAVQA_SK_TILES" in __import__("os").environ:
        pytest.skip("SAVQA_SK_TILES overrides the planner")
    O = ops()
    A, B = g(M + 17, K, seed=91), g(K, N, seed=92)
    idx = torch.randint(0, M + 17, (M,), generator=torch.Generator().manual_seed(93)).to(dev)
    kw = dict(lda=K, ldb=N, ldc=N, a_rows=idx, prec=6)
    assert O.gemm(A, B, None, M, N, K, plan_only=True, **kw)[0] == tile
    out = torch.empty(M, N, device=dev)
    O.gemm(A, B, out, M, N, K, **kw)
    assert rel(out, A[idx].double() @ B.double()) < 1e-5
