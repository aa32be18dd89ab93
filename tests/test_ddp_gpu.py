"""The engine's streamed gradient declarations (per layer, per backward phase) tile the
live range of the arena, and the per-bucket Adam (opt.step(reducer=...)) equals one
Adam launch over the whole range -- on one GPU, with a recording stand-in for the
all-reduce (world=2 semantics without a second rank; RCCL itself is exercised by
bench.py --gpus N and the gloo tests)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Done:
    def wait(self):
        pass


def _model():
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.utils import init_params_
    m = AttModel(None, 256, 64, 12, 16, 60, 10, 2, 4, 0.5, 0.0, 2, True, device="cuda",
                 init=False)
    init_params_(m, seed=3)
    m.train()
    return m


def test_streamed_ranges_tile_live_range_and_bucketed_adam_matches():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from savqa_amd.data import model_args, synthetic_batch
    from savqa_amd.ddp import GradReducer
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam

    class Recorder(GradReducer):
        def __init__(self, arena):
            self.arena, self.group, self.world = arena, None, 2
            self.bucket = 1 << 18
            self.works, self.pending, self.log = [], {}, []
            self.sparse, self._ids, self._rows = [], None, None

        def add_sparse_table(self, lo, hi, width):   # dense tiling only (no 2nd rank)
            pass

        def _issue(self, lo, hi):
            self.log.append((lo, hi))
            self.works.append((_Done(), lo, hi))

    m = _model()
    batch = synthetic_batch(4, Nv=6, Lq=5, Ns=8, topN=5, num_classes=12, seed=5, device="cuda")
    red = Recorder(m._arena)
    m.attach_reducer(red)
    opt = Adam(m, lr=1e-3)
    lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
    loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
    opt.zero_grad()
    red.begin()
    loss.backward()
    a = m._arena
    p0 = a.flat[:a.n_live].clone()
    opt.step(reducer=red)
    spans = sorted(red.log)
    pos = 0
    for lo, hi in spans:
        assert lo == pos and hi > lo
        pos = hi
    assert pos == a.n_live
    assert len(spans) > 8  # streamed layer by layer, not one range per stack
    bucketed = a.flat[:a.n_live].clone()
    # same gradients, one launch over the live range with the same 1/world factor
    a.flat[:a.n_live].copy_(p0)
    opt.m.zero_()
    opt.v.zero_()
    opt.step_count = 0
    opt.grad_scale = 0.5
    opt.step()
    torch.cuda.synchronize()
    assert torch.equal(a.flat[:a.n_live], bucketed)
    assert not torch.equal(bucketed, p0)


def _rows_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from savqa_amd.data import model_args, synthetic_batch
        from savqa_amd.ddp import GradReducer
        from savqa_amd.loss import smoothed_loss
        from savqa_amd.optim import Adam
        batch = synthetic_batch(4, Nv=6, Lq=5, Ns=8, topN=5, num_classes=12, seed=5 + rank,
                                device="cuda")
        out = []
        for sparse in (True, False):
            m = _model()
            red = GradReducer(m._arena, bucket_mb=1.0)
            m.attach_reducer(red)
            if not sparse:
                red.sparse = []          # every range dense: DDP's exchange
            opt = Adam(m, lr=1e-3)
            for step in range(2):
                torch.manual_seed(100 + step)
                red.begin()
                lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
                loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
                opt.zero_grad()
                loss.backward()
                assert red.rows_exchanged == (2 if sparse else 0)
                opt.step(reducer=red)
            torch.cuda.synchronize()
            out.append(m._arena.flat[:m._arena.n_live].cpu())
        q.put((rank, float((out[0] - out[1]).abs().max()), float((out[0] - out[1]).abs().sum()),
               None))
    except Exception as e:  # report instead of leaving the parent waiting
        import traceback
        q.put((rank, float("nan"), 0.0, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_rows_exchange_of_stack_tables_matches_dense_two_ranks():
    """Two ranks (gloo on the same HIP device) train 2 steps with the stack tables'
    row-sparse exchange and with the dense exchange: identical parameters."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rows_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, tot, exc in res:
        assert exc is None, exc
        assert err <= 1e-7, (rank, err, tot)


# ---------------------------------------------------------------- 1 rank on B == 2 ranks on B/2
def _equiv_model():
    from savqa_amd.AttModel_x3 import AttModel
    from savqa_amd.utils import init_params_
    m = AttModel(None, 256, 64, 12, 16, 60, 10, 2, 4, 0.0, 0.0, 2, True, device="cuda",
                 init=False)
    init_params_(m, seed=3)
    m.train()
    return m


def _equiv_batch():
    from savqa_amd.data import synthetic_batch
    return synthetic_batch(8, Nv=6, Lq=5, Ns=8, topN=5, num_classes=12, seed=41, device="cuda")


def _digest(arena, t):
    """Per live parameter: the tensor (cpu), or for the 407000-row tables the rows that hold
    a non-zero gradient (touched rows) -- keeps the message small."""
    out = {}
    g = arena.grad
    for n in arena.live_names:
        o, shp = arena.offsets[n]
        v = t[o:o + shp.numel()].view(shp)
        if shp.numel() > (1 << 22):
            rows = g[o:o + shp.numel()].view(shp).abs().sum(1).nonzero().reshape(-1)
            out[n] = (rows.cpu(), v.index_select(0, rows).cpu())
        else:
            out[n] = v.detach().cpu().clone()
    return out


def _equiv_run(world, rank, steps=2, sparse=True):
    """`steps` full training steps (forward, loss, backward, streamed GradReducer, per-bucket
    Adam) on this rank's contiguous shard of the 8-sample batch; returns per step the
    gradient Adam consumed (summed / world) and the parameters after the step."""
    from savqa_amd.data import model_args
    from savqa_amd.ddp import GradReducer
    from savqa_amd.loss import smoothed_loss
    from savqa_amd.optim import Adam
    m = _equiv_model()
    full = _equiv_batch()
    n = 8 // world
    batch = {k: v[rank * n:(rank + 1) * n] for k, v in full.items()}
    red = None
    if world > 1:
        red = GradReducer(m._arena, bucket_mb=1.0)
        m.attach_reducer(red)      # multi_rank: the gated enc4 backward schedule is on
        assert m._engine.vis_gate() is not None
        if not sparse:
            red.sparse = []
    opt = Adam(m, lr=1e-4)
    a = m._arena
    rec = []
    for _ in range(steps):
        if red:
            red.begin()
        lc, lv, ls, mil, _ = m(*model_args(batch), decMask=True, mcb=False)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil)
        opt.zero_grad()
        loss.backward()
        opt.step(reducer=red)
        torch.cuda.synchronize()
        g = a.grad[:a.n_live] / world
        rec.append((_digest(a, g), _digest(a, a.flat[:a.n_live])))
    return rec


def _equiv_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {s: _equiv_run(world, rank, sparse=s) for s in (True, False)}
        q.put((rank, _to_numpy(res), None))   # by value: the parent reads after we exit
    except Exception:
        import traceback
        q.put((rank, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _to_numpy(x):
    if isinstance(x, torch.Tensor):
        return x.numpy()
    if isinstance(x, dict):
        return {k: _to_numpy(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_numpy(v) for v in x)
    return x


def _to_torch(x):
    import numpy as np
    if isinstance(x, np.ndarray):
        return torch.from_numpy(x)
    if isinstance(x, dict):
        return {k: _to_torch(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_torch(v) for v in x)
    return x


def _cmp(a, b):
    """Frobenius-relative difference of two digests' entries (tables: same touched rows)."""
    if isinstance(b, tuple):
        assert torch.equal(a[0], b[0])
        a, b = a[1], b[1]
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def test_two_ranks_on_half_batches_equal_one_rank_on_the_batch():
    """SURVEY 4 / main:203,363 (DistributedDataParallel): the same global batch gives the same
    update on 1 rank and on 2 ranks with B/2 each -- 2 training steps through the full path
    (forward, loss, backward with the gated enc4 schedule, streamed bucketed all-reduce,
    per-bucket Adam), with the stack tables exchanged by rows and densely. The two replicas
    are bit-identical; against the 1-rank run, the gradient Adam consumes agrees per tensor
    to 1e-4 (Frobenius-relative: only the fp32 summation order differs) and the parameters'
    2-step updates to 1e-3 (Adam divides by sqrt(v), so near-zero gradient entries amplify
    rounding; the key-projection biases have an exactly-zero true gradient -- softmax shift
    invariance -- and their Adam update is rounding noise in every implementation, so they
    are left out)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import socket
    import torch.multiprocessing as mp
    ref = _equiv_run(1, 0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_equiv_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = dict((r, (_to_torch(out), exc)) for r, out, exc in
                   (q.get(timeout=240) for _ in procs))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in (0, 1):
        assert res[r][1] is None, res[r][1]
    for p in procs:
        assert p.exitcode == 0
    for sparse in (True, False):
        r0, r1 = res[0][0][sparse], res[1][0][sparse]
        worst_g, worst_u = [], []
        for step in range(2):
            (g0, w0), (g1, w1) = r0[step], r1[step]
            gref, wref = ref[step]
            for n in wref:
                x0, x1 = w0[n], w1[n]
                if isinstance(x0, tuple):
                    x0, x1 = x0[1], x1[1]
                assert torch.equal(x0, x1), ("replicas diverged", sparse, step, n)
                if n.endswith("K_proj.0.bias"):
                    continue
                if not isinstance(gref[n], tuple) and float(gref[n].abs().max()) == 0.0:
                    assert float(g0[n].abs().max()) == 0.0, n
                    continue
                worst_g.append((_cmp(g0[n], gref[n]), step, n))
                if isinstance(wref[n], tuple):   # tables: gradient rows compared above
                    continue
                du = w0[n] - _start(n, step, ref)
                dr = wref[n] - _start(n, step, ref)
                worst_u.append((_cmp(du, dr), step, n))
        worst_g.sort(reverse=True)
        worst_u.sort(reverse=True)
        assert worst_g[0][0] < 1e-4, (sparse, worst_g[:4])
        assert worst_u[0][0] < 1e-3, (sparse, worst_u[:4])


def _start(n, step, ref):
    """Parameters before `step`'s update in the 1-rank run (step 0: the seeded init that
    every run starts from)."""
    return _init_params()[n] if step == 0 else ref[step - 1][1][n]


_INIT = {}


def _init_params():
    if not _INIT:
        m = _equiv_model()
        a = m._arena
        for n in a.live_names:
            o, shp = a.offsets[n]
            if shp.numel() <= (1 << 22):
                _INIT[n] = a.flat[o:o + shp.numel()].view(shp).cpu().clone()
    return _INIT
