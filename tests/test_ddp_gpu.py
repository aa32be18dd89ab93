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
