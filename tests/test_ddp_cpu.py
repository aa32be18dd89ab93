"""Data-parallel gradient exchange (savqa_amd.ddp.GradReducer) with world_size 2 on the
gloo backend (CPU): ranged, bucketed, asynchronous all-reduce of the flat gradient arena
and the 1/world factor folded into Adam -- i.e. what DDP's all-reduce does (main:203)."""
import os
import socket
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from savqa_amd.ddp import GradReducer
    n = 10007
    g = torch.arange(n, dtype=torch.float32) * (rank + 1)
    arena = types.SimpleNamespace(grad=g.clone())
    red = GradReducer(arena, bucket_mb=0.01)  # 2621 floats per bucket
    red.begin()
    red.reduce_range(0, 3000, True)     # "heads" phase (flushed)
    # "visual stack", declared layer by layer: coalesced into full buckets
    for lo in range(3000, 7000, 500):
        red.reduce_range(lo, lo + 500)
    red.reduce_range(7000, 7000, True)  # empty declaration that only flushes
    red.reduce_range(7000, 9000)        # "semantic stack": remainder left pending ...
    red.reduce_range(9000, n)           # ... and extended
    works, scale = red.drain()          # drain flushes what is pending
    spans = [(lo, hi) for _, lo, hi in works]
    for w, _, _ in works:
        w.wait()
    expect = torch.arange(n, dtype=torch.float32) * sum(r + 1 for r in range(world))
    # finish() on an empty reducer is a no-op returning the 1/world factor
    q.put((rank, float((arena.grad - expect).abs().max()), scale, spans, red.finish()))
    dist.destroy_process_group()


def test_grad_reducer_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, scale, spans, scale2 in res:
        assert err == 0.0
        assert scale == 0.5 and scale2 == 0.5
        # buckets tile [0, n) exactly, none larger than the bucket size
        assert spans[0] == (0, 2621) and spans[1] == (2621, 3000)
        pos = 0
        for lo, hi in sorted(spans):
            assert lo == pos and 0 < hi - lo <= 2621
            pos = hi
        assert pos == 10007
        assert spans[2] == (3000, 5621)   # full bucket issued during the layer loop


def _sparse_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from savqa_amd.ddp import GradReducer
    width, rows = 7, 50
    t0, t1 = 1000, 1000 + width * rows            # a row table inside the arena
    u0, u1 = t1 + 13, t1 + 13 + width * rows       # a second one (same ids), 13 floats later
    n = u1 + 777
    gen = torch.Generator().manual_seed(rank)
    ids = torch.randint(0, rows, (3, 6), generator=gen)  # duplicates within and across ranks
    ids[0, 0] = rows - 1                           # last row touched by every rank
    g = torch.randn(n, generator=gen)
    for a0, a1 in ((t0, t1), (u0, u1)):
        table = torch.zeros(rows, width)
        table.index_add_(0, ids.reshape(-1), torch.randn(ids.numel(), width, generator=gen))
        g[a0:a1] = table.reshape(-1)               # untouched rows are zero, as in the model
    dense = g.clone()
    dist.all_reduce(dense)
    arena = types.SimpleNamespace(grad=g.clone())
    red = GradReducer(arena, bucket_mb=0.001)      # 262 floats per bucket: the table spans several
    red.add_sparse_table(u0, u1, width)            # registration order does not matter
    red.add_sparse_table(t0, t1, width)
    red.begin()
    red.set_rows(ids)
    red.reduce_range(0, 600, True)
    red.prepare_rows()
    red.reduce_range(600, 1100)                    # declarations split the table ...
    red.reduce_range(1100, u1 + 5)                 # ... and complete both
    red.reduce_range(u1 + 5, n, True)
    works, scale = red.drain()
    assert red.rows_exchanged == 2
    spans = sorted((lo, hi) for _, lo, hi in works)
    for w, _, _ in works:
        w.wait()
    q.put((rank, float((arena.grad - dense).abs().max()), spans, scale, n, (u0, u1),
           list(red.trace)))
    dist.destroy_process_group()


def test_sparse_table_rows_exchange_equals_dense_gloo_world2():
    """Row-sparse exchange of a table range (GradReducer.add_sparse_table / set_rows):
    after wait() the arena equals the dense all-reduce, and the spans still tile [0, n)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sparse_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # RCCL needs every rank to issue the same collectives in the same order
    assert res[0][6] == res[1][6] and len(res[0][6]) > 3, (res[0][6], res[1][6])
    assert [k for k, _, _ in res[0][6]].count("rows") == 2
    for rank, err, spans, scale, n, tab2, _ in res:
        assert err < 1e-6
        assert scale == 0.5
        assert (1000, 1350) in spans and tab2 in spans
        pos = 0
        for lo, hi in spans:
            assert lo == pos and hi > lo
            pos = hi
        assert pos == n


def _ragged_worker(rank, world, port, q, static_cap=False):
    """Ranks with different question lengths (the collate pads to each batch's own longest
    question), two forwards before one backward, and declarations that leave a gap.
    static_cap: the lists are padded to a bound every rank knows (no host count exchange)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from savqa_amd.ddp import GradReducer
    from savqa_amd.optim import Adam
    width, rows = 5, 40
    t0, t1 = 300, 300 + width * rows
    n = t1 + 400
    gen = torch.Generator().manual_seed(10 + rank)
    ids_a = torch.randint(0, rows, (3, 4 + 5 * rank), generator=gen)   # Lq 4 vs 9
    ids_b = torch.randint(0, rows, (2, 7 - 3 * rank), generator=gen)   # Lq 7 vs 4
    g = torch.randn(n, generator=gen)
    table = torch.zeros(rows, width)
    for ids in (ids_a, ids_b):
        table.index_add_(0, ids.reshape(-1), torch.randn(ids.numel(), width, generator=gen))
    g[t0:t1] = table.reshape(-1)
    dense = g.clone()
    dist.all_reduce(dense)
    arena = types.SimpleNamespace(grad=g.clone())
    red = GradReducer(arena, bucket_mb=0.001, filler=rows - 1)
    red.add_sparse_table(t0, t1, width)
    red.begin()
    if static_cap:
        red.meta = None                 # no host metadata group: a count exchange would fail
        red.set_rows(ids_a, cap=3 * 10)
        red.set_rows(ids_b, cap=2 * 8)  # second forward: its rows join the union
        try:
            red.set_rows(ids_a, cap=4)
            raise AssertionError("ids beyond the cap must raise")
        except ValueError:
            pass
    else:
        red.set_rows(ids_a)
        red.set_rows(ids_b)             # second forward: its rows join the union
    red.reduce_range(0, 100, True)
    red.reduce_range(250, n, True)      # [100, 250) never declared
    works, scale = red.drain()
    works = works + Adam._coverage_gaps(red, works, n)
    for w, _, _ in works:
        w.wait()
    q.put((rank, float((arena.grad - dense).abs().max()),
           sorted((lo, hi) for _, lo, hi in works), list(red.trace)))
    dist.destroy_process_group()


@pytest.mark.parametrize("static_cap", [False, True])
def test_ragged_rows_accumulated_forwards_and_coverage_gap_gloo_world2(static_cap):
    """ragged q_ipt across ranks must not desynchronise the id all-gather; rows of
    every forward since begin() are exchanged; an undeclared span is all-reduced densely
    before Adam instead of being updated with the local gradient. static_cap: the
    per-forward host count exchange is replaced by padding to a bound every rank shares."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ragged_worker, args=(r, 2, port, q, static_cap))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][3] == res[1][3], (res[0][3], res[1][3])  # same collective sequence
    for rank, err, spans, _ in res:
        assert err < 1e-6, (rank, err)
        assert (100, 250) in spans
        pos = 0
        for lo, hi in spans:
            assert lo == pos
            pos = hi


def test_adam_grad_scale_matches_mean_of_grads():
    """Adam(grad_scale=1/world) on summed grads == Adam on the mean (oracle restatement)."""
    from oracle import savqa_oracle as O
    g1, g2 = torch.randn(50), torch.randn(50)
    p0 = torch.randn(50)
    P = {"w": p0.clone()}
    O.adam_step(P, {"w": (g1 + g2) / 2}, {}, 1)
    # the fused kernel computes g' = g*grad_scale first; restate that order
    P2 = {"w": p0.clone()}
    O.adam_step(P2, {"w": (g1 + g2) * 0.5}, {}, 1)
    assert torch.allclose(P["w"], P2["w"])


def _metrics_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from savqa_amd.train import gather_metrics
    vals = [(0.5 + rank, 3.0 + rank, 8.0), (2.0, 1.0 + 2 * rank, 4.0 + rank)]
    q.put((rank, [gather_metrics(v, world, torch.device("cpu")) for v in vals], vals))
    dist.destroy_process_group()


def test_epoch_metric_gather_matches_reference_gloo_world2():
    """main:383-404 (3-float all_gather, loss mean over ranks, counts summed) for both the
    validation and the train-split metrics, against the oracle's restatement."""
    from oracle import savqa_oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_metrics_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in range(2):
        ref = O.gather_epoch_metrics([res[r][2][k] for r in range(2)])
        for rank in range(2):
            got = res[rank][1][k]
            assert all(abs(a - b) < 1e-6 for a, b in zip(got, ref)), (got, ref)
