"""Data-parallel gradient exchange for the flat arena (replaces DDP, main:203/:363).

The reference wraps the model in DistributedDataParallel(find_unused_parameters=True),
which all-reduces all 1.14B registered parameters every step (681.9M of them unused
and zero-filled). Here only the live range of the flat gradient arena is exchanged
(457M floats), as contiguous buckets, with RCCL (torch.distributed "nccl" = RCCL on
ROCm) over xGMI:

  * the arena groups live parameters by the backward phase that FINISHES them, so the
    engine reports final contiguous ranges (heads; visual stack; semantic stack +
    MIL-NCE) on the stream that produced them;
  * every finished bucket is all-reduced asynchronously right away: RCCL's stream
    waits for the kernels that produced it and then runs beside the rest of the
    backward (overlap), exactly the dependency, nothing more;
  * the 1/world average is folded into the Adam kernel (Adam.grad_scale), so no
    extra pass over 1.8 GB of gradients;
  * row tables whose gradient rows are known from the inputs (the two stacks' 407000x300
    syb_emb tables: only the question-token rows, AttModel_x3.py:96-99 / :216-219, get a
    gradient) are exchanged by rows instead of densely (SURVEY 8(e) "exchange only the
    touched rows"): the token ids are all-gathered in the forward (padded to a static cap
    with a filler row, so no host exchange); at the table's turn in the backward every rank
    sends ITS OWN rows once -- its id list sorted, duplicates zeroed -- by an all-gather of
    [cap, 300], and every rank then sums the rows of each id over the ranks in rank order
    (an index_add per rank: at most one non-zero row per id and rank, so the sums are the
    same bits on every rank) into the table before Adam. Rows nobody touched stay zero, so
    the result equals the dense all-reduce; an all-gather of cap rows moves half the bytes of
    an all-reduce of the world*cap-row union (ring: (N-1)*cap vs 2(N-1)*cap rows per rank).
Works with any torch.distributed backend (gloo on CPU tensors for the host tests).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


class _RowsWork:
    """Work handle of a row-sparse table exchange: wait() makes the current stream wait for
    the all-gather of every rank's compact rows, then writes their per-id sums into the table
    (zero the union's rows, then one index_add per rank in rank order)."""

    def __init__(self, work, table, union, ids, outs):
        self.work, self.table, self.union, self.ids, self.outs = work, table, union, ids, outs

    def wait(self):
        self.work.wait()
        self.table.index_fill_(0, self.union, 0.0)
        for r, rows in enumerate(self.outs):
            self.table.index_add_(0, self.ids[r], rows)
        return True


class GradReducer:
    """Bucketed, streamed all-reduce of the live gradient range of a ParamArena.

    reduce_range(lo, hi) declares arena gradient elements [lo, hi) final on the CURRENT
    stream. Contiguous declarations from one stream are coalesced, and every full bucket
    (bucket_mb) is all-reduced asynchronously at once; flush=True (end of a backward
    phase) also sends the remainder. drain() returns the (work, lo, hi) list so the
    optimizer can update each bucket as soon as ITS all-reduce lands (Adam of the early
    buckets overlaps the all-reduce of the last ones)."""

    # collective timing of diagnostic steps (time_collectives): off by default
    stats = None
    _comm = None
    _bwd_end = None

    def __init__(self, arena, bucket_mb: float = 64.0, group=None, filler: int = 400000,
                 force: bool = False):
        self.arena = arena
        self.group = group
        # padding row of the static-cap set_rows lists (any row of every sparse table; the
        # default is the PAD token's row, AttModel_x3.py:13)
        self.filler = int(filler)
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # active: the exchange runs (world > 1; `force` runs every collective at world 1 too --
        # the single-GPU RCCL test of the streamed path)
        self.active = self.world > 1 or bool(force)
        # host-side metadata exchange (the per-rank id counts of set_rows without a static
        # cap): a gloo group on CPU tensors, so agreeing on a size never synchronises a GPU
        # stream. Created here, where every rank constructs its reducer (new_group is
        # collective).
        self.meta = None
        if self.active:
            self.meta = group if dist.get_backend(group) == "gloo" else dist.new_group(
                ranks=None if group is None else dist.get_process_group_ranks(group),
                backend="gloo")
        self.bucket = max(1, int(bucket_mb * (1 << 20) // 4))
        self.works: List = []
        self.pending = {}
        self.sparse: List = []      # [(lo, hi, width)] arena ranges exchanged by rows
        self._ids = None            # (all_gather work, [world] id tensors) of this step
        self._rows = None           # (union ids, per-rank sorted ids, this rank's first mask)
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        # every collective this reducer issued since begin(), in issue order: (kind, lo, hi)
        # -- RCCL needs the same sequence on every rank (tests compare it across ranks)
        self.trace: List = []
        self._rows_done = set()     # arena offsets of the tables exchanged by rows this step
        self.rows_exchanged = 0     # tables exchanged by rows in the current step
        # collective timing (diagnostic steps only, bench.py's N > 1 "comm" report): None = off;
        # a list = every collective of the step issued from a side stream bracketed by HIP
        # events, [(kind, bytes, e_start, e_landed)], plus the end of the backward
        self.stats = None
        self._comm = None
        self._bwd_end = None

    def add_sparse_table(self, lo: int, hi: int, width: int):
        """Exchange arena range [lo, hi) (a row-major table of `width`-wide rows) by the
        rows set_rows() names instead of densely."""
        assert (hi - lo) % width == 0
        self.sparse.append((int(lo), int(hi), int(width)))
        self.sparse.sort()

    def rows_tracked(self, offset: int) -> bool:
        """Whether the table starting at arena `offset` is exchanged by rows (its touched-row
        flags then get the union of every rank's ids, so Adam may update it row by row)."""
        return self.active and offset in self._rows_done

    def time_collectives(self, on: bool = True):
        """Diagnostic mode for the next steps: each collective is issued from a side stream
        that first waits for the producing stream, with an event before the issue and one
        after the collective has landed (the side stream waits for it), so comm_summary() can
        report the exchange's busy time, how much of it outlasted the backward, and the
        bytes. Off (None) in timed steps: the normal path issues on the producer stream."""
        self.stats = [] if on else None

    def _timed(self, kind: str, nbytes: int, issue):
        if self.stats is None or not torch.cuda.is_available():
            return issue()
        cur = torch.cuda.current_stream()
        if self._comm is None or self._comm.device != cur.device:
            self._comm = torch.cuda.Stream(device=cur.device)
        s = self._comm
        s.wait_stream(cur)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            e0.record(s)
            w = issue()
            w.wait()
            e1.record(s)
        self.stats.append((kind, int(nbytes), e0, e1))
        return w

    def comm_summary(self):
        """Of the last step run with time_collectives(): collectives issued, the sum of
        their durations (each starts once its data is final and the previous one has
        landed), the part of the exchange that ended after the backward did (exposed), and
        bytes per kind (dense all-reduce buffers; row all-gather outputs)."""
        if not self.stats:
            return None
        torch.cuda.synchronize()
        busy = sum(e0.elapsed_time(e1) for _, _, e0, e1 in self.stats)
        exposed = None
        if self._bwd_end is not None:
            exposed = max(0.0, max(self._bwd_end.elapsed_time(e1) for *_, e1 in self.stats))
        by = {}
        for kind, nb, _, _ in self.stats:
            by[kind] = by.get(kind, 0) + nb
        out = {"collectives": len(self.stats), "allreduce_ms": round(busy, 3),
               "exposed_ms": None if exposed is None else round(exposed, 3),
               "dense_MB": round(by.get("dense", 0) / 2 ** 20, 2),
               "rows_MB": round(by.get("rows", 0) / 2 ** 20, 2),
               "rows_tables": sum(1 for k, *_ in self.stats if k == "rows")}
        return out

    def begin(self):
        self._bwd_end = None
        if self.stats is not None:
            self.stats = []
        self._rows_done = set()
        self.works = []
        self.pending = {}
        self._ids = None
        self._rows = None
        self.rows_exchanged = 0
        self.trace = []

    def set_rows(self, ids: torch.Tensor, cap: Optional[int] = None):
        """This step's touched rows of the sparse tables (any integer tensor): all-gathered
        now, async, while the forward runs. Ranks may hold different numbers of ids (the
        collate pads questions to each batch's own longest one, and drops bad samples, so
        q_ipt is ragged across ranks); every rank pads its list to one common length:
          * cap given (the static bound every rank shares, e.g. batch_size * maxlen_q: see
            AttModel.attach_reducer): padded to `cap` with the fixed filler row (ctor) -- no
            host exchange at all. A filler row nobody touched has a zero gradient on every
            rank, so exchanging it changes nothing. More than `cap` ids raise.
          * cap None: the counts are agreed on the host first (gloo, no GPU synchronisation,
            but one host rendezvous of the ranks per call) and the lists padded to the largest.
        Duplicates are exchanged once. Several calls before the backward (e.g. several
        forwards) accumulate: the union of their rows is exchanged."""
        if not self.active or not self.sparse:
            return
        ids = ids.reshape(-1).to(torch.int64).contiguous()
        n = ids.numel()
        if cap is not None:
            cap = int(cap)
            if n > cap:
                raise ValueError(f"GradReducer.set_rows: {n} row ids exceed the static cap {cap} "
                                 "(batch_size * maxlen_q); raise maxlen_q")
        else:
            cnt = [torch.zeros(1, dtype=torch.int64) for _ in range(self.world)]
            dist.all_gather(cnt, torch.tensor([n], dtype=torch.int64), group=self.meta)
            cap = max(int(c) for c in cnt)
        if cap == 0:
            return
        if n < cap:
            fill = torch.full((1,), self.filler, dtype=torch.int64, device=ids.device)
            ids = torch.cat([ids, fill.expand(cap - n)])
        outs = [torch.empty_like(ids) for _ in range(self.world)]
        w = dist.all_gather(outs, ids, group=self.group, async_op=True)
        self.trace.append(("ids", 0, cap))
        if self._ids is None or self._rows is not None:
            self._ids = []
        self._ids.append((w, outs))
        self._rows = None

    def prepare_rows(self):
        """Sort the gathered ids (on the current stream; call at the start of the
        backward, when the all-gather has long landed): every rank's own list sorted (the
        order its rows travel in; the same computation on every rank), this rank's
        first-occurrence mask (duplicates send zero rows), and the union for the write-back
        and the Adam row flags."""
        if self._ids is None or self._rows is not None:
            return
        per = [[] for _ in range(self.world)]
        for w, o in self._ids:
            w.wait()
            for r in range(self.world):
                per[r].append(o[r])
        ids = [torch.sort(torch.cat(p)).values for p in per]
        mine = ids[self.rank]
        first = torch.ones_like(mine, dtype=torch.bool)
        first[1:] = mine[1:] != mine[:-1]
        self._rows = (torch.cat(ids), ids, first)

    @staticmethod
    def _stream_key():
        return torch.cuda.current_stream().cuda_stream if torch.cuda.is_available() else 0

    def _dense(self, lo: int, hi: int):
        g = self.arena.grad
        w = self._timed("dense", (hi - lo) * g.element_size(), lambda: dist.all_reduce(
            g[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        self.works.append((w, lo, hi))
        self.trace.append(("dense", lo, hi))

    def _issue(self, lo: int, hi: int):
        # final range [lo, hi): dense pieces around the sparse tables; a table goes out
        # (by rows) once the range that completes it is declared (declarations are
        # monotone per stream and a table is produced on one stream)
        for t0, t1, width in self.sparse:
            if hi <= t0 or lo >= t1:
                continue
            if lo < t0:
                self._dense(lo, t0)
            if hi >= t1:
                self._sparse(t0, t1, width)
            lo = min(hi, t1)
        if hi > lo:
            self._dense(lo, hi)

    def _sparse(self, t0: int, t1: int, width: int):
        self.prepare_rows()
        if self._rows is None:       # no set_rows() this step: dense exchange
            self._dense(t0, t1)
            return
        union, ids, first = self._rows
        table = self.arena.grad[t0:t1].view(-1, width)
        mark = getattr(self.arena, "mark_table_rows", None)
        if mark is not None:  # rows other ranks touched get a gradient here too
            mark(t0, union)
        self._rows_done.add(t0)
        buf = table.index_select(0, ids[self.rank])
        buf.mul_(first.unsqueeze(1).to(buf.dtype))
        outs = [torch.empty_like(buf) for _ in range(self.world)]
        w = self._timed("rows", buf.numel() * buf.element_size() * self.world,
                        lambda: dist.all_gather(outs, buf, group=self.group, async_op=True))
        self.works.append((_RowsWork(w, table, union, ids, outs), t0, t1))
        self.trace.append(("rows", t0, t1))
        self.rows_exchanged += 1

    def reduce_range(self, start: int, end: int, flush: bool = False):
        if not self.active:
            return
        end = min(int(end), self.arena.grad.numel())
        start = int(start)
        key = self._stream_key()
        lo, hi = self.pending.get(key, (start, start))
        if hi != start:          # not contiguous with this stream's pending range
            if hi > lo:
                self._issue(lo, hi)
            lo = start
        hi = max(end, start)
        while hi - lo >= self.bucket:
            self._issue(lo, lo + self.bucket)
            lo += self.bucket
        if flush and hi > lo:
            self._issue(lo, hi)
            lo = hi
        self.pending[key] = (lo, hi)

    def _flush_all(self):
        # called on the stream that joined every producer stream (engine.backward ends
        # with main.wait_stream(...)), so the remainders are final there as well
        for lo, hi in self.pending.values():
            if hi > lo:
                self._issue(lo, hi)
        self.pending = {}

    def drain(self):
        """Issue what is pending; return ([(work, lo, hi)...] in issue order, 1/world)."""
        if not self.active:
            return [], 1.0
        if self.stats is not None and torch.cuda.is_available():
            # the backward has been issued on this stream: its end, for comm_summary()
            self._bwd_end = torch.cuda.Event(enable_timing=True)
            self._bwd_end.record()
        self._flush_all()
        works, self.works = self.works, []
        return works, 1.0 / self.world

    def finish(self):
        """Make the current stream wait for every bucket; returns the 1/world factor the
        optimizer folds into its update (DDP averages)."""
        works, scale = self.drain()
        for w, _, _ in works:
            w.wait()
        return scale
