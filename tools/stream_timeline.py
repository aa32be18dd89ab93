#!/usr/bin/env python
"""Two-stream timeline of one training step (what does the M = B decoder /
head chain overlap?). rocprofv3's kernel trace serialises the step's kernels, so this tool
times the step as it really runs -- both stacks on their own streams -- with a HIP event pair
around every library call on the stream it is issued to (ops.call wrapped), all relative to one
start event. Reported: each stream's busy time, the time both stack streams are busy, and for
each kernel family the fraction of its time during which the OTHER stack stream was busy too.
The raw intervals go to a CSV (stream, call, kernel, start_us, end_us).

usage: python tools/stream_timeline.py [--workload cfg3] [--csv out.csv]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from savqa_amd import ops  # noqa: E402
from gemm_replay import build  # noqa: E402

SKIP = ("_plan", "_bytes", "_elems", "_supported", "savqa_last_error", "savqa_version")


def family(name, args):
    """kernel family of a library call (GEMM calls by the kernel their plan picks)"""
    try:
        if name == "savqa_gemm":
            return ops.GemmProbe.variant(args[1]._obj).split("<")[0]
        if name == "savqa_gemm_lp":
            return ops.lp_variant(args[1]._obj).split("<")[0]
    except Exception:  # noqa: BLE001 -- a label only
        pass
    return name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--csv", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m, step = build(a.workload, dev)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    orig = ops.call
    recs = []

    def timed_call(name, *args):
        if name.endswith(SKIP):
            return orig(name, *args)
        s = torch.cuda.current_stream()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        rc = orig(name, *args)
        e1.record(s)
        recs.append((s.cuda_stream, name, family(name, args), e0, e1))
        return rc

    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    ops.call = timed_call
    try:
        start.record()
        step()
        end.record()
    finally:
        ops.call = orig
    torch.cuda.synchronize()
    wall = start.elapsed_time(end) * 1e3
    rows = [(st, nm, fam, start.elapsed_time(e0) * 1e3, start.elapsed_time(e1) * 1e3)
            for st, nm, fam, e0, e1 in recs]
    main_stream = torch.cuda.current_stream().cuda_stream
    streams = sorted({r[0] for r in rows}, key=lambda x: min(r[3] for r in rows if r[0] == x))
    label = {}
    k = 0
    for st in streams:
        if st == main_stream:
            label[st] = "main"
        else:
            label[st] = f"side{k}"
            k += 1

    def merged(iv):
        out = []
        for s0, s1 in sorted(iv):
            if out and s0 <= out[-1][1]:
                out[-1][1] = max(out[-1][1], s1)
            else:
                out.append([s0, s1])
        return out

    busy = {st: merged([(r[3], r[4]) for r in rows if r[0] == st]) for st in streams}

    def length(iv):
        return sum(b - a for a, b in iv)

    def intersect(x, y):
        out, i, j = [], 0, 0
        while i < len(x) and j < len(y):
            lo, hi = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
            if lo < hi:
                out.append([lo, hi])
            if x[i][1] < y[j][1]:
                i += 1
            else:
                j += 1
        return out

    print(f"{a.workload}: one step {wall / 1e3:.2f} ms wall (events), {len(rows)} library calls")
    for st in streams:
        print(f"  stream {label[st]:6s}: {len([r for r in rows if r[0] == st]):4d} calls, busy "
              f"{length(busy[st]) / 1e3:7.2f} ms")
    sides = [st for st in streams if st != main_stream]
    if len(sides) >= 2:
        both = intersect(busy[sides[0]], busy[sides[1]])
        print(f"  both stack streams busy: {length(both) / 1e3:.2f} ms")
    fam_t = collections.defaultdict(float)
    fam_ov = collections.defaultdict(float)
    for st, nm, fam, t0, t1 in rows:
        others = merged([iv for o in sides if o != st for iv in busy[o]]) if st in sides else []
        fam_t[(label[st], fam)] += t1 - t0
        fam_ov[(label[st], fam)] += length(intersect([[t0, t1]], others))
    print(f"\n{'stream':7s} {'kernel family':34s} {'ms':>7s} {'overlapped by the other stack':>30s}")
    for key, t in sorted(fam_t.items(), key=lambda kv: -kv[1])[:25]:
        print(f"{key[0]:7s} {key[1]:34s} {t / 1e3:7.2f} {fam_ov[key] / max(t, 1e-9):29.0%}")
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("stream,call,kernel,start_us,end_us\n")
            for st, nm, fam, t0, t1 in rows:
                f.write(f"{label[st]},{nm},{fam},{t0:.1f},{t1:.1f}\n")


if __name__ == "__main__":
    main()
