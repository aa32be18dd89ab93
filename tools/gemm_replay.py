#!/usr/bin/env python
"""In-step GEMM launches replayed on their own descriptors (why does the
bf16 split-K dW take 115 us inside a cfg-3 step and 77-90 us in tools/lp_bench.py?).

One probe step of the workload runs with both stacks on one stream (as bench.py's roofline
probe) under ops.GemmProbe(detail=True, keep=True): every savqa_gemm / savqa_gemm_lp launch is
timed with HIP events on its stream AND its descriptor is kept. Then, per launch shape of the
top kernels, the recorded descriptor is re-issued:
  step    -- the in-step mean per launch (events around the launch in the probe step)
  replay  -- the same descriptor (same buffers, workspace, epilogue) back to back, x iters
  fresh   -- the same descriptor with A / B pointed at new N(0, 1) bf16 / fp32 operands of
             the same extents (separates operand VALUES from layout and epilogue)
  cold    -- the descriptor issued once after a 512 MB write (L2 / MALL flushed)

Launches with row maps (gathers / scatters) are listed but never re-issued: their index
buffers may be freed temporaries after the step.

usage: python tools/gemm_replay.py [--workload cfg3] [--top 3] [--iters 20] [--grep gemm_lp]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from savqa_amd import _lib, ops  # noqa: E402
from savqa_amd.AttModel_x3 import AttModel  # noqa: E402
from savqa_amd.data import model_args, synthetic_batch  # noqa: E402
from savqa_amd.loss import smoothed_loss  # noqa: E402
from savqa_amd.optim import Adam  # noqa: E402
from savqa_amd.utils import init_params_  # noqa: E402


def build(wl, dev):
    W = bench.WORKLOADS[wl]
    B = W["batch"]
    m = AttModel(None, W["d"], W.get("hm", 1024), 914, 40, W.get("maxlen", 450), 49, 6, W["H"],
                 0.5, 0.1, 311, True, device=dev, init=False, gemm_precision=W.get("prec", "fp32"))
    init_params_(m, seed=0)
    m.train()
    opt = Adam(m, lr=1e-4)
    batch = synthetic_batch(B, Nv=W["Nv"], Ns=W["Ns"], seed=1234, device=dev)
    margs = model_args(batch)
    kw = {}
    if W.get("prec") == "fp8":
        R, Dv = B * W["Nv"], batch["vis_fea"].shape[-1]
        q8 = torch.empty(R, Dv, dtype=torch.uint8, device=dev)
        s8 = torch.empty(R, Dv // 32, dtype=torch.uint8, device=dev)
        ops.quant_fp8(batch["vis_fea"].reshape(R, Dv), R, Dv, Dv, q8, Dv, s8, Dv // 32)
        margs[0] = q8.view(torch.float8_e4m3fn).reshape(B, W["Nv"], Dv)
        kw["vis_fea_scale"] = s8.reshape(B, W["Nv"], Dv // 32)

    def step():
        lc, lv, ls, mil, mr = m(*margs, decMask=True, mcb=False, **kw)
        loss, _ = smoothed_loss(lc, lv, ls, batch["answer"], mil, with_milnce=True, mil_nce_rel=mr)
        opt.zero_grad()
        loss.backward()
        opt.step()
    return m, step


def issue(kind, d):
    s = ops._stream()
    if kind == "lp":
        _lib.call("savqa_gemm_lp", s, C.byref(d))
    else:
        _lib.call("savqa_gemm", s, C.byref(d))


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def fresh_operands(kind, d, dev, keep):
    """d with A / B at new N(0,1) buffers of the descriptor's extents (gathers keep their row
    maps: the buffers cover every row the maps can name, up to the recorded pointers' rows)."""
    d2 = type(d).from_buffer_copy(d)
    if kind == "lp":
        dt = {0: torch.float32, 1: torch.bfloat16}
        if d.a_type not in dt or d.b_type not in dt:
            return None
        ea = (d.K if d.a_trans else d.M) * d.lda + 64
        eb = (d.N if d.b_trans else d.K) * d.ldb + 64
        A = torch.randn(ea, device=dev).to(dt[d.a_type])
        Bm = torch.randn(eb, device=dev).to(dt[d.b_type])
    else:
        ea = (d.K if d.a_trans else d.M) * d.lda + 64
        eb = (d.N if d.b_trans else d.K) * d.ldb + 64
        A = torch.randn(ea, device=dev)
        Bm = torch.randn(eb, device=dev)
    keep += [A, Bm]
    d2.A, d2.B = A.data_ptr(), Bm.data_ptr()
    return d2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--top", type=int, default=2, help="kernel variants (by in-step time)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--grep", default="")
    ap.add_argument("--hints", default="",
                    help="lp weight-gradient launches (TN, no mask): also replay under these "
                         "tile_hint kernel variants, e.g. 1,3,4,5 (hot / cold)")
    ap.add_argument("--hints-all", action="store_true",
                    help="--hints on every bf16 launch (forward / dX too), not only the dW")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m, step = build(a.workload, dev)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    m._engine.concurrent = False
    probe = ops.GemmProbe(detail=True, keep=True)
    ops.set_gemm_probe(probe)
    step()
    ops.set_gemm_probe(None)
    torch.cuda.synchronize()
    per_var, per_key = {}, {}
    for (key, fl, e0, e1), (kind, d) in zip(probe.records, probe.descs):
        us = e0.elapsed_time(e1) * 1e3
        var = key.split(" | ")[0]
        per_var[var] = per_var.get(var, 0.0) + us
        r = per_key.setdefault(key, [0, 0.0, fl, kind, d])
        r[0] += 1
        r[1] += us
    tot = sum(per_var.values())
    print(f"{a.workload}: {len(probe.records)} GEMM launches, {tot / 1e3:.2f} ms in-step (serial)")
    vars_ = [v for v, _ in sorted(per_var.items(), key=lambda kv: -kv[1]) if a.grep in v][:a.top]
    flush = torch.empty(128 * 1024 * 1024, device=dev)
    keep = []
    for v in vars_:
        print(f"\n== {v}: {per_var[v] / 1e3:.2f} ms/step ({per_var[v] / tot:.1%})")
        print(f"{'shape':58s} {'n':>3s} {'step':>8s} {'replay':>8s} {'fresh':>8s} {'cold':>8s}"
              f" {'TF(step)':>9s} {'TF(rep)':>8s}")
        for key, (n, us, fl, kind, d) in sorted(per_key.items(), key=lambda kv: -kv[1][1]):
            if key.split(" | ")[0] != v:
                continue
            if d.a_rows or d.c_rows or (kind == "gemm" and d.b_rows):
                # row maps may point into temporaries freed after the step: re-issuing them
                # reads stale indices (a GPU memory fault in round 6's first run) -- never
                print(f"{key.split(' | ', 1)[1]:58s} {n:3d} {us / n:8.1f}   (row maps: not replayed)")
                continue
            rep = timed(lambda: issue(kind, d), a.iters)
            d2 = fresh_operands(kind, d, dev, keep)
            fr = timed(lambda: issue(kind, d2), a.iters) if d2 is not None else float("nan")
            cold = []
            for _ in range(3):
                flush.fill_(1.0)
                cold.append(timed(lambda: issue(kind, d), 1))
            cold = sorted(cold)[1]
            shape = key.split(" | ", 1)[1]
            print(f"{shape:58s} {n:3d} {us / n:8.1f} {rep:8.1f} {fr:8.1f} {cold:8.1f}"
                  f" {fl / (us / n) / 1e6:9.1f} {fl / rep / 1e6:8.1f}")
            if a.hints and kind == "lp" and d.a_type == 1 and not d.bits_out and \
                    not (d.mask and d.mask_type == 3) and (a.hints_all or (d.a_trans and not
                                                                          d.mask and not d.Cb)):
                for h in [int(x) for x in a.hints.split(",")]:
                    dh = type(d).from_buffer_copy(d)
                    dh.tile_hint = h
                    hot = timed(lambda: issue(kind, dh), a.iters)
                    cs = []
                    for _ in range(3):
                        flush.fill_(1.0)
                        cs.append(timed(lambda: issue(kind, dh), 1))
                    print(f"{'   tile_hint ' + str(h) + ' ' + ops.lp_variant(dh):58s} {'':3s} "
                          f"{'':8s} {hot:8.1f} {'':8s} {sorted(cs)[1]:8.1f}")


if __name__ == "__main__":
    main()
