#!/usr/bin/env python
"""Summarise a round's rocprofv3 runs of bench.py into profiles/.

usage: summarize_prof.py TRACE_DIR PMC_FETCH_DIR PMC_WRITE_DIR OUT_PREFIX LAUNCHES_PER_STEP_JSON

* TRACE_DIR: `rocprofv3 --kernel-trace --stats` of `python bench.py ...` (the judged command).
  Copies its kernel stats and adds the per-kernel average over the LAST 2 steps' launches of
  each GEMM variant (bench.py's roofline probe runs 2 serial steps at the end).
* PMC_*_DIR: separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes of the same command.
  HBM bytes per launch = 2 x FETCH_SIZE (gfx950 reports half the bytes of wide coalesced
  reads, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, both in KB -> bytes.
"""
import collections
import csv
import json
import os
import re
import shutil
import sys


def norm(name):
    """'void savqa::gemm_f32_kernel<128, 128, 16, false, true>(...)' -> 'gemm_f32_kernel<128,128,false,true>';
    non-template kernels by their own name ('savqa::gattn_fwd_flash_kernel(savqa::AttnArgsT<...>'
    -> 'gattn_fwd_flash_kernel', not the argument type's template)."""
    m = re.match(r"(?:void )?savqa::(\w+)(?:<([^(]*)>)?\(", name)
    if not m:
        m2 = re.search(r"savqa::(\w+)\(", name)
        return m2.group(1) if m2 else name[:60]
    if m.group(2) is None:
        return m.group(1)
    args = [a.strip() for a in m.group(2).split(",")]
    if m.group(1) == "gemm_f32_kernel" and len(args) == 5:
        args = args[:2] + args[3:]  # drop BK
    return f"{m.group(1)}<{','.join(args)}>"


def read_trace(d):
    rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def pmc_means(d, counter):
    path = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(path):
        return {}
    acc = collections.defaultdict(list)
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        per[r["Dispatch_Id"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = norm(r["Kernel_Name"])
    for k, v in per.items():
        acc[names[k]].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    trace_dir, fetch_dir, write_dir, out_prefix, lps_json = sys.argv[1:6]
    lps = json.loads(lps_json)  # {"gemm_f32_kernel<128,128,false,true>": 47, ...}
    shutil.copy(os.path.join(trace_dir, "run_kernel_stats.csv"), out_prefix + "_kernel_stats.csv")
    rows = read_trace(trace_dir)
    by = collections.defaultdict(list)
    for r in rows:
        by[norm(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    probe = {}
    for k, n in lps.items():
        durs = by.get(k, [])
        tail = durs[-2 * n:] if len(durs) >= 2 * n else durs
        if tail:
            probe[k] = {"launches": len(tail), "avg_us": sum(tail) / len(tail),
                        "all_launches_avg_us": sum(durs) / len(durs)}
    fetch = pmc_means(fetch_dir, "FETCH_SIZE")
    write = pmc_means(write_dir, "WRITE_SIZE")
    traffic = {}
    for k in set(fetch) | set(write):
        if k in fetch and k in write:
            traffic[k] = {"fetch_kb_raw": fetch[k], "write_kb": write[k],
                          "hbm_bytes_per_launch": (2.0 * fetch[k] + write[k]) * 1024.0}
    out = {"probe_window": probe, "traffic": traffic,
           "note": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) KB per dispatch, mean over the "
                   "kernel's dispatches in separate --pmc passes of the same bench command"}
    json.dump(out, open(out_prefix + "_roofline.json", "w"), indent=1, sort_keys=True)
    print(json.dumps(probe, indent=1))


if __name__ == "__main__":
    main()
