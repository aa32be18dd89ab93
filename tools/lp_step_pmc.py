#!/usr/bin/env python
"""PMC of the bf16 split-K weight gradient (gemm_lp_kernel<true,...>) in-step vs replayed
(VERDICT r05 item 1): summarise the --pmc passes of
  rocprofv3 --pmc <counters> -- python tools/gemm_replay.py --workload cfg3 --grep 'gemm_lp_kernel<true' --top 1
The replay tool runs 3 warm-up steps and one probe step (in-step launches: the first
4 x launches_per_step dispatches of the kernel), then re-issues every launch shape back to
back (hot) and once after a 512 MB flush (cold). Per group: mean of each counter per dispatch.
usage: python tools/lp_step_pmc.py PER_STEP DIR [DIR ...]   (each DIR: one --pmc pass)"""
import collections
import csv
import glob
import sys


def load(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for r in csv.DictReader(open(f)):
        if "gemm_lp_kernel<true" not in r["Kernel_Name"]:
            continue
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] += float(r["Counter_Value"])
        name[i] = r["Kernel_Name"]
    return [per[i] for i in sorted(per)]


def main():
    n_step = int(sys.argv[1]) * 4
    for d in sys.argv[2:]:
        rows = load(d)
        groups = {"in-step (4 steps)": rows[:n_step], "replayed (hot + cold)": rows[n_step:]}
        for g, rs in groups.items():
            if not rs:
                continue
            keys = sorted(rs[0])
            means = {k: sum(r.get(k, 0.0) for r in rs) / len(rs) for k in keys}
            txt = ", ".join(f"{k} {v:.4g}" for k, v in means.items())
            extra = ""
            if "TCC_HIT_sum" in means and "TCC_MISS_sum" in means:
                extra = f"  L2 hit rate {means['TCC_HIT_sum'] / max(1.0, means['TCC_HIT_sum'] + means['TCC_MISS_sum']):.3f}"
            if "SQ_WAIT_ANY" in means and "SQ_BUSY_CYCLES" in means:
                extra += f"  wait/busy {means['SQ_WAIT_ANY'] / max(1.0, means['SQ_BUSY_CYCLES']):.3f}"
            print(f"{g:24s} n={len(rs):4d}  {txt}{extra}")


if __name__ == "__main__":
    main()
