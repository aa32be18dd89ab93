#!/usr/bin/env python
"""Per-kernel averages of rocprofv3 counter CSVs (one row per kernel, one column per counter,
mean over dispatches; each counter summed over its instances within a dispatch).
usage: pmc_table.py DIR [DIR ...] [--match SUBSTR]"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"savqa::(\w+<[^>]*>)", name) or re.search(r"savqa::(\w+)", name)
    return m.group(1).replace(" ", "") if m else name[:60]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
    args = [a for a in args if a != match]
    table = collections.defaultdict(dict)
    for d in args:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(float)
            kname = {}
            for r in csv.DictReader(open(path)):
                key = (r["Dispatch_Id"], r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
                kname[r["Dispatch_Id"]] = r["Kernel_Name"]
            agg = collections.defaultdict(list)
            for (disp, ctr), v in per.items():
                if match in kname[disp]:
                    agg[(short(kname[disp]), ctr)].append(v)
            for (k, ctr), vs in agg.items():
                table[k][ctr] = sum(vs) / len(vs)
        for path in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                if match in r["Name"]:
                    table[short(r["Name"])]["avg_ns"] = float(r["AverageNs"])
    for k, cs in table.items():
        print(k)
        for c in sorted(cs):
            print(f"  {c:28s} {cs[c]:.6g}")


if __name__ == "__main__":
    main()
