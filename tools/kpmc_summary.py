#!/usr/bin/env python3
"""Per-kernel PMC counters of `tools/gpu.sh kpmc` (rocprofv3 --pmc over one eager kbench dt):
the mean over dispatches of each counter, per kernel whose name matches a pattern.

    python tools/kpmc_summary.py gpurun_out/kpmc_0_0 [pattern ...]
"""
import csv
import os
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mpas::", "")
        acc[name][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = {}
    for name, per in acc.items():
        tot = defaultdict(list)
        for (disp, cn), vals in per.items():
            tot[cn].append(sum(vals))  # summed over the dispatch's dimension instances
        out[name] = {cn: sum(v) / len(v) for cn, v in tot.items()}
    return out


def main():
    d = sys.argv[1]
    pats = sys.argv[2:] or [""]
    for name, cs in sorted(load(d).items()):
        if any(p in name for p in pats):
            print(name)
            for cn, v in sorted(cs.items()):
                print(f"    {cn:32s} {v:16.4g}")


if __name__ == "__main__":
    main()
