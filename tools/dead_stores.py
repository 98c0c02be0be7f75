#!/usr/bin/env python3
"""Dead-store candidates of the step: walk the kernel sequence of two dt from a rocprofv3 kernel
trace of bench.py (tools/gpu.sh prof) and flag every array a kernel writes that the next write
overwrites before any kernel reads it.  Reads and writes per kernel come from tools/kernel_access.py
(text scan of the kernels' Ptrs accesses) with the template-variant rules of kernel_roofline.py.

It is a candidate list, not a proof: the scan does not see element ranges (a kernel over the halo
cells only overwrites nothing of the owned ones), runtime store flags, or the pool the host reads
after the step.  Each candidate was checked by hand.

    python tools/dead_stores.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import kernel_roofline as kr  # noqa: E402
from kernel_access import access_map  # noqa: E402


def main():
    amap = access_map()
    reg = kr.registry(163842, 56)
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "k_summary_final" in r["Kernel_Name"] and
            (i + 1 == len(rows) or "k_summary" not in rows[i + 1]["Kernel_Name"])]
    seq = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mpas::", "").strip()
           for r in rows[ends[-3] + 1:ends[-1] + 1]]

    def acc(full):
        base = full.split("<")[0]
        if base not in amap:
            return set(), set()
        R, W = (set(x) for x in amap[base])
        R -= kr.NOT_DEFAULT
        W -= kr.NOT_DEFAULT
        for pre, rule in kr.VARIANT.items():
            if full.startswith(pre):
                R -= rule.get("drop", set())
                W -= rule.get("drop_w", set())

        def key(m):
            k = kr.field_key(m, reg)
            if k is None:
                return None
            return k + ":" + m.rstrip("_rd")[-1] if k.startswith("state.") else k
        R = {key(m) for m in R} | {k + ":x" for k in kr.EXTRA_READS.get(base, set())}
        W = {key(m) for m in W}
        return {r for r in R if r}, {w for w in W if w}

    n = len(seq)
    pending, dead = {}, {}
    both = seq + seq
    for i, k in enumerate(both):
        R, W = acc(k)
        for a in R:
            pending.pop(a, None)
        for a in W:
            if a in pending and i >= n:
                dead.setdefault((both[pending[a]], a), []).append(k)
            pending[a] = i
    for (w, a), by in sorted(dead.items()):
        print(f"{w[:40]:40s} writes {a:28s} overwritten by {by[0][:40]} (x{len(by) // 2 or 1} per dt)")


if __name__ == "__main__":
    main()
