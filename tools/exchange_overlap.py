#!/usr/bin/env python3
"""How much of the halo-exchange kernels' time is exposed, from a rocprofv3 kernel trace of a
decomposed run (tools/gpu.sh prof8b: 8 RCCL blocks on one GPU, split-phase exchanges).

The exchange kernels (k_halo_copy packs / unpacks and the RCCL kernels) run on the exchange
stream while the compute stream works on interior elements.  For each exchange
kernel this counts the part of its interval during which no compute kernel was running: that
part is on the critical path, the rest is hidden behind compute.

    python tools/exchange_overlap.py gpurun_out/prof8b/run_kernel_trace.csv [STEPS]

STEPS (default 3): the last STEPS atm_timestep launches, delimited as in tools/step_trace.py.
"""
import csv
import sys
from collections import defaultdict


def is_exchange(name):
    return "k_halo_copy" in name or "nccl" in name.lower() or "rccl" in name.lower()


def union(intervals):
    out = []
    for a, b in sorted(intervals):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def covered(a, b, merged):
    """length of [a, b) covered by the sorted disjoint intervals `merged`"""
    s = 0
    for x, y in merged:
        if y <= a:
            continue
        if x >= b:
            break
        s += min(b, y) - max(a, x)
    return s


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "k_summary_final" in r["Kernel_Name"] and
            (i + 1 == len(rows) or "k_summary" not in rows[i + 1]["Kernel_Name"])]
    if len(ends) < steps + 1:
        sys.exit(f"only {len(ends)} steps in the trace")
    sel = rows[ends[-steps - 1] + 1:ends[-1] + 1]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
    comp = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel
                  if not is_exchange(r["Kernel_Name"])])
    tot = defaultdict(float)
    exposed = defaultdict(float)
    calls = defaultdict(int)
    for r in sel:
        n = r["Kernel_Name"]
        if not is_exchange(n):
            continue
        key = "k_halo_copy" if "k_halo_copy" in n else n.split("(")[0][:60]
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        tot[key] += b - a
        exposed[key] += (b - a) - covered(a, b, comp)
        calls[key] += 1
    ex_union = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel
                      if is_exchange(r["Kernel_Name"])])
    ex_only = sum(y - x - covered(x, y, comp) for x, y in ex_union)
    wall = (t1 - t0) / steps
    print(f"wall per dt {wall / 1e6:.3f} ms over {steps} steps; compute-kernel busy "
          f"{sum(y - x for x, y in comp) / steps / 1e6:.3f} ms per dt")
    print(f"{'exchange kernel':60s} {'calls/dt':>9s} {'ms/dt':>8s} {'exposed ms/dt':>14s}")
    for k in sorted(tot, key=lambda k: -tot[k]):
        print(f"{k:60s} {calls[k] / steps:9.1f} {tot[k] / steps / 1e6:8.3f} {exposed[k] / steps / 1e6:14.3f}")
    print(f"time per dt with only exchange kernels running: {ex_only / steps / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
