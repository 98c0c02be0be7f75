#!/usr/bin/env python3
"""Per-kernel durations of the acoustic loop that bench.py times, from a rocprofv3 kernel_trace.csv.

mpas_dyc_time_acoustic_step runs REPS sub-steps with small_step = 2, as srk3 does:
  * the edge phase; for every further sub-step, the edge phase with the previous damping fused in (k_acoustic_edges<true>);
  * the cell phase;
  * after the last sub-step, one standalone k_divdamp.
Those are the last REPS edge dispatches, the last REPS cell dispatches and the last damping dispatch.

    python tools/acoustic_from_trace.py gpurun_out/prof/run_kernel_trace.csv [REPS] [BYTES]

Prints JSON: the per-sub-step average of each family, their sum, and, given B_ac, the GB/s.
"""
import csv
import json
import sys
from collections import defaultdict

FAMILIES = ("k_acoustic_edges", "k_acoustic_cells", "k_divdamp")


def tail_dispatches(rows, reps):
    """{family: [durations]}: the timed loop's dispatches, from (dispatch_id, name, value) rows."""
    d = defaultdict(list)
    for did, name, v in sorted(rows):
        for key in FAMILIES:
            if key in name:
                d[key].append(v)
    return {k: v[-(1 if k == "k_divdamp" else reps):] for k, v in d.items()}


def main():
    path = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    b_ac = float(sys.argv[3]) if len(sys.argv) > 3 else 3535036176.0
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"],
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3))
    out = {}
    for key, v in tail_dispatches(rows, reps).items():
        out[key] = dict(timed_dispatches=len(v), us_per_substep=sum(v) / reps)
    sub = sum(x["us_per_substep"] for x in out.values())
    out["substep_us"] = sub
    out["bytes_per_substep"] = b_ac
    out["achieved_GBs"] = b_ac / (sub * 1e-6) / 1e9
    out["frac_of_8TBs"] = out["achieved_GBs"] / 8000.0
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
