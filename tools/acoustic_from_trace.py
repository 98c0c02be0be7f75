#!/usr/bin/env python3
"""Per-kernel durations of the acoustic sub-step that bench.py times (the last REPS
dispatches of k_acoustic_edges / k_acoustic_cells / k_divdamp, launched by
mpas_dyc_time_acoustic_step with small_step = 2), from a rocprofv3 kernel_trace.csv.

    python tools/acoustic_from_trace.py gpurun_out/prof/run_kernel_trace.csv [REPS] [BYTES]
Prints JSON: average us per kernel, the sub-step sum and, given B_ac, the GB/s.
"""
import csv
import json
import sys
from collections import defaultdict

path = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
b_ac = float(sys.argv[3]) if len(sys.argv) > 3 else 3535036176.0
d = defaultdict(list)
with open(path) as f:
    for r in csv.DictReader(f):
        n = r["Kernel_Name"]
        for key in ("k_acoustic_edges", "k_acoustic_cells", "k_divdamp"):
            if key in n:
                d[key].append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3))
out = {}
for key, v in d.items():
    v.sort()
    tail = [t for _, t in v[-reps:]]
    out[key] = dict(dispatches_total=len(v), timed_reps=len(tail), avg_us=sum(tail) / len(tail))
sub = sum(x["avg_us"] for x in out.values())
out["substep_us"] = sub
out["bytes_per_substep"] = b_ac
out["achieved_GBs"] = b_ac / (sub * 1e-6) / 1e9
out["frac_of_8TBs"] = out["achieved_GBs"] / 8000.0
print(json.dumps(out, indent=1))
