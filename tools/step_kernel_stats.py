#!/usr/bin/env python3
"""Kernel stats of the timed steps alone, from a rocprofv3 kernel_trace.csv of bench.py.

bench.py runs init, --warmup steps, --steps timed steps, then the acoustic timing loop
(mpas_dyc_time_acoustic_step: REPS edge + cell sub-steps and one damping).  Every atm_timestep
launches one k_copy_many (atm_rk_integration_setup's scalars_2 = scalars_1), so the timed steps are
the dispatches from the (warmup+1)-th k_copy_many up to the first dispatch of the timing loop.
Writes a kernel_stats-style CSV (Name, Calls, TotalDurationNs, AverageNs) for tools/kernel_roofline.py.

    python tools/step_kernel_stats.py TRACE.csv WARMUP [REPS] > stats.csv
"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from acoustic_from_trace import FAMILIES  # noqa: E402


def main():
    path, warmup = sys.argv[1], int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    copies = [i for i, (_, n, _) in enumerate(rows) if "k_copy_many" in n]
    start = copies[warmup]
    # the timing loop: the last REPS edge and cell dispatches and the last damping
    fam = defaultdict(list)
    for i, (_, n, _) in enumerate(rows):
        for k in FAMILIES:
            if k in n:
                fam[k].append(i)
    tail = [i for k, v in fam.items() for i in v[-(1 if k == "k_divdamp" else reps):]]
    end = min(tail)
    agg = defaultdict(list)
    for _, n, dur in rows[start:end]:
        agg[n].append(dur)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs"])
    for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        w.writerow([n, len(v), sum(v), sum(v) / len(v)])
    print(f"steps: dispatches {start}..{end} of {len(rows)}, k_copy_many in range: "
          f"{sum(1 for i in copies if start <= i < end)}", file=sys.stderr)


if __name__ == "__main__":
    main()
