#!/usr/bin/env python3
"""Per-dt breakdown of a rocprofv3 kernel trace of bench.py: the last STEPS atm_timestep launches
(delimited by the summary kernels that end every step), with the wall time of each step,
the summed kernel time by kernel, the busy fraction of the device, and the gaps.

    python tools/step_trace.py gpurun_out/prof8b/run_kernel_trace.csv [STEPS] [TOP]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # a step ends with its blocks' summary kernels (one k_summary_partial / k_summary_final pair each)
    ends = [i for i, r in enumerate(rows) if "k_summary_final" in r["Kernel_Name"] and
            (i + 1 == len(rows) or "k_summary" not in rows[i + 1]["Kernel_Name"])]
    if len(ends) < steps + 1:
        sys.exit(f"only {len(ends)} steps in the trace")
    lo, hi = ends[-steps - 1] + 1, ends[-1] + 1
    sel = rows[lo:hi]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
    per = defaultdict(lambda: [0, 0.0])
    busy, last_end = 0.0, t0
    for r in sel:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mpas::", "")
        per[n][0] += 1
        per[n][1] += (e - s)
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
    wall = (t1 - t0) / 1e6 / steps
    print(f"steps {steps}: wall {wall:.3f} ms/dt, device busy {busy / 1e6 / steps:.3f} ms/dt "
          f"({100 * busy / (t1 - t0):.1f} %), {len(sel) / steps:.0f} kernels/dt")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"  {n[:58]:58s} {c / steps:7.1f}/dt {t / c / 1e3:8.1f} us {t / 1e6 / steps:8.3f} ms/dt")


if __name__ == "__main__":
    main()
