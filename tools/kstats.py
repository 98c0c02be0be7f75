#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, avg us, total ms, %."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    with open(path) as f:
        rows = list(csv.DictReader(f))
    for r in rows[:int(__import__("os").environ.get("TOP", "25"))]:
        name = r["Name"].split("(")[0].replace("mpas::", "")
        print(f"{name:34s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us {float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['Percentage']):6.2f}%")
