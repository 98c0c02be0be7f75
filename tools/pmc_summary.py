#!/usr/bin/env python3
"""Summarise the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_traffic.sh per kernel.

Counter values are KiB per dispatch.  FETCH_SIZE on gfx950 under-reports
streaming reads (MI355X_MICROARCH.md "HBM"); the factor for this code's
8-byte-per-lane column loads is calibrated on k_copy_many, whose bytes are known
exactly (atm_rk_integration_setup: ten contiguous copies).
Usage: python tools/pmc_summary.py gpurun_out [ncells levels ns] > profiles/...
"""
import csv
import json
import os
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("mpas::", "")
            per[name].append((float(r["Counter_Value"]) * 1024.0,
                              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9,
                              int(r["Dispatch_Id"])))
    return per


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    nC, K, ns = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (163842, 56, 1)
    fetch = load(os.path.join(d, "pmc_fetch", "fetch_counter_collection.csv"))
    write = load(os.path.join(d, "pmc_write", "write_counter_collection.csv"))
    # calibration: k_copy_many (atm_rk_integration_setup's scalars_2 = scalars_1, the one copy the
    # step still makes) moves (nC + 1) * K * ns doubles each way
    known = 8.0 * (nC + 1) * K * ns
    cf = known / (sum(x[0] for x in fetch["k_copy_many"]) / len(fetch["k_copy_many"]))
    cw = known / (sum(x[0] for x in write["k_copy_many"]) / len(write["k_copy_many"]))
    rows = []
    for name in fetch:
        if name not in write:
            continue
        f = sum(x[0] for x in fetch[name]) / len(fetch[name]) * cf
        w = sum(x[0] for x in write[name]) / len(write[name]) * cw
        rows.append(dict(kernel=name, dispatches=len(fetch[name]), read_bytes=f, write_bytes=w))
    rows.sort(key=lambda r: -(r["read_bytes"] + r["write_bytes"]) * r["dispatches"])
    out = dict(ncells=nC, levels=K, num_scalars=ns, fetch_calibration=cf, write_calibration=cw,
               method="rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; per-dispatch mean; "
                      "FETCH/WRITE scaled by the factor that makes k_copy_many (known bytes) exact",
               kernels=rows)
    # the roofline sub-step is the one bench.py times: the acoustic loop of time_acoustic_step
    # (small_step = 2), selected as in tools/acoustic_from_trace.py, per sub-step
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from acoustic_from_trace import tail_dispatches
    reps = int(os.environ.get("ACOUSTIC_REPS", "5"))
    tot = 0.0
    per = {}
    for src, scale, key in ((fetch, cf, "read_bytes"), (write, cw, "write_bytes")):
        rows = [(x[2], name, x[0]) for name, v in src.items() for x in v]
        for fam, vals in tail_dispatches(rows, reps).items():
            b = sum(vals) / reps * scale
            per.setdefault(fam, {})[key] = b
            tot += b
    out["acoustic_substep_kernels"] = per
    out["bytes_per_substep"] = tot
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
