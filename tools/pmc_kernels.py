#!/usr/bin/env python3
"""Per-kernel means of the counters collected by tools/pmc_kernels.sh (one row per kernel).

    python tools/pmc_kernels.py gpurun_out/pmck [kernel-substring ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmck"
    want = sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for path in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"].split("(")[0].replace("mpas::", "").replace("void ", "")
                if want and not any(w in name for w in want):
                    continue
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    for name in sorted(vals, key=lambda n: -sum(dur[n]) / len(dur[n])):
        c = {k: sum(v) / len(v) for k, v in vals[name].items()}
        us = sum(dur[name]) / len(dur[name])
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        line = [f"{name:34s} {us:8.1f} us"]
        if "SQ_WAVES" in c:
            line.append(f"waves {c['SQ_WAVES']:.0f}")
            line.append(f"wait {c.get('SQ_WAIT_ANY', 0) / wc:.2f} stall {c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
                        f"active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} valu {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f} "
                        f"vmem {c.get('SQ_ACTIVE_INST_VMEM', 0) / wc:.2f}")
            if c.get("SQ_BUSY_CYCLES"):
                line.append(f"avg-waves {c['SQ_WAVE_CYCLES'] / c['SQ_BUSY_CYCLES']:.1f}")
        if "SQ_INSTS_VALU" in c and c.get("SQ_WAVES"):
            pass
        if "SQ_INSTS_VALU" in c:
            line.append(f"valu/inst {c['SQ_INSTS_VALU']:.3g} vmem_rd {c.get('SQ_INSTS_VMEM_RD', 0):.3g} "
                        f"smem {c.get('SQ_INSTS_SMEM', 0):.3g} salu {c.get('SQ_INSTS_SALU', 0):.3g} "
                        f"lvl_vmem/waves {c.get('SQ_INST_LEVEL_VMEM', 0) / max(c.get('SQ_LEVEL_WAVES', 1), 1):.2f}")
        if "TA_BUSY_sum" in c and c.get("GRBM_GUI_ACTIVE"):
            line.append(f"ta_busy {c['TA_BUSY_sum'] / (c['GRBM_GUI_ACTIVE'] / 8 * 32):.2f} "
                        f"ta_stall_tc {c.get('TA_ADDR_STALLED_BY_TC_CYCLES_sum', 0) / max(c['TA_BUSY_sum'], 1):.2f} "
                        f"clk {c['GRBM_GUI_ACTIVE'] / 8 / us / 1e3:.2f} GHz")
        print("  ".join(line))


if __name__ == "__main__":
    main()
