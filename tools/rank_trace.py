#!/usr/bin/env python3
"""Attribute one rank's time per dt from rocprofv3 kernel traces of tools/rank_emulation.py
(gpurun step prof8e): the compute-only emulation (every block alone, no lists) against the
split-phase emulation (the block's real lists, messages looped back), and optionally the
8-RCCL-blocks run of bench.py --blocks 8 --rccl-local (gpurun step prof8b).

Each emulated block runs STEPS_PER_BLOCK steps (2 warm-up + the timed ones); the last STEPS of
each block are used.  Kernels are grouped into: interior / full-range compute kernels, phase-2
launches of the split kernels (their grids are small: the halo-boundary lists), k_halo_copy,
RCCL kernels.  Per group: kernel time per dt per block, and for the exchange kernels the part no
compute kernel overlaps.

    python tools/rank_trace.py COMPUTE_TRACE EXCHANGE_TRACE [BLOCKS8_TRACE] [--steps 3] [--per-block 5]
"""
import argparse
import csv
from collections import defaultdict


def kname(r):
    return r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mpas::", "")


def is_exchange(n):
    return "k_halo_copy" in n or "k_p2p" in n or "nccl" in n.lower() or "rccl" in n.lower()


def union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def covered(a, b, merged):
    s = 0
    for x, y in merged:
        if y <= a:
            continue
        if x >= b:
            break
        s += min(b, y) - max(a, x)
    return s


def step_ends(rows):
    return [i for i, r in enumerate(rows) if "k_summary_final" in r["Kernel_Name"] and
            (i + 1 == len(rows) or "k_summary" not in rows[i + 1]["Kernel_Name"])]


def segments(rows, per_block, steps, nblocks=None):
    """(lo, hi) row ranges of the last `steps` steps of each emulated block"""
    ends = step_ends(rows)
    if nblocks is None:  # one segment: the last `steps` steps
        return [(ends[-steps - 1] + 1, ends[-1] + 1)]
    segs = []
    for b in range(nblocks):
        last = (b + 1) * per_block - 1
        segs.append((ends[last - steps] + 1, ends[last] + 1))
    return segs


def classify(r, big_grid):
    n = kname(r)
    if is_exchange(n):
        return "rccl" if "k_halo_copy" not in n else "k_halo_copy", n
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"])
    return ("phase2" if g < big_grid else "compute"), n


def analyse(rows, segs, steps, big_grid):
    grp = defaultdict(float)
    exposed = defaultdict(float)
    per = defaultdict(lambda: [0, 0.0])
    wall = busy = 0.0
    for lo, hi in segs:
        sel = rows[lo:hi]
        t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
        wall += t1 - t0
        comp = union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel if not is_exchange(kname(r))])
        busy += sum(y - x for x, y in union([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel]))
        for r in sel:
            g, n = classify(r, big_grid)
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            grp[g] += b - a
            per[(g, n)][0] += 1
            per[(g, n)][1] += b - a
            if g in ("rccl", "k_halo_copy"):
                exposed[g] += (b - a) - covered(a, b, comp)
    nb = len(segs) * steps
    return {"wall": wall / nb / 1e6, "busy": busy / nb / 1e6,
            "groups": {g: t / nb / 1e6 for g, t in grp.items()},
            "exposed": {g: t / nb / 1e6 for g, t in exposed.items()},
            "per": {k: (c / nb, t / nb / 1e6) for k, (c, t) in per.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("compute")
    ap.add_argument("exchange")
    ap.add_argument("blocks8", nargs="?")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--per-block", type=int, default=5)
    ap.add_argument("--nblocks", type=int, default=8)
    ap.add_argument("--big-grid", type=int, default=2000, help="workgroups below this = a phase-2 launch")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    res = {}
    for tag, path in (("compute", a.compute), ("exchange", a.exchange)):
        rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
        res[tag] = analyse(rows, segments(rows, a.per_block, a.steps, a.nblocks), a.steps, a.big_grid)
    if a.blocks8:
        rows = sorted(csv.DictReader(open(a.blocks8)), key=lambda r: int(r["Start_Timestamp"]))
        r8 = analyse(rows, segments(rows, 0, a.steps), a.steps, a.big_grid)
        # per block: everything over the 8 blocks of one process
        r8 = {"wall": r8["wall"] / a.nblocks, "busy": r8["busy"] / a.nblocks,
              "groups": {g: t / a.nblocks for g, t in r8["groups"].items()},
              "exposed": {g: t / a.nblocks for g, t in r8["exposed"].items()},
              "per": {k: (c / a.nblocks, t / a.nblocks) for k, (c, t) in r8["per"].items()}}
        res["blocks8/8"] = r8
    tags = list(res)
    print("ms per dt per block (rank)  " + "".join(f"{t:>14s}" for t in tags))
    print("  wall (trace)              " + "".join(f"{res[t]['wall']:14.3f}" for t in tags))
    print("  device busy               " + "".join(f"{res[t]['busy']:14.3f}" for t in tags))
    for g in ("compute", "phase2", "k_halo_copy", "rccl"):
        print(f"  {g:26s}" + "".join(f"{res[t]['groups'].get(g, 0.0):14.3f}" for t in tags))
    for g in ("k_halo_copy", "rccl"):
        print(f"  {g + ' exposed':26s}" + "".join(f"{res[t]['exposed'].get(g, 0.0):14.3f}" for t in tags))
    keys = set()
    for t in tags:
        keys |= set(res[t]["per"])
    diff = sorted(keys, key=lambda k: -abs(res["exchange"]["per"].get(k, (0, 0))[1] - res["compute"]["per"].get(k, (0, 0))[1]))
    print(f"\nkernels by |exchange - compute| (calls/dt, ms/dt per block):")
    for k in diff[:a.top]:
        cells = "".join(f"{res[t]['per'].get(k, (0, 0))[0]:7.1f} {res[t]['per'].get(k, (0, 0))[1]:7.3f}" for t in tags)
        print(f"  {k[0][:7]:7s} {k[1][:50]:50s} {cells}")


if __name__ == "__main__":
    main()
