#!/usr/bin/env python3
"""Time one rank's share of an N-way decomposition on a single GPU (no exchanges).

Builds block 0 of an N-block SFC partition of the x1.<ncells> case and steps it
alone: the time per dt is the compute a rank would spend at N GPUs, without the
RCCL traffic (halo values go stale -- timing only, numerics are not checked).
    python tools/rank_emulation.py [--ncells 163842] [--parts 2 4 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpas-model_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ncells", type=int, default=163842)
    ap.add_argument("--parts", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--order", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true", help="eager launches (what a rank without hipGraph costs)")
    a = ap.parse_args()
    from mpas_dycore import Dycore, decomp
    from mpas_dycore.cases import jw_case
    case = jw_case(a.ncells, K=56, order=a.order)
    dt = case["dt"]
    res = {}
    for n in a.parts:
        if n == 1:
            dy = Dycore(case, device=0)
        else:
            (b,) = decomp.decompose(case, decomp.partition_sfc(case["nCells"], n), parts=[0])
            dy = Dycore(b.case, device=0, solve=b.solve)
        dy.init_diagnostics(dt)
        dy.use_graph(not a.no_graph)
        for i in range(2):
            dy.atm_timestep(dt, i + 1)
            dy.shift_time_levels()
        dy.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            dy.atm_timestep(dt, i + 3)
            dy.shift_time_levels()
        dy.synchronize()
        res[n] = (time.perf_counter() - t0) / a.steps * 1e3
        dy.close()
        print(json.dumps(dict(parts=n, graph=not a.no_graph, ms_per_dt=res[n], compute_speedup=res[a.parts[0]] / res[n])),
              flush=True)


if __name__ == "__main__":
    main()
