#!/usr/bin/env python3
"""Per-kernel micro-benchmark of the acoustic sub-step (and optionally one dt) for
the library named by $MPAS_DYCORE_LIB (default: the in-tree build).

    MPAS_DYCORE_LIB=exp/lib_x.so python tools/kbench.py [--ncells 163842] [--steps 2]
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
    ap.add_argument("--levels", type=int, default=56)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--moist", action="store_true", help="BASELINE configs[3]: ns=6 moist species")
    a = ap.parse_args()
    from mpas_dycore import Dycore
    from mpas_dycore.cases import jw_case
    ns = 6 if a.moist else 1
    case = jw_case(a.ncells, K=a.levels, ns=ns, moist=a.moist)
    dt = case["dt"]
    dy = Dycore(case, device=0, moist_end=ns)
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
    ms_dt = (time.perf_counter() - t0) / a.steps * 1e3
    # the prognostic state after the timed steps: equal digests = the two libraries' steps agree bit for bit
    import hashlib
    hsh = hashlib.sha256()
    for name in ("u", "w", "theta_m", "rho_zz", "scalars"):
        hsh.update(dy.get("state", name).tobytes())
    digest = hsh.hexdigest()[:16]
    dts = dt / case["config"]["config_dynamics_split_steps"] / case["config"]["config_number_of_sub_steps"]
    ms, ks = dy.time_acoustic_step(dts, 2, a.reps)
    b = dy.acoustic_bytes()
    print(json.dumps(dict(lib=os.environ.get("MPAS_DYCORE_LIB", "in-tree"), state=digest, ms_dt=ms_dt, ms_sub=sum(ks),
                          edges=ks[0], cells=ks[1], divdamp=ks[2], frac=b / (sum(ks) / 1e3) / 8e12)))


if __name__ == "__main__":
    main()
