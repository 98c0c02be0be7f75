#!/usr/bin/env python3
"""Cost of the drop-in's per-step summarize_timestep read-back (mpas_dyc_get_summary blocks the host
until the step is done, so the next step is launched after an idle device) at a per-rank size.

One rank of an 8-way split of x1.163842 x 56 holds about 20480 owned cells, between the
icosahedral x1.10242 and x1.40962 meshes (a rank of a 16- and a 4-way split); this runs the
Fortran drop-in under the harness driver on each for 20 steps with config_print_global_minmax_vel
(the namelist default, Registry.xml:339) on and off, and prints the ms per dt of steps 3..20.

    python tools/dropin_summary_cost.py [ROUNDS]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpas-model_amd")]


def main():
    from mpas_dycore.cases import jw_case
    from oracle import ref_runner
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for nc in (10242, 40962):
        run(jw_case(nc, K=56, ns=1), nc, rounds)


def run(c, nc, rounds):
    from oracle import ref_runner
    n, dt = 20, float(c["dt"])
    for r in range(rounds):
        for pm in (1, 0):
            _, _, total = ref_runner.run_reference(c, nsteps=n, dt=dt, dump_steps=[n], nthreads=1,
                                                   dump_only=["state.u"], binary=ref_runner.DROPIN_HARNESS,
                                                   with_total=True, print_minmax=pm)
            print(f"x1.{nc} round {r} print_global_minmax_vel={pm}: {1e3 * total['after2'] / (n - 2):.3f} ms/dt", flush=True)


if __name__ == "__main__":
    main()
