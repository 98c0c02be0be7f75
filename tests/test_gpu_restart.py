"""GPU: a restart run (config_do_restart) continues bit for bit.

MPAS restarts from a file holding the state and the diagnostics the step carries over; model init
then skips atm_init_coupled_diagnostics and runs only atm_compute_solve_diagnostics
(mpas_atm_core.F:387-404).  Here: a run of 4 steps vs 2 steps, every state / diag field copied
out as a restart file would hold it, a fresh context given those fields, mpas_dyc_solve_diagnostics
(the restart model init), and 2 more steps.  The drop-in module takes the same path when its
atm_compute_solve_diagnostics is called without atm_init_coupled_diagnostics.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STATE = ("u", "w", "theta_m", "rho_zz", "scalars")
# Registry.xml diag fields the device keeps (the drop-in's diag list, minus the uReconstruct outputs)
DIAG = ("theta", "rho", "rho_base", "theta_base", "rho_p", "rho_p_save", "rho_pp", "rho_zz_old_split",
        "rtheta_base", "rtheta_p", "rtheta_p_save", "rtheta_pp", "rtheta_pp_old", "exner", "exner_base",
        "pressure_base", "pressure_p", "h_divergence", "kdiff", "ke", "divergence", "pv_cell", "tend_rtheta_adv",
        "cqw", "cofwr", "cofwz", "cofwt", "coftz", "a_tri", "alpha_tri", "gamma_tri", "cofrz", "rw", "rw_p",
        "rw_save", "wwAvg", "wwAvg_split", "ru", "ruAvg", "ruAvg_split", "ru_p", "ru_save", "cqu", "rho_edge",
        "v", "pv_edge", "gradPVn", "gradPVt", "vorticity", "pv_vertex")


@pytest.mark.parametrize("moist", [False, True])
def test_restart_continues_bitwise(small_case, moist_case, moist):
    from mpas_dycore import Dycore
    case = moist_case if moist else small_case
    dt = float(case.get("dt", 2880.0))

    def steps(dy, first, n):
        for it in range(first, first + n):
            dy.atm_timestep(dt, it)
            dy.shift_time_levels()
        dy.synchronize()

    a = Dycore(case, device=0)
    a.init_diagnostics(dt)
    steps(a, 1, 4)
    want = {n: a.get_raw("state", n, 1) for n in STATE}
    a.close()

    b = Dycore(case, device=0)
    b.init_diagnostics(dt)
    steps(b, 1, 2)
    restart = {("state", n): b.get_raw("state", n, 1) for n in STATE}
    restart.update({("diag", n): b.get_raw("diag", n) for n in DIAG})
    b.close()

    c = Dycore(case, device=0)   # mesh from the case; state and diag from the "restart file"
    for (pool, n), img in restart.items():
        c.set_raw(pool, n, img, 1)
    c.restart_diagnostics(dt)
    steps(c, 3, 2)
    for n in STATE:
        got = c.get_raw("state", n, 1)
        assert np.array_equal(got, want[n]), f"{n}: restart differs, max |d| {np.max(np.abs(got - want[n])):.3e}"
    c.close()
