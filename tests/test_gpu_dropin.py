"""GPU: the Fortran drop-in module under the reference's own driver.

`oracle/_ref/mpas_dropin_harness` is the unmodified harness driver
(oracle/harness/mpas_ref_harness.F90). It is linked against
mpas-model_amd/fortran/atm_time_integration_mi355x.F90 (module
atm_time_integration over the C ABI) and libmpas_dycore.so, in place of the
reference's mpas_atm_time_integration.F. The driver makes the calls
mpas_atm_core.F makes:
  * init diagnostics;
  * host mpas_init_reconstruct;
  * atm_srk3 followed by mpas_pool_shift_time_levels.
The pools it dumps are then checked in three ways:
  * against the reference harness (rel L∞, same tolerances as test_gpu_parity);
  * bit for bit against the Python host driving the same library;
  * for the dump after model init, against the reference's init diagnostics.
"""
import numpy as np
import pytest

from conftest import rel_linf

pytestmark = pytest.mark.gpu

DT = 2880.0
NSTEPS = 3
PROG = ["state.u.tl1", "state.theta_m.tl1", "state.rho_zz.tl1", "state.w.tl1", "state.scalars.tl1"]
RECON = ["diag." + n for n in ("uReconstructX", "uReconstructY", "uReconstructZ", "uReconstructZonal",
                               "uReconstructMeridional")]
INIT = ["state.theta_m.tl1", "state.rho_zz.tl1", "diag.ru", "diag.rw", "diag.pv_edge", "diag.exner"]
LOOSE = {"state.w.tl1", "diag.rw"} | set(RECON)   # small components of the zonal JW flow


def _runs(case, moist_end=1):
    from oracle import ref_runner
    if not (ref_runner.available() and ref_runner.available(ref_runner.DROPIN_HARNESS)):
        pytest.skip("oracle/_ref harness binaries not built (make -C oracle all dropin)")
    ref, _ = ref_runner.run_reference(case, nsteps=NSTEPS, dt=DT, dump_steps=[0, NSTEPS], nthreads=4,
                                      moist_end=moist_end)
    # one thread: the drop-in's first atm_compute_solve_diagnostics call creates the device context
    got, _ = ref_runner.run_reference(case, nsteps=NSTEPS, dt=DT, dump_steps=[0, NSTEPS], nthreads=1,
                                      moist_end=moist_end, binary=ref_runner.DROPIN_HARNESS)
    return ref, got


def _python_host(case, moist_end=1):
    from mpas_dycore import Dycore
    dy = Dycore(case, device=0, moist_end=moist_end)
    dy.init_diagnostics(DT)
    for it in range(NSTEPS):
        dy.atm_timestep(DT, it + 1)
        dy.shift_time_levels()
    dy.synchronize()
    out = {k: dy.get(k.split(".")[0], k.split(".")[1], 1) for k in PROG + RECON}
    dy.close()
    return out


@pytest.mark.parametrize("moist", [False, True])
def test_dropin_harness_matches_reference(small_case, moist_case, moist):
    case = moist_case if moist else small_case
    ref, got = _runs(case)
    errs = {}
    for k in INIT:
        errs["init " + k] = rel_linf(got[0][k], ref[0][k])
    for k in PROG + RECON:
        errs[k] = rel_linf(got[NSTEPS][k], ref[NSTEPS][k])
    bad = {k: v for k, v in errs.items() if not v <= (1e-11 if k.split()[-1] in LOOSE else 1e-12)}
    assert not bad, f"drop-in vs reference: {bad} (all {errs})"
    # the Fortran API path and the Python host drive the same library on the same inputs
    py = _python_host(case)
    for k in PROG + RECON:
        a = got[NSTEPS][k]
        assert np.array_equal(a, py[k].reshape(a.shape)), f"{k}: drop-in differs from the Python host"
