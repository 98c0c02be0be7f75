"""GPU parity: the HIP dycore (through the C ABI) vs the reference Fortran dycore.

The oracle is the unmodified reference atm_srk3 compiled from /root/reference
(oracle/Makefile) -- its binary travels to the GPU box in oracle/_ref, so the
same synthetic case is run through both here.  Tolerances (north_star):
relative L-infinity <= 1e-10 on u / theta_m / rho_zz (and w, scalars) after
10 dt steps; init diagnostics and one step are checked tighter.
"""
import numpy as np
import pytest

from conftest import rel_linf

pytestmark = pytest.mark.gpu

DT = 2880.0  # x1.642 (~960 km): SURVEY.md §8d scales dt with resolution (2562 -> 2880 s)
# mpas_reconstruct outputs (cos/sin of lat/lon come from the device math library)
RECON = [("diag", n, "diag." + n) for n in ("uReconstructX", "uReconstructY", "uReconstructZ", "uReconstructZonal",
                                             "uReconstructMeridional")]
# diagnostics as the last atm_compute_solve_diagnostics of the step leaves them (gradPVt / gradPVn
# are stored by that call only: nothing reads them in between)
DIAG = [("diag", n, "diag." + n) for n in ("gradPVt", "gradPVn", "pv_edge", "pv_vertex", "pv_cell", "vorticity",
                                           "divergence", "ke", "rho_edge", "v", "h_divergence", "tend_rtheta_adv")] + \
    [("tend_physics", "rthdynten", "tend_physics.rthdynten")]
PROG = [("state", "u", "state.u.tl1"), ("state", "theta_m", "state.theta_m.tl1"),
        ("state", "rho_zz", "state.rho_zz.tl1"), ("state", "w", "state.w.tl1")]


def _dycore(case):
    from mpas_dycore import Dycore
    dy = Dycore(case, device=0)
    dy.init_diagnostics(DT)
    return dy


@pytest.fixture(scope="module")
def ref_run(small_case):
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    res, _ = ref_runner.run_reference(small_case, nsteps=10, dt=DT, dump_steps=[0, 1, 10], nthreads=4)
    return res


def test_init_diagnostics_match_reference(small_case, ref_run):
    dy = _dycore(small_case)
    ref = ref_run[0]
    for pool, name, key in (PROG + [("diag", "exner", "diag.exner"), ("diag", "pressure_p", "diag.pressure_p"),
                                   ("diag", "ru", "diag.ru"), ("diag", "rw", "diag.rw"),
                                   ("diag", "pv_edge", "diag.pv_edge"), ("diag", "ke", "diag.ke"),
                                   ("diag", "v", "diag.v"), ("diag", "rho_edge", "diag.rho_edge"),
                                   ("diag", "divergence", "diag.divergence"), ("diag", "vorticity", "diag.vorticity")]
                                  + RECON):
        got = dy.get(pool, name, 1)
        err = rel_linf(got, ref[key])
        assert err <= 1e-13, f"{key}: rel Linf {err:.3e}"


# w is a small derived field (|w| << |u|); its relative error is looser by construction
@pytest.mark.parametrize("nsteps,tol,wtol", [(1, 1e-13, 1e-11), (10, 1e-10, 1e-10)])
def test_timestep_matches_reference(small_case, ref_run, nsteps, tol, wtol):
    dy = _dycore(small_case)
    for it in range(nsteps):
        dy.atm_timestep(DT, it + 1)
        dy.shift_time_levels()
    dy.synchronize()
    ref = ref_run[nsteps]
    errs = {}
    for pool, name, key in PROG + [("state", "scalars", "state.scalars.tl1")] + RECON + DIAG:
        got = dy.get(pool, name, 1)
        errs[key] = rel_linf(got.reshape(ref[key].shape), ref[key])
    # w and the reconstructed Z / meridional components are small for the zonal JW flow, so
    # their error relative to their own (small) maximum is looser by construction; so are the
    # derived diagnostics (differences of pv and ke between neighbours)
    loose = {"state.w.tl1"} | {k for _, _, k in RECON} | {k for _, _, k in DIAG}
    bad = {k: v for k, v in errs.items() if not v <= (wtol if k in loose else tol)}
    assert not bad, f"rel Linf above {tol}: {bad} (all: {errs})"


def test_moist_trajectory_matches_reference_fixture():
    """Moist JW + 2 tracer blobs (num_scalars=3, monotone split transport exercised) vs the
    committed reference trajectory: rel Linf <= 1e-10 after 10 steps (north_star bar)."""
    import os
    from mpas_dycore import Dycore
    from mpas_dycore.cases import jw_case
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "srk3_x1.642_K26_ns3.npz"))
    case = jw_case(642, K=26, ns=3, moist=True, cache=False)
    dt = float(z["dt"])
    dy = Dycore(case, device=0)
    dy.init_diagnostics(dt)
    for it in range(10):
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
        if it + 1 in (1, 10):
            dy.synchronize()
            for pool, name, key in PROG + [("state", "scalars", "state.scalars.tl1")]:
                ref = z[f"step{it + 1}_{key}"]
                got = dy.get(pool, name, 1).reshape(ref.shape)
                err = rel_linf(got, ref)
                tol = 1e-10 if (it + 1 == 10 or name in ("w", "scalars")) else 1e-12
                assert err <= tol, f"step {it + 1} {key}: rel Linf {err:.3e}"
    dy.close()


def test_output_diagnostics(small_case):
    """atm_compute_output_diagnostics (mpas_atm_core.F:753-800) after one step, against the
    routine's three expressions evaluated in numpy on the downloaded state (bitwise)."""
    dy = _dycore(small_case)
    dy.atm_timestep(DT, 1)
    dy.shift_time_levels()
    dy.output_diagnostics(1)
    dy.synchronize()
    rvord = 461.6 / 287.0
    th_m, rzz, q = dy.get("state", "theta_m", 1), dy.get("state", "rho_zz", 1), dy.get("state", "scalars", 1)
    pb, pp = dy.get("diag", "pressure_base"), dy.get("diag", "pressure_p")
    zz = np.asarray(small_case["zz"])
    assert np.array_equal(dy.get("diag", "theta"), th_m / (1.0 + rvord * q[:, :, 0]))
    assert np.array_equal(dy.get("diag", "rho"), rzz * zz)
    assert np.array_equal(dy.get("diag", "pressure"), pb + pp)
    dy.close()
