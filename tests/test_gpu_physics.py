"""GPU parity of the physics coupling: the reference's DO_PHYSICS build.

Oracle: the unmodified reference dycore compiled with -DDO_PHYSICS (make -C oracle phys), whose
physics_get_tend is a test double handing over prescribed tendencies (conftest.physics_forcing).
Product: Dycore.set_physics + the same tendencies set into tend_physics.tend_{ru,rtheta,rho}_physics
and tend.scalars_tend before every step, as the drop-in's atm_srk3 does after its host-side
physics_get_tend.  Exercises tend_u / tend_theta / tend_rho physics terms (dyn_tend 4500-5200),
the scalar physics source in both transport paths (3437, 3743), the clip of negative mixing
ratios and rqvdynten (1610-1648).  Tolerances as test_gpu_parity: rel Linf <= 1e-10 after 10 steps.
"""
import numpy as np
import pytest

from conftest import physics_forcing, rel_linf

pytestmark = pytest.mark.gpu

KEYS = [("state", "u", "state.u.tl1"), ("state", "theta_m", "state.theta_m.tl1"),
        ("state", "rho_zz", "state.rho_zz.tl1"), ("state", "w", "state.w.tl1"),
        ("state", "scalars", "state.scalars.tl1")]


def _img(a):
    """element-major (n, ...) -> the Fortran (..., n+1) memory image with a zero garbage slot."""
    out = np.zeros((a.shape[0] + 1,) + a.shape[1:])
    out[:-1] = a
    return out


@pytest.mark.parametrize("monotonic,convection", [(True, "cu_tiedtke"), (False, "off")])
def test_physics_coupling_matches_reference(monotonic, convection):
    from oracle import ref_runner
    from mpas_dycore import Dycore
    from mpas_dycore.cases import jw_case
    if not ref_runner.available(ref_runner.PHYS_HARNESS):
        pytest.skip("oracle/_ref/mpas_ref_harness_phys not built")
    case = jw_case(642, K=26, ns=3, moist=True, cache=False)
    case["config"] = dict(case["config"], config_monotonic=monotonic)
    dt = float(case["dt"])
    phys = physics_forcing(case)
    ref, _ = ref_runner.run_reference(case, 10, dt, [1, 10], nthreads=4,
                                      physics=dict(phys, convection_scheme=convection))
    dy = Dycore(case, device=0)
    dy.init_diagnostics(dt)
    rqv = convection != "off"
    dy.set_physics(tendencies=True, rqvdynten=rqv)
    for n in ("tend_ru_physics", "tend_rtheta_physics", "tend_rho_physics"):
        dy.set_raw("tend_physics", n, _img(phys[n]))
    for it in range(10):
        dy.set_raw("tend", "scalars_tend", _img(phys["scalars_tend"]))
        dy.atm_timestep(dt, it + 1)
        if rqv and it + 1 in (1, 10):
            got = dy.get("tend_physics", "rqvdynten")
            want = ref[it + 1]["tend_physics.rqvdynten"]
            assert rel_linf(got, want) <= 1e-10, f"step {it + 1} rqvdynten"
        dy.shift_time_levels()
        if it + 1 in (1, 10):
            dy.synchronize()
            for pool, name, key in KEYS:
                want = ref[it + 1][key]
                got = dy.get(pool, name, 1).reshape(want.shape)
                tol = 1e-10 if (it + 1 == 10 or name in ("w", "scalars")) else 1e-12
                err = rel_linf(got, want)
                assert err <= tol, f"step {it + 1} {key}: rel Linf {err:.3e}"
            if it + 1 == 10:
                assert dy.get("state", "scalars", 1).min() >= 0.0  # clipped
    dy.close()


def test_physics_zero_tendencies_bitwise():
    """Coupling on with all-zero tendencies gives the same bits as coupling off."""
    from mpas_dycore import Dycore
    from mpas_dycore.cases import jw_case
    case = jw_case(642, K=26, ns=3, moist=True, cache=False)
    dt = float(case["dt"])
    out = []
    for on in (False, True):
        dy = Dycore(case, device=0)
        dy.init_diagnostics(dt)
        if on:
            dy.set_physics(tendencies=True)
        for it in range(3):
            if on:
                dy.set_raw("tend", "scalars_tend", np.zeros((case["nCells"] + 1, case["nVertLevels"],
                                                            case["num_scalars"])))
            dy.atm_timestep(dt, it + 1)
            dy.shift_time_levels()
        dy.synchronize()
        out.append([dy.get(p, n, 1) for p, n, _ in KEYS])
        dy.close()
    for (p, n, _), a, b in zip(KEYS, *out):
        assert np.array_equal(a, b), n
