"""GPU parity across the dycore's namelist branches (Registry.xml nhyd_model options).

Each variant runs 3 `atm_timestep` calls on x1.642, once through the HIP dycore
and once through the live reference `atm_srk3` (oracle/_ref), and compares the
prognostics. The variants cover:
  * RK3 order 3;
  * the 2d_fixed mixing path (∇², ∇⁴, vertical mixing, mix_full on and off);
  * Rayleigh damping and the CAM top filter;
  * scalar transport inside the RK loop (no dynamics/transport split);
  * positive-definite-only and unlimited scalar transport.
Tolerance: relative L∞ 1e-11. The north_star bar is 1e-10 after 10 steps.
"""
import copy

import numpy as np
import pytest

from conftest import rel_linf

pytestmark = pytest.mark.gpu

DT = 2880.0
NSTEPS = 3
KEYS = [("state", "u", "state.u.tl1"), ("state", "theta_m", "state.theta_m.tl1"),
        ("state", "rho_zz", "state.rho_zz.tl1"), ("state", "w", "state.w.tl1"),
        ("state", "scalars", "state.scalars.tl1")]

FIXED = dict(config_horiz_mixing="2d_fixed", config_h_mom_eddy_visc2=2.0e5, config_h_mom_eddy_visc4=4.0e15,
             config_h_theta_eddy_visc2=1.0e5, config_h_theta_eddy_visc4=2.0e15, config_v_mom_eddy_visc2=5.0,
             config_v_theta_eddy_visc2=5.0)
VARIANTS = {
    "order3": (False, dict(config_time_integration_order=3)),
    "fixed_mixing": (False, FIXED),
    "fixed_mixing_no_mix_full": (False, dict(FIXED, config_mix_full=False)),
    "rayleigh_cam": (False, dict(config_rayleigh_damp_u=True, config_number_rayleigh_damp_u_levels=5,
                                 config_rayleigh_damp_u_timescale_days=2.0, config_mpas_cam_coef=0.2)),
    "transport_in_dynamics": (True, dict(config_split_dynamics_transport=False)),
    # selects the same atm_advance_scalars_mono path as the default monotonic option: v7's
    # mono routine has no positive-definite-only branch, so the trajectory is the default's
    "positive_definite": (True, dict(config_monotonic=False, config_positive_definite=True)),
    "no_limiter": (True, dict(config_monotonic=False, config_positive_definite=False)),
    "order3_transport_in_dynamics": (True, dict(config_time_integration_order=3,
                                                config_split_dynamics_transport=False)),
    # every scalar a moist species (moist_end = num_scalars): qtot sums them all (1899-1931)
    "all_scalars_moist": (True, dict(moist_end=3)),
}


@pytest.fixture(scope="module")
def default_refs(small_case, moist_case):
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    return {moist: ref_runner.run_reference(c, nsteps=NSTEPS, dt=DT, dump_steps=[NSTEPS], nthreads=4)[0][NSTEPS]
            for moist, c in ((False, small_case), (True, moist_case))}


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_config_variant_matches_reference(name, small_case, moist_case, default_refs):
    from mpas_dycore import Dycore
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    moist, cfg = VARIANTS[name]
    cfg = dict(cfg)
    moist_end = cfg.pop("moist_end", 1)
    case = copy.copy(moist_case if moist else small_case)
    case["config"] = dict(case["config"], **cfg)
    res, _ = ref_runner.run_reference(case, nsteps=NSTEPS, dt=DT, dump_steps=[NSTEPS], nthreads=4, moist_end=moist_end)
    ref = res[NSTEPS]
    dy = Dycore(case, device=0, moist_end=moist_end)
    dy.init_diagnostics(DT)
    for it in range(NSTEPS):
        dy.atm_timestep(DT, it + 1)
        dy.shift_time_levels()
    dy.synchronize()
    errs = {}
    for pool, fname, key in KEYS:
        got = dy.get(pool, fname, 1)
        errs[key] = rel_linf(got.reshape(ref[key].shape), ref[key])
    dy.close()
    # the option really changes the trajectory (so the branch is exercised, not skipped)
    base = default_refs[moist]
    changed = max(rel_linf(ref[k], base[k]) for _, _, k in KEYS)
    if name == "positive_definite":
        assert changed == 0.0
    else:
        assert changed > 1e-9, f"{name}: option did not change the reference trajectory ({changed:.2e})"
    bad = {k: v for k, v in errs.items() if not v <= 1e-11}
    assert not bad, f"{name}: {bad} (all {errs})"
    assert np.isfinite(list(errs.values())).all()
