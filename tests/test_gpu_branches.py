"""GPU parity for the atm_srk3 sequencer branches that the default namelist never takes.

The reference's acoustic-loop shape is set by config_number_of_sub_steps and
config_time_integration_order (mpas_atm_time_integration.F:296-326): order 3 gives
(1, n/2, n) sub-steps per RK stage, order 2 (n/2, n/2, n).  The default n = 2 only ever
runs stages of 1 and 2 sub-steps.  The variants below run stages of 3, 4 and 6 sub-steps.
That exercises the code the default leaves alone:
  * the fused damping and edge phase of sub-steps >= 3 (k_acoustic_edges_p<true>);
  * the Theta''/rho'' exchange between sub-steps;
  * the stage-last fusions (k_acoustic_cells_r<ME, true>, k_divdamp_p<true>);
  * order 2 with a first stage of several sub-steps.
They also run the dynamics/transport split with 1, 2 and 4 dynamics substeps
(config_dynamics_split_steps, 472-1341), which changes the substep_finish averaging
(5993-6081) and the exchanges at a substep boundary (1282-1297).  Then scalar advection
switched off (config_scalar_advection, 1355).  Then the reference's default 55 levels
(core_init_atmosphere/Registry.xml:100), moist with num_scalars = 6 and the monotone limiter.
At that odd K the pair-layout kernels run their odd-K instantiations (ODD = true: the last lane pair
holds level K-1 and a masked level past the column).

Each variant runs 10 atm_timestep calls on x1.2562 with the captured hipGraph (the product
path).  It is compared with the unmodified reference atm_srk3 (oracle/_ref) on the same mesh
and state.  Tolerance (north_star): relative L-infinity <= 1e-10 on u, theta_m, rho_zz;
<= 1e-9 on w and the mixing ratios (relative to their own maxima).

The multi-block case: 4 MPAS blocks on one device, every halo message through RCCL with
split-phase exchanges, at number_of_sub_steps = 6.  It must equal the one-block run bit for bit.
"""
import copy

import numpy as np
import pytest

from conftest import heartbeat, progress, rel_linf

pytestmark = pytest.mark.gpu

NSTEPS = 10
PROG = [("state", "u", "state.u.tl1", "edge"), ("state", "theta_m", "state.theta_m.tl1", "cell"),
        ("state", "rho_zz", "state.rho_zz.tl1", "cell"), ("state", "w", "state.w.tl1", "cell"),
        ("state", "scalars", "state.scalars.tl1", "cell")]
DUMP = ["state.u", "state.theta_m", "state.rho_zz", "state.w", "state.scalars"]
TIGHT = ("state.u.tl1", "state.theta_m.tl1", "state.rho_zz.tl1")
TOL, TOL_LOOSE = 1e-10, 1e-9

# name -> (case key, namelist overrides).  dt = 2880 s on x1.2562 (~480 km): acoustic dts stays
# at or below 480 s, as in the default (split 3, n = 2).
VARIANTS = {
    "substeps4_order2": ("dry", dict(config_number_of_sub_steps=4, config_time_integration_order=2)),
    "substeps4_order3": ("dry", dict(config_number_of_sub_steps=4, config_time_integration_order=3)),
    "substeps6_order2": ("dry", dict(config_number_of_sub_steps=6, config_time_integration_order=2)),
    "substeps6_order3": ("dry", dict(config_number_of_sub_steps=6, config_time_integration_order=3)),
    "split1_substeps6": ("moist", dict(config_dynamics_split_steps=1, config_number_of_sub_steps=6,
                                       config_time_integration_order=3)),
    "split2_substeps4": ("moist", dict(config_dynamics_split_steps=2, config_number_of_sub_steps=4)),
    "split4": ("moist", dict(config_dynamics_split_steps=4)),
    "no_scalar_advection": ("moist", dict(config_scalar_advection=False)),
    "substeps6_transport_in_dynamics": ("moist", dict(config_number_of_sub_steps=6,
                                                      config_split_dynamics_transport=False)),
    "L55_moist_ns6_mono": ("moist55", dict(config_time_integration_order=3)),
}
MOIST_END = {"dry": 1, "moist": 3, "moist55": 6}
_BASE = {}  # default-namelist GPU runs per case key


@pytest.fixture(scope="module")
def cases():
    from mpas_dycore.cases import jw_case
    with heartbeat("building x1.2562 cases (K=26 dry, K=26 moist ns=3, K=55 moist ns=6)"):
        return {"dry": jw_case(2562, K=26, ns=1),
                "moist": jw_case(2562, K=26, ns=3, moist=True),
                "moist55": jw_case(2562, K=55, ns=6, moist=True)}


def _variant_case(cases, name):
    key, cfg = VARIANTS[name]
    c = copy.copy(cases[key])
    c["config"] = dict(c["config"], **cfg)
    return c, MOIST_END[key]


def _gpu(case, moist_end, nsteps=NSTEPS):
    from mpas_dycore import Dycore
    dy = Dycore(case, device=0, moist_end=moist_end)
    dt = float(case["dt"])
    dy.init_diagnostics(dt)
    dy.use_graph(True)
    for it in range(nsteps):
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
    dy.synchronize()
    out = {key: dy.get(pool, name, 1) for pool, name, key, _ in PROG}
    dy.close()
    return out


def _reference(case, moist_end, nsteps=NSTEPS):
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    res, _ = ref_runner.run_reference(case, nsteps=nsteps, dt=float(case["dt"]), dump_steps=[nsteps],
                                      nthreads=16, moist_end=moist_end, dump_only=DUMP)
    return res[nsteps]


@pytest.mark.parametrize("name", list(VARIANTS))
def test_srk3_branch_matches_reference_10_steps(name, cases):
    c, me = _variant_case(cases, name)
    ref = _reference(c, me)
    got = _gpu(c, me)
    errs = {k: rel_linf(got[k].reshape(ref[k].shape), ref[k]) for k in got}
    progress(f"{name}: rel Linf {errs}")
    assert all(np.isfinite(list(errs.values())))
    bad = {k: v for k, v in errs.items() if not v <= (TOL if k in TIGHT else TOL_LOOSE)}
    assert not bad, f"{name}: {bad} (all {errs})"
    # the branch changes the trajectory (it is exercised, not skipped)
    if name != "L55_moist_ns6_mono":
        key = VARIANTS[name][0]
        if key not in _BASE:
            _BASE[key] = _gpu(cases[key], me)
        base = _BASE[key]
        changed = max(rel_linf(got[k], base[k]) for k in got)
        assert changed > 1e-9, f"{name}: option did not change the trajectory ({changed:.2e})"


def test_four_rccl_blocks_substeps6_bitwise(cases):
    from mpas_dycore import Dycore, decomp
    c, me = _variant_case(cases, "substeps6_order3")
    single = _gpu(c, me)
    blocks = decomp.decompose(c, decomp.partition_sfc(c["nCells"], 4))
    dy = Dycore.from_blocks(blocks, device=0, comm_id=Dycore.comm_unique_id(), nranks=1, rank=0,
                            rccl_local=True, moist_end=me)
    dy.set_overlap(True)
    dt = float(c["dt"])
    dy.init_diagnostics(dt)
    dy.use_graph(True)
    for it in range(NSTEPS):
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
    dy.synchronize()
    n_glob = {"cell": c["nCells"], "edge": c["nEdges"]}
    for pool, name, key, loc in PROG:
        per = [dy.get(pool, name, 1, block=i) for i in range(len(blocks))]
        got = decomp.gather_owned(blocks, per, loc, n_glob[loc])
        assert np.array_equal(got, single[key]), f"{key}: 4 RCCL blocks (n_sub=6) differ from one block"
    dy.close()
