"""GPU parity at BASELINE.json's own configurations (not just the small test meshes).

north_star bar: relative L-infinity <= 1e-10 on u / theta_m / rho_zz after 10 RK3 steps vs the
reference Fortran dycore on the same mesh and initial state.  The oracle is the unmodified
reference atm_srk3 (oracle/_ref/mpas_ref_harness, built from /root/reference by oracle/Makefile)
run on the GPU box's host cores on the same synthetic case.

  * configs[1]: x1.10242, 56 levels, dry JW, dt = 1440 s, one block -- and the same mesh as 4
    MPAS blocks whose halo exchanges go through RCCL (send/recv to self), which must also be
    bitwise equal to the one-block run (decomposition independence);
  * configs[3] species set at 56 levels: moist JW + tracer blobs, num_scalars = 6 (every
    scalar a moist species, as bench.py --moist), monotone split transport, on x1.2562.
"""
import numpy as np
import pytest

from conftest import rel_linf

pytestmark = pytest.mark.gpu

NSTEPS = 10
PROG = [("state", "u", "state.u.tl1", "edge"), ("state", "theta_m", "state.theta_m.tl1", "cell"),
        ("state", "rho_zz", "state.rho_zz.tl1", "cell"), ("state", "w", "state.w.tl1", "cell"),
        ("state", "scalars", "state.scalars.tl1", "cell")]
TOL = 1e-10          # u, theta_m, rho_zz (north_star)
TOL_LOOSE = 1e-9     # w and the tracer mixing ratios: small fields, error relative to their own max


def _reference(case, moist_end=1):
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    res, _ = ref_runner.run_reference(case, nsteps=NSTEPS, dt=float(case["dt"]), dump_steps=[NSTEPS],
                                      nthreads=16, moist_end=moist_end)
    return res[NSTEPS]


def _check(got, ref):
    errs = {key: rel_linf(got[key].reshape(ref[key].shape), ref[key]) for key in got}
    bad = {k: v for k, v in errs.items()
           if not v <= (TOL if k in ("state.u.tl1", "state.theta_m.tl1", "state.rho_zz.tl1") else TOL_LOOSE)}
    assert not bad, f"rel Linf above tolerance: {bad} (all: {errs})"
    return errs


def _run(dy, dt):
    dy.init_diagnostics(dt)
    dy.use_graph(True)
    for it in range(NSTEPS):
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
    dy.synchronize()


@pytest.fixture(scope="module")
def case10242():
    from mpas_dycore.cases import jw_case
    return jw_case(10242, K=56, ns=1, cache=False)


@pytest.fixture(scope="module")
def ref10242(case10242):
    return _reference(case10242)


@pytest.fixture(scope="module")
def single10242(case10242):
    from mpas_dycore import Dycore
    dy = Dycore(case10242, device=0)
    _run(dy, float(case10242["dt"]))
    out = {key: dy.get(pool, name, 1) for pool, name, key, _ in PROG}
    dy.close()
    return out


def test_configs1_x1_10242_L56_matches_reference(single10242, ref10242):
    _check(single10242, ref10242)


def test_configs1_x1_10242_L56_four_rccl_blocks(case10242, single10242, ref10242):
    from mpas_dycore import Dycore, decomp
    case = case10242
    blocks = decomp.decompose(case, decomp.partition_sfc(case["nCells"], 4))
    dy = Dycore.from_blocks(blocks, device=0, comm_id=Dycore.comm_unique_id(), nranks=1, rank=0, rccl_local=True)
    _run(dy, float(case["dt"]))
    n_glob = {"cell": case["nCells"], "edge": case["nEdges"]}
    got = {}
    for pool, name, key, loc in PROG:
        per = [dy.get(pool, name, 1, block=i) for i in range(len(blocks))]
        got[key] = decomp.gather_owned(blocks, per, loc, n_glob[loc])
    dy.close()
    for key in got:
        assert np.array_equal(got[key], single10242[key]), f"{key}: 4 RCCL blocks differ from one block"
    _check(got, {k: v for k, v in ref10242.items() if k in got})


def test_moist_ns6_x1_2562_L56_matches_reference():
    from mpas_dycore import Dycore
    from mpas_dycore.cases import jw_case
    case = jw_case(2562, K=56, ns=6, moist=True, cache=False)
    assert case["config"]["config_monotonic"]
    ref = _reference(case, moist_end=6)
    dy = Dycore(case, device=0, moist_end=6)
    _run(dy, float(case["dt"]))
    got = {key: dy.get(pool, name, 1) for pool, name, key, _ in PROG}
    dy.close()
    _check(got, ref)
