"""GPU parity on a variable-resolution mesh (BASELINE.json configs[4] analogue).

The mesh is a 4x-refined SCVT with 2562 cells. It has pentagons, hexagons and
heptagons, so maxEdges = 7 and maxEdges2 = 14. That exercises:
  * the non-hexagon paths of every kernel;
  * the mesh-density scaling of the filters.
The run is moist with monotone transport. Its reference is the live oracle.
Decomposing it gives irregular halos, and the result must still be bitwise equal
to a single block.
"""
import numpy as np
import pytest

from conftest import rel_linf

pytestmark = pytest.mark.gpu

KEYS = [("state", "u", "state.u.tl1"), ("state", "theta_m", "state.theta_m.tl1"),
        ("state", "rho_zz", "state.rho_zz.tl1"), ("state", "w", "state.w.tl1"),
        ("state", "scalars", "state.scalars.tl1")]


def test_varres_mesh_is_irregular(varres_case_small):
    c = varres_case_small
    counts = np.bincount(c["nEdgesOnCell"])
    assert c["maxEdges"] == 7 and counts[7] > 0 and counts[5] > 0


@pytest.mark.parametrize("nsteps,tol,wtol", [(1, 1e-12, 1e-10), (10, 1e-10, 1e-9)])
def test_varres_matches_reference(varres_case_small, nsteps, tol, wtol):
    from mpas_dycore import Dycore
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    c = varres_case_small
    dt = c["dt"]
    res, _ = ref_runner.run_reference(c, nsteps=nsteps, dt=dt, dump_steps=[nsteps], nthreads=4, moist_end=3)
    ref = res[nsteps]
    dy = Dycore(c, device=0, moist_end=3)
    dy.init_diagnostics(dt)
    for it in range(nsteps):
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
    dy.synchronize()
    errs = {k: rel_linf(dy.get(p, n, 1).reshape(ref[k].shape), ref[k]) for p, n, k in KEYS}
    dy.close()
    bad = {k: v for k, v in errs.items() if not v <= (wtol if k == "state.w.tl1" else tol)}
    assert not bad, f"{bad} (all {errs})"


def test_varres_decomposition_bitwise(varres_case_small):
    from mpas_dycore import Dycore, decomp
    c = varres_case_small
    dt = c["dt"]

    def run(dy):
        dy.init_diagnostics(dt)
        for it in range(3):
            dy.atm_timestep(dt, it + 1)
            dy.shift_time_levels()
        dy.synchronize()

    one = Dycore(c, device=0, moist_end=3)
    run(one)
    ref = {n: one.get(p, n, 1) for p, n, _ in KEYS}
    one.close()
    blocks = decomp.decompose(c, decomp.partition_sfc(c["nCells"], 5))
    dy = Dycore.from_blocks(blocks, device=0, moist_end=3)
    dy.set_overlap(True)
    run(dy)
    for p, n, _ in KEYS:
        loc = "edge" if n == "u" else "cell"
        got = decomp.gather_owned(blocks, [dy.get(p, n, 1, block=i) for i in range(len(blocks))], loc,
                                  c["nEdges"] if loc == "edge" else c["nCells"])
        assert np.array_equal(got, ref[n]), n
    dy.close()
