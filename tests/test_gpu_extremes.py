"""GPU parity at the ends of the supported ranges, against the unmodified reference atm_srk3
(oracle/_ref, the harness on the box's host cores).

nVertLevels is a namelist dimension of the reference (core_init_atmosphere/Registry.xml:31,100) and
the library takes 4..127: the smallest column (K = 4: the pair layout's two lane pairs, the
w-recovery's three-level bottom extrapolation cf1..cf3 on a 4-level column), the largest
one-wavefront column (K = 63, odd: the last lane pair holds one level), the smallest and the
largest wide columns (K = 64, K = 127: one wavefront per column in the pair kernels, a 128-lane
workgroup in the per-cell kernels), and the smallest icosahedral mesh the case builder makes (x1.162,
12 pentagons among 162 cells).  Every case runs in the default (pair) kernel family, moist monotone
where marked, with the captured hipGraph.  Bars: the parity tests' (rel Linf <= 1e-10 on u, theta_m,
rho_zz; <= 1e-9 on w and the mixing ratios).
"""
import numpy as np
import pytest

from conftest import progress, rel_linf

pytestmark = pytest.mark.gpu

PROG = [("state", "u", "state.u.tl1"), ("state", "theta_m", "state.theta_m.tl1"),
        ("state", "rho_zz", "state.rho_zz.tl1"), ("state", "w", "state.w.tl1"),
        ("state", "scalars", "state.scalars.tl1")]
DUMP = ["state.u", "state.theta_m", "state.rho_zz", "state.w", "state.scalars"]
TIGHT = ("state.u.tl1", "state.theta_m.tl1", "state.rho_zz.tl1")


@pytest.mark.parametrize("ncells,K,ns,nsteps", [(642, 4, 1, 3), (642, 63, 3, 3), (642, 64, 3, 3), (642, 127, 1, 2),
                                                (162, 26, 3, 3)])
def test_extreme_sizes_match_reference(ncells, K, ns, nsteps):
    from mpas_dycore import Dycore
    from mpas_dycore.cases import jw_case
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    moist = ns > 1
    case = jw_case(ncells, K=K, ns=ns, moist=moist, cache=False)
    dt = float(case["dt"])
    res, _ = ref_runner.run_reference(case, nsteps=nsteps, dt=dt, dump_steps=[nsteps], nthreads=16, moist_end=ns,
                                      dump_only=DUMP)
    ref = res[nsteps]
    dy = Dycore(case, device=0, moist_end=ns)
    lay = dy.layout()
    assert lay["family"] == "pair" and lay["column"] == ("wide" if K > 63 else "wavefront"), lay
    dy.init_diagnostics(dt)
    dy.use_graph(True)
    for it in range(nsteps):
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
    dy.synchronize()
    got = {key: dy.get(pool, name, 1) for pool, name, key in PROG}
    dy.close()
    errs = {k: rel_linf(got[k].reshape(ref[k].shape), ref[k]) for k in got}
    progress(f"x1.{ncells} K={K} ns={ns}: rel Linf {errs}")
    assert all(np.isfinite(list(errs.values())))
    bad = {k: v for k, v in errs.items() if not v <= (1e-10 if k in TIGHT else 1e-9)}
    assert not bad, f"{bad} (all {errs})"
