"""GPU parity above 63 vertical levels: the library's wide build (dycore.hip / kernels.hip with
MPAS_WIDE), which api_dispatch.cpp selects for nVertLevels 64..127.  Its pair-layout kernels give
one wavefront to a column, two levels per lane (the K <= 63 build's lane map and DPP moves, one
element per wavefront instead of two); its per-cell kernels one workgroup of 128 lanes, lane =
level, cross-level moves through LDS.  nVertLevels is a namelist dimension of the reference
(core_init_atmosphere/Registry.xml:31,100), which has no limit of its own.

  * K = 80 dry and K = 100 moist (num_scalars = 3, monotone transport) on x1.2562, 10 steps with
    the captured hipGraph, against the unmodified reference atm_srk3 (oracle/_ref):
    relative L-infinity <= 1e-10 on u, theta_m, rho_zz; <= 1e-9 on w and the mixing ratios;
  * K = 80 on 4 MPAS blocks, every halo message through RCCL with split-phase exchanges: equal
    to the one-block run bit for bit;
  * the three kernel families (general, batched, pair) give the same bits at K = 80 and at the
    largest, odd K = 127, moist monotone, as they do below 64 levels (test_gpu_kernels.py), and the
    default family there is the pair layout.
"""
import os

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


@pytest.fixture(scope="module")
def cases():
    from mpas_dycore.cases import jw_case
    with heartbeat("building x1.2562 cases (K=80 dry, K=100 moist ns=3)"):
        return {"K80": (jw_case(2562, K=80, ns=1), 1), "K100_moist": (jw_case(2562, K=100, ns=3, moist=True), 3)}


def _gpu(case, moist_end):
    from mpas_dycore import Dycore
    dy = Dycore(case, device=0, moist_end=moist_end)
    dt = float(case["dt"])
    dy.init_diagnostics(dt)
    dy.use_graph(True)
    for it in range(NSTEPS):
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
    dy.synchronize()
    out = {key: dy.get(pool, name, 1) for pool, name, key, _ in PROG}
    dy.close()
    return out


@pytest.mark.parametrize("name", ["K80", "K100_moist"])
def test_wide_columns_match_reference_10_steps(name, cases):
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    c, me = cases[name]
    res, _ = ref_runner.run_reference(c, nsteps=NSTEPS, dt=float(c["dt"]), dump_steps=[NSTEPS], nthreads=16,
                                      moist_end=me, dump_only=DUMP)
    ref = res[NSTEPS]
    got = _gpu(c, me)
    errs = {k: rel_linf(got[k].reshape(ref[k].shape), ref[k]) for k in got}
    progress(f"{name}: rel Linf {errs}")
    assert all(np.isfinite(list(errs.values())))
    bad = {k: v for k, v in errs.items() if not v <= (TOL if k in TIGHT else TOL_LOOSE)}
    assert not bad, f"{name}: {bad} (all {errs})"


def test_wide_columns_four_rccl_blocks_bitwise(cases):
    from mpas_dycore import Dycore, decomp
    c, me = cases["K80"]
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
        assert np.array_equal(got, single[key]), f"{key}: 4 RCCL blocks (K=80) differ from one block"
    dy.close()


def _steps_with_kernels(case, family, nsteps=2):
    from mpas_dycore import Dycore
    saved = os.environ.get("MPAS_DYCORE_KERNELS")
    os.environ["MPAS_DYCORE_KERNELS"] = family
    try:
        dy = Dycore(case, device=0, moist_end=case["num_scalars"])
    finally:
        if saved is None:
            os.environ.pop("MPAS_DYCORE_KERNELS")
        else:
            os.environ["MPAS_DYCORE_KERNELS"] = saved
    lay = dy.layout()
    dt = float(case["dt"])
    dy.init_diagnostics(dt)
    dy.use_graph(True)
    for i in range(nsteps):
        dy.atm_timestep(dt, i + 1)
        dy.shift_time_levels()
    dy.synchronize()
    out = {n: dy.get("state", n, 1) for n in ("u", "w", "theta_m", "rho_zz", "scalars")}
    out.update({n: dy.get("diag", n) for n in ("pv_edge", "rho_edge", "exner", "ru", "rw", "uReconstructZonal")})
    dy.close()
    return lay, out


@pytest.mark.parametrize("K", [80, 127])
def test_wide_kernel_families_give_identical_bits(K):
    from mpas_dycore.cases import jw_case
    with heartbeat(f"x1.642 K={K} moist, three kernel families"):
        case = jw_case(642, K=K, ns=2, moist=True, cache=False)
        lay, ref = _steps_with_kernels(case, "general")
        assert lay["family"] == "general" and lay["column"] == "wide"
        for fam in ("batched", "pair"):
            lay, got = _steps_with_kernels(case, fam)
            assert lay["family"] == fam and lay["column"] == "wide"
            for n in ref:
                assert np.array_equal(got[n], ref[n]), f"K={K} {fam}: {n}"
