"""GPU parity above 255 vertical levels: the library's fourth build (kernels.hip / dycore.hip with
MPAS_WIDE and WIDE_THREADS = 512), which api_dispatch.cpp selects for nVertLevels 256..511: every
kernel runs one column per 512-lane workgroup, lane = level, cross-level moves through LDS, and the
implicit w solve runs eight levels per lane of the first wavefront (column_solve, the same operands
as the sequential sweep).  nVertLevels is a namelist dimension of the reference
(core_init_atmosphere/Registry.xml:31,100) with no limit of its own.

  * K = 300 on x1.2562, 10 steps with the captured hipGraph, against the unmodified reference atm_srk3
    (oracle/_ref): relative L-infinity <= 1e-10 on u, theta_m, rho_zz, <= 1e-9 on w;
  * K = 300 on 4 MPAS blocks exchanging through the one-sided transfer: equal to one block bit for bit;
  * the general and batched kernel families give the same bits at K = 300 and at the largest, odd
    K = 511, moist monotone.
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
def case300():
    from mpas_dycore.cases import jw_case
    with heartbeat("building x1.2562 K=300"):
        return jw_case(2562, K=300, ns=1)


def _gpu(case, nsteps=NSTEPS):
    from mpas_dycore import Dycore
    dy = Dycore(case, device=0)
    assert dy.layout()["column"] == "wide512"
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


def test_wide512_matches_reference_10_steps(case300):
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    res, _ = ref_runner.run_reference(case300, nsteps=NSTEPS, dt=float(case300["dt"]), dump_steps=[NSTEPS], nthreads=16,
                                      dump_only=DUMP)
    ref = res[NSTEPS]
    got = _gpu(case300)
    errs = {k: rel_linf(got[k].reshape(ref[k].shape), ref[k]) for k in got}
    progress(f"K=300: rel Linf {errs}")
    assert all(np.isfinite(list(errs.values())))
    bad = {k: v for k, v in errs.items() if not v <= (TOL if k in TIGHT else TOL_LOOSE)}
    assert not bad, f"K=300: {bad} (all {errs})"


def test_wide512_four_blocks_bitwise(case300):
    from mpas_dycore import Dycore, decomp
    single = _gpu(case300, 3)
    blocks = decomp.decompose(case300, decomp.partition_sfc(case300["nCells"], 4))
    dy = Dycore.from_blocks(blocks, device=0, comm_id=Dycore.comm_unique_id(), nranks=1, rank=0, rccl_local=True,
                            p2p=True)
    dt = float(case300["dt"])
    dy.init_diagnostics(dt)
    dy.use_graph(True)
    for it in range(3):
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
    dy.synchronize()
    n_glob = {"cell": case300["nCells"], "edge": case300["nEdges"]}
    for pool, name, key, loc in PROG:
        per = [dy.get(pool, name, 1, block=i) for i in range(len(blocks))]
        got = decomp.gather_owned(blocks, per, loc, n_glob[loc])
        assert np.array_equal(got, single[key]), f"{key}: 4 blocks (K=300) differ from one block"
    dy.close()


@pytest.mark.parametrize("K", [300, 511])
def test_wide512_kernel_families_give_identical_bits(K):
    from mpas_dycore import Dycore
    from mpas_dycore.cases import jw_case
    with heartbeat(f"x1.642 K={K} moist, general vs batched"):
        case = jw_case(642, K=K, ns=2, moist=True, cache=False)
        outs = {}
        for fam in ("general", "batched"):
            saved = os.environ.get("MPAS_DYCORE_KERNELS")
            os.environ["MPAS_DYCORE_KERNELS"] = fam
            try:
                dy = Dycore(case, device=0, moist_end=2)
            finally:
                if saved is None:
                    os.environ.pop("MPAS_DYCORE_KERNELS")
                else:
                    os.environ["MPAS_DYCORE_KERNELS"] = saved
            lay = dy.layout()
            assert lay["family"] == fam and lay["column"] == "wide512", lay
            dt = float(case["dt"])
            dy.init_diagnostics(dt)
            dy.use_graph(True)
            for i in range(2):
                dy.atm_timestep(dt, i + 1)
                dy.shift_time_levels()
            dy.synchronize()
            outs[fam] = {n: dy.get("state", n, 1) for n in ("u", "w", "theta_m", "rho_zz", "scalars")}
            dy.close()
        for n in outs["general"]:
            assert np.isfinite(outs["general"][n]).all(), f"K={K}: {n} not finite"
            assert np.array_equal(outs["batched"][n], outs["general"][n]), f"K={K} batched: {n}"
