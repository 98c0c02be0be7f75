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
The driver calls atm_timestep with its nowTime, so the xtime stamp (mpas_atm_time_integration.F:
127-137) is checked too.  The drop-in keeps the state in HBM and the driver calls
atm_dycore_to_host before each dump; MPAS_DYCORE_SYNC_EVERY_STEP=1 (the per-step copy-back)
must give the same bits.  Further cases: two blocks in one process (the domain context built from
domain%blocklist and the parinfo copy lists), and the -DDO_PHYSICS build (physics_get_tend on the
host, its tendencies into HBM every step) against the reference's DO_PHYSICS build.
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


def _runs(case, moist_end=1, nthreads_dropin=1, env=None):
    from oracle import ref_runner
    if not (ref_runner.available() and ref_runner.available(ref_runner.DROPIN_HARNESS)):
        pytest.skip("oracle/_ref harness binaries not built (make -C oracle all dropin)")
    ref, _ = ref_runner.run_reference(case, nsteps=NSTEPS, dt=DT, dump_steps=[0, NSTEPS], nthreads=4,
                                      moist_end=moist_end)
    got, _ = ref_runner.run_reference(case, nsteps=NSTEPS, dt=DT, dump_steps=[0, NSTEPS],
                                      nthreads=nthreads_dropin, moist_end=moist_end,
                                      binary=ref_runner.DROPIN_HARNESS, env_extra=env)
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
    # 3 OpenMP threads: the init calls come per thread, the one whose range starts at cell 1 works
    ref, got = _runs(case, nthreads_dropin=1 if moist else 3)
    assert got[NSTEPS]["state.xtime.tl1"] == ref[NSTEPS]["state.xtime.tl1"] == "2000-01-01_02:24:00"
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


def test_dropin_wide_columns_match_reference():
    """80 levels (the library's wide build, picked by nVertLevels behind the same Fortran API),
    moist ns = 3 with the monotone transport: the drop-in under the reference's driver against the
    reference, and bit for bit against the Python host."""
    from mpas_dycore.cases import jw_case
    case = jw_case(642, K=80, ns=3, moist=True, cache=False)
    ref, got = _runs(case, moist_end=3)
    errs = {k: rel_linf(got[NSTEPS][k], ref[NSTEPS][k]) for k in PROG + RECON}
    bad = {k: v for k, v in errs.items() if not v <= (1e-11 if k in LOOSE else 1e-12)}
    assert not bad, f"drop-in (K = 80) vs reference: {bad} (all {errs})"
    py = _python_host(case, moist_end=3)
    for k in PROG + RECON:
        a = got[NSTEPS][k]
        assert np.array_equal(a, py[k].reshape(a.shape)), f"{k}: drop-in differs from the Python host"


def test_dropin_sync_every_step_same_bits(small_case):
    """MPAS_DYCORE_SYNC_EVERY_STEP=1 (copy-back after every step) == on-demand atm_dycore_to_host."""
    from oracle import ref_runner
    if not ref_runner.available(ref_runner.DROPIN_HARNESS):
        pytest.skip("drop-in harness not built")
    runs = []
    for env in ({}, {"MPAS_DYCORE_SYNC_EVERY_STEP": "1"}):
        got, _ = ref_runner.run_reference(small_case, nsteps=NSTEPS, dt=DT, dump_steps=[1, NSTEPS], nthreads=1,
                                          binary=ref_runner.DROPIN_HARNESS, env_extra=env)
        runs.append(got)
    for step in (1, NSTEPS):
        for k in PROG + RECON + ["diag.pressure_p", "diag.exner", "diag.ru", "diag.pv_edge"]:
            assert np.array_equal(runs[0][step][k], runs[1][step][k]), f"step {step} {k}"


_N = {"cell": "nCells", "edge": "nEdges", "vertex": "nVertices"}
BLOCK_FIELDS = [("state.u.tl1", "edge"), ("state.theta_m.tl1", "cell"), ("state.rho_zz.tl1", "cell"),
                ("state.w.tl1", "cell"), ("diag.pv_edge", "edge"), ("diag.ru", "edge"), ("diag.rw", "cell"),
                ("diag.exner", "cell"), ("diag.uReconstructZonal", "cell")]


@pytest.mark.parametrize("nblocks", [2, 3])
def test_dropin_blocks_bitwise_one_block(nblocks):
    """The drop-in on several blocks of one process (its domain context from domain%blocklist, the
    exchange lists from parinfo % xToCopy) equals the one-block drop-in bit for bit on owned
    elements and halo layer 1, and the reference on the same blocks to the parity tolerances."""
    from mpas_dycore import decomp
    from mpas_dycore.cases import jw_case
    from oracle import ref_runner
    if not ref_runner.available(ref_runner.DROPIN_HARNESS):
        pytest.skip("drop-in harness not built")
    c = jw_case(642, K=26, ns=1, cache=False)
    blocks = decomp.decompose(c, decomp.partition_sfc(c["nCells"], nblocks))
    blocks.sort(key=lambda b: (-b.case["nCells"], -b.case["nEdges"]))  # reference: largest block first
    one, _ = ref_runner.run_reference(c, nsteps=NSTEPS, dt=DT, dump_steps=[0, NSTEPS], nthreads=1,
                                      binary=ref_runner.DROPIN_HARNESS)
    multi, _ = ref_runner.run_reference_blocks(c, blocks, nsteps=NSTEPS, dt=DT, dump_steps=[0, NSTEPS], nthreads=2,
                                               binary=ref_runner.DROPIN_HARNESS)
    ref, _ = ref_runner.run_reference_blocks(c, blocks, nsteps=NSTEPS, dt=DT, dump_steps=[NSTEPS], nthreads=4)
    for step in (0, NSTEPS):
        for key, loc in BLOCK_FIELDS:
            want_all = one[step][key].reshape((c[_N[loc]], -1))
            for ib, (m, b) in enumerate(zip(multi[step], blocks)):
                a = m[key].reshape((b.case[_N[loc]], -1))
                n1 = b.layer_end[loc][0 if "Reconstruct" in key else 1]
                got, want = a[:n1], want_all[b.glob[loc][:n1]]
                assert np.array_equal(got, want), f"step {step} {key} block {b.part}: {rel_linf(got, want):.3e}"
                if step == NSTEPS:
                    r = ref[step][ib][key].reshape((b.case[_N[loc]], -1))[:n1]
                    tol = 1e-11 if key in ("state.w.tl1", "diag.rw", "diag.uReconstructZonal") else 1e-12
                    assert rel_linf(got, r) <= tol, f"{key} block {b.part} vs reference: {rel_linf(got, r):.3e}"
        if step == NSTEPS:
            assert multi[step][0]["state.xtime.tl1"] == one[step]["state.xtime.tl1"]


@pytest.mark.parametrize("convection", ["cu_tiedtke", "off"])
def test_dropin_physics_matches_reference(convection):
    """The -DDO_PHYSICS drop-in (physics_get_tend on the host each step, tendencies into HBM, state
    back for the host physics) against the reference's DO_PHYSICS build, both with the prescribed
    tendencies of the physics_get_tend test double."""
    from conftest import physics_forcing
    from mpas_dycore.cases import jw_case
    from oracle import ref_runner
    if not (ref_runner.available(ref_runner.PHYS_HARNESS) and ref_runner.available(ref_runner.DROPIN_PHYS_HARNESS)):
        pytest.skip("physics harness binaries not built (make -C oracle phys dropin)")
    case = jw_case(642, K=26, ns=3, moist=True, cache=False)
    dt = float(case["dt"])
    phys = dict(physics_forcing(case), convection_scheme=convection)
    n = 6
    ref, _ = ref_runner.run_reference(case, n, dt, [1, n], nthreads=4, physics=phys)
    got, _ = ref_runner.run_reference(case, n, dt, [1, n], nthreads=1, physics=phys,
                                      binary=ref_runner.DROPIN_PHYS_HARNESS)
    keys = PROG + (["tend_physics.rqvdynten"] if convection != "off" else [])
    for step in (1, n):
        for k in keys:
            err = rel_linf(got[step][k], ref[step][k])
            assert err <= 1e-10, f"step {step} {k}: rel Linf {err:.3e}"
    assert got[n]["state.scalars.tl1"].min() >= 0.0


@pytest.mark.parametrize("moist", [False, True])
def test_dropin_regional_matches_reference(moist):
    """A regional run (config_apply_lbcs) through the drop-in: the boundary-zone masks go up with the
    mesh, the lbc pool whenever the host has read new boundary data, and before every step the
    seconds to the LBC interval end, read through mpas_atm_get_bdy_state (the reference's own
    getter; here the test double of oracle/shims, which the harness drives as the clock would).
    Against the reference run regionally by the same harness, 6 steps, at test_gpu_lbc's bars."""
    from mpas_dycore.cases import jw_case, regional_lbc
    from oracle import ref_runner
    if not (ref_runner.available() and ref_runner.available(ref_runner.DROPIN_HARNESS)):
        pytest.skip("oracle/_ref harness binaries not built (make -C oracle all dropin)")
    case0 = jw_case(2562, K=26, ns=6 if moist else 1, moist=moist, cache=False)
    case, lbc = regional_lbc(case0)
    dt, n, me = float(case["dt"]), 6, 6 if moist else 1
    ref, _ = ref_runner.run_reference(case, n, dt, [1, n], nthreads=4, lbc=lbc, moist_end=me)
    got, _ = ref_runner.run_reference(case, n, dt, [1, n], nthreads=1, lbc=lbc, moist_end=me,
                                      binary=ref_runner.DROPIN_HARNESS)
    for step in (1, n):
        for k in PROG:
            tol = 1e-9 if k in ("state.w.tl1", "state.scalars.tl1") else 1e-10
            err = rel_linf(got[step][k], ref[step][k])
            assert err <= tol, f"regional step {step} {k}: rel Linf {err:.3e}"
    # the boundary conditions act: the global drop-in run of the same state differs
    glob, _ = ref_runner.run_reference(case0, n, dt, [n], nthreads=1, moist_end=me, binary=ref_runner.DROPIN_HARNESS,
                                       dump_only=["state.theta_m"])
    assert np.isfinite(glob[n]["state.theta_m.tl1"]).all()
    assert rel_linf(glob[n]["state.theta_m.tl1"], got[n]["state.theta_m.tl1"]) > 1e-6


@pytest.mark.parametrize("regional", [False, True])
def test_dropin_microphysics_then_step_tail_matches_reference(regional):
    """-DDO_PHYSICS with a microphysics step (the test double of oracle/shims selected by
    config_microp_scheme = 'mp_test_double'): the reference runs it inside atm_srk3 (1650-1660) and
    only then resets the specified zone (1672-1790) and writes summarize_timestep's lines (1794).  The
    drop-in runs it on the host between mpas_dyc_timestep and mpas_dyc_finish_step, so the reset and
    the logged scalar extrema see the microphysics' theta_m / qv.  Prognostics at 1e-10 (w and the
    mixing ratios 1e-9) after 4 steps, and the logged global min/max lines equal to 1e-10."""
    import re
    from conftest import physics_forcing
    from mpas_dycore.cases import jw_case, regional_lbc
    from oracle import ref_runner
    if not (ref_runner.available(ref_runner.PHYS_HARNESS) and ref_runner.available(ref_runner.DROPIN_PHYS_HARNESS)):
        pytest.skip("physics harness binaries not built (make -C oracle phys dropin)")
    case = jw_case(2562, K=26, ns=3, moist=True, cache=False)
    lbc = None
    if regional:
        case, lbc = regional_lbc(case)
    dt, n = float(case["dt"]), 4
    phys = dict(physics_forcing(case, scale=0.2), microp_scheme="mp_test_double")
    kw = dict(nsteps=n, dt=dt, dump_steps=[n], physics=phys, lbc=lbc, moist_end=3, print_minmax=1 | 4)
    ref, _ = ref_runner.run_reference(case, nthreads=4, **kw)
    got, _ = ref_runner.run_reference(case, nthreads=1, binary=ref_runner.DROPIN_PHYS_HARNESS, **kw)
    for k in PROG:
        tol = 1e-9 if k in ("state.w.tl1", "state.scalars.tl1") else 1e-10
        err = rel_linf(got[n][k], ref[n][k])
        assert err <= tol, f"step {n} {k}: rel Linf {err:.3e}"
    # the microphysics test double really runs: without it the reference trajectory differs
    off, _ = ref_runner.run_reference(case, nthreads=4, **dict(kw, physics=dict(phys, microp_scheme="off")))
    assert rel_linf(off[n]["state.theta_m.tl1"], ref[n]["state.theta_m.tl1"]) > 1e-8
    num = r"(-?[0-9.]+(?:E[-+][0-9]+)?)"
    pat = re.compile(rf"global min, max (w|u|scalar\s+\d+) {num} {num}")
    lines_ref, lines_got = pat.findall(ref["log"]), pat.findall(got["log"])
    assert len(lines_ref) == n * (2 + 3) and len(lines_got) == len(lines_ref)
    for a, b in zip(lines_ref, lines_got):
        assert a[0] == b[0]
        for x, y in ((a[1], b[1]), (a[2], b[2])):
            x, y = float(x), float(y)
            assert abs(x - y) <= 1e-10 * abs(x) + 1e-300, f"{a[0]}: {x} vs {y}"
