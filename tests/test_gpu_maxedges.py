"""GPU: meshes that declare more neighbour slots than their cells use.

MPAS mesh files declare maxEdges = 10 and maxEdges2 = 20 ("the largest number of neighbors that a
primal mesh cell *may* have", core_atmosphere/Registry.xml:13-16) whatever the cells' actual
degree, and the reference never reads a slot past nEdgesOnCell / nEdgesOnEdge (its loops stop there;
edgesOnCell_sign is 0 beyond, mpas_atm_core.F:1025-1050).  The library keeps the Fortran images at
the declared strides and runs its kernels on copies at the mesh's own degree (dycore.hip pack_mesh),
so such a mesh must:
  * step to the same bits as the same mesh declared with maxEdges = 6 (or 7), through the Python
    host, an init file and the Fortran drop-in;
  * run the same kernel family (mpas_dyc_block_layout: pair layout, maxEdges 6 / 7);
  * be accepted for regional runs (they need the pair layout);
  * hand the declared images back unchanged through get_field.
Padding conventions: index -1 (0 in the file) or the row's last entry repeated.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import rel_linf

pytestmark = pytest.mark.gpu

PROG = ("u", "w", "theta_m", "rho_zz", "scalars")


def _run(case, nsteps=3, dt=None, lbc=None, moist_end=None):
    from mpas_dycore import Dycore
    from oracle import ref_runner
    dt = float(dt or (2880.0 if case["nCells"] <= 700 else case["dt"]))
    me = moist_end or case["num_scalars"]
    dy = Dycore(case, device=0, moist_end=me)
    if lbc is not None:  # as the drop-in does: LBCs on before the model init
        for (name, tl), img in ref_runner.lbc_images(case, lbc).items():
            dy.set_raw("lbc", name, img, tl)
        dy.set_lbc(True, lbc["interval_end"])
    dy.init_diagnostics(dt)
    dy.use_graph(True)
    for it in range(nsteps):
        if lbc is not None:
            dy.set_lbc(True, lbc["interval_end"] - it * dt)
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
    dy.synchronize()
    out = {n: dy.get("state", n, 1) for n in PROG}
    out["layout"] = dy.layout()
    out["graph"] = dy.graph_active()
    dy.close()
    return out


def _same(a, b, what):
    for n in PROG:
        assert np.array_equal(a[n], b[n]), f"{what}: {n} differs"


@pytest.mark.parametrize("fill", ["none", "repeat"])
def test_declared_max_edges_10_bitwise(moist_case, fill):
    from mpas_dycore.mesh import pad_max_edges
    a = _run(moist_case)
    b = _run(pad_max_edges(moist_case, 10, 20, fill))
    _same(a, b, f"maxEdges 10 / maxEdges2 20 ({fill})")
    assert a["layout"] == b["layout"] == {"maxEdges": 6, "maxEdges2": 10, "family": "pair", "column": "wavefront"}
    assert a["graph"] and b["graph"]


def test_declared_max_edges_10_wide_columns():
    """80 levels (the wide build) on a mesh declaring maxEdges 10: the same bits and the same pair
    layout as the maxEdges 6 declaration."""
    from mpas_dycore.cases import jw_case
    from mpas_dycore.mesh import pad_max_edges
    c = jw_case(642, K=80, ns=3, moist=True, cache=False)
    a = _run(c)
    b = _run(pad_max_edges(c, 10, 20, "none"))
    _same(a, b, "K = 80, maxEdges 10 / maxEdges2 20")
    assert a["layout"] == b["layout"] == {"maxEdges": 6, "maxEdges2": 10, "family": "pair", "column": "wide"}


def test_declared_max_edges_heptagons(varres_case_small):
    """The var-res SCVT holds pentagons to heptagons: its blocks run maxEdges 7 (the <7> / NE2 12
    instantiations), declared 10 or not."""
    from mpas_dycore.mesh import pad_max_edges
    c = dict(varres_case_small, dt=float(varres_case_small.get("dt", 2880.0)))
    assert c["maxEdges"] == 7 and (c["nEdgesOnCell"] == 7).any()
    a = _run(c, nsteps=2)
    b = _run(pad_max_edges(c, 10, 20, "repeat"), nsteps=2)
    _same(a, b, "var-res maxEdges 10")
    assert b["layout"]["maxEdges"] == 7 and b["layout"]["maxEdges2"] == 12 and b["layout"]["family"] == "pair"


def test_get_field_returns_declared_image(moist_case):
    """set_field / get_field / field_bytes speak the declared strides; the kernels' copies are
    internal.  Re-setting a packed mesh field after a step takes effect (the copy is redone)."""
    from mpas_dycore import Dycore
    from mpas_dycore.layout import to_fortran
    from mpas_dycore.mesh import pad_max_edges
    p = pad_max_edges(moist_case, 10, 20, "repeat")
    dy = Dycore(p, device=0, moist_end=3)
    lib, h = dy.lib, dy.h
    for name in ("edgesOnCell", "edgesOnEdge", "kiteForCell"):
        want = to_fortran(p, name)
        assert want.dtype == np.int32
        if name == "kiteForCell":  # a small 1-based index, not an element: values < 1 are stored as 1
            want = np.maximum(want, 1)
        nb = lib.mpas_dyc_field_bytes(h, b"mesh", name.encode())
        assert nb == want.nbytes, name
        got = np.empty(nb // 4, dtype=np.int32)
        assert lib.mpas_dyc_get_field(h, b"mesh", name.encode(), 1, got.ctypes.data_as(C.c_void_p), nb) == 0
        assert np.array_equal(got, want.ravel()), name
    for name in ("zb_cell", "weightsOnEdge", "coeffs_reconstruct"):
        want = np.ascontiguousarray(to_fortran(p, name), dtype=np.float64).ravel()
        assert np.array_equal(dy.get_raw("mesh", name), want), name
    dt = 2880.0
    dy.init_diagnostics(dt)
    dy.atm_timestep(dt, 1)
    dy.shift_time_levels()
    assert dy.layout()["maxEdges"] == 6
    # change a packed mesh field after a step: the kernels must see the new image
    dy.set("mesh", "zb_cell", 0.5 * np.asarray(p["zb_cell"]))
    dy.atm_timestep(dt, 2)
    dy.shift_time_levels()
    dy.synchronize()
    w_new = dy.get("state", "w", 1)
    dy.close()
    ref = Dycore(moist_case, device=0, moist_end=3)
    ref.init_diagnostics(dt)
    ref.atm_timestep(dt, 1)
    ref.shift_time_levels()
    ref.set("mesh", "zb_cell", 0.5 * np.asarray(moist_case["zb_cell"]))
    ref.atm_timestep(dt, 2)
    ref.shift_time_levels()
    ref.synchronize()
    assert np.array_equal(w_new, ref.get("state", "w", 1))
    ref.close()
    assert not np.array_equal(w_new, _run(moist_case, nsteps=2, dt=dt)["w"])


def test_declared_max_edges_init_file(moist_case, tmp_path):
    """An init file declaring maxEdges = 10 (read_init, then the model-init precompute at those
    strides) steps to the bits of the in-memory maxEdges = 6 case."""
    from mpas_dycore import mpas_files
    from mpas_dycore.mesh import pad_max_edges
    f = str(tmp_path / "x1.642.init.nc")
    mpas_files.write_init(f, pad_max_edges(moist_case, 10, 20, "none"), version=5)
    c = mpas_files.read_init(f, config=moist_case["config"])
    c["dt"] = moist_case["dt"]
    assert c["maxEdges"] == 10 and c["maxEdges2"] == 20
    _same(_run(moist_case), _run(c), "init file with maxEdges 10")


def test_declared_max_edges_regional():
    """Regional LBCs need the pair layout; a maxEdges = 10 mesh now gets it and runs to the bits of
    the maxEdges = 6 one (LBCs switched on before the model init, as the drop-in does)."""
    from mpas_dycore.cases import jw_case, regional_lbc
    from mpas_dycore.mesh import pad_max_edges
    case, lbc = regional_lbc(jw_case(2562, K=26, ns=6, moist=True, cache=False))
    a = _run(case, nsteps=3, lbc=lbc, moist_end=6)
    b = _run(pad_max_edges(case, 10, 20, "none"), nsteps=3, lbc=lbc, moist_end=6)
    _same(a, b, "regional, maxEdges 10")
    assert b["layout"]["family"] == "pair"


def test_declared_max_edges_dropin(moist_case):
    """The Fortran drop-in under the harness driver with the pools at maxEdges = 10 (what
    atm_time_integration_mi355x.F90 passes straight through from the mesh file) equals the Python
    host on the maxEdges = 6 case bit for bit, and the reference harness on the padded pools to the
    drop-in tests' tolerances."""
    from oracle import ref_runner
    from mpas_dycore import Dycore
    from mpas_dycore.mesh import pad_max_edges
    if not (ref_runner.available() and ref_runner.available(ref_runner.DROPIN_HARNESS)):
        pytest.skip("oracle/_ref harness binaries not built")
    dt, n = 2880.0, 3
    p = pad_max_edges(moist_case, 10, 20, "repeat")
    got, _ = ref_runner.run_reference(p, nsteps=n, dt=dt, dump_steps=[n], nthreads=1, moist_end=3,
                                      binary=ref_runner.DROPIN_HARNESS)
    ref, _ = ref_runner.run_reference(p, nsteps=n, dt=dt, dump_steps=[n], nthreads=4, moist_end=3)
    dy = Dycore(moist_case, device=0, moist_end=3)
    dy.init_diagnostics(dt)
    for it in range(n):
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
    dy.synchronize()
    for name in PROG:
        a = got[n][f"state.{name}.tl1"]
        assert np.array_equal(a, dy.get("state", name, 1).reshape(a.shape)), f"drop-in (maxEdges 10) {name}"
        err = rel_linf(a, ref[n][f"state.{name}.tl1"])
        assert err <= (1e-11 if name in ("w", "scalars") else 1e-12), f"{name} vs reference: {err:.3e}"
    dy.close()
