"""GPU: the model-init precompute on the device (mpas_dyc_model_init: atm_compute_signs,
atm_adv_coef_compression, atm_couple_coef_3rd_order, atm_compute_mesh_scaling,
atm_compute_damping_coefs and the inverses of atm_mpas_init_block, mpas_atm_core.F:311-358, 927-1288).

Checked against the reference's own outputs on our meshes (tests/golden/init_*.npz, the unmodified
mpas_atm_core.F run by the harness) and against init_atm.model_init (the host restatement):
  * signs, kiteForCell, advCellsForEdge, nAdvCellsForEdge: bit for bit;
  * adv_coefs / adv_coefs_3rd: bit for bit (the compression is pure arithmetic on deriv_two, which
    init_atm computes to the reference's bits, tests/test_init_pinned.py);
  * zb_cell / zb3_cell (copies of zb / zb3 times config_coef_3rd_order), inverses: bit for bit vs host;
  * meshScalingDel2 / Del4, dss: bit for bit when the host hands in the C library's x**0.25 and sin
    (Dycore(model_init="device"), init_atm.model_init_libm: what the compiled reference computes);
    without them (model_init="device_cr") the device's correctly rounded values (checked against a
    60-digit evaluation here), which differ where the reference's C library does not round x**0.25 or
    sin correctly: 1 ulp in the root / sine, so at most 2 ulp in meshScalingDel2 and 4 ulp in dss.
Then a model run from the device-initialised mesh equals the host-initialised one bit for bit."""
import math
from decimal import Decimal, getcontext

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

getcontext().prec = 60


def cr_root4(x: float) -> float:
    """x**0.25, correctly rounded (Decimal's sqrt is exact to 60 digits; float() rounds to nearest)."""
    return float(Decimal(x).sqrt().sqrt())


def cr_sin(x: float) -> float:
    x = Decimal(x)
    s, term, k = Decimal(0), x, 1
    while abs(term) > Decimal(10) ** -58:
        s += term
        term = -term * x * x / ((2 * k) * (2 * k + 1))
        k += 1
    return float(s)


def _cases():
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    import make_golden
    return make_golden


def _device(case, fields, mode="device"):
    from mpas_dycore import Dycore
    dy = Dycore(case, device=0, model_init=mode)
    out = {}
    for n in fields:
        nb = dy.lib.mpas_dyc_field_bytes(dy.h, b"mesh", n.encode())
        if n in ("kiteForCell", "advCellsForEdge", "nAdvCellsForEdge"):
            import ctypes as C
            buf = np.empty(nb // 4, dtype=np.int32)
            assert dy.lib.mpas_dyc_get_field(dy.h, b"mesh", n.encode(), 1, buf.ctypes.data_as(C.c_void_p), nb) == 0
            out[n] = buf
        else:
            out[n] = dy.get_raw("mesh", n)
    dy.close()
    return out


def _expected_scaling(case):
    """meshScalingDel2 / Del4 / Regional and dss as the reference writes them, with correctly rounded
    pow / sin, and a mask of where that differs from the C library's result."""
    cfg = case["config"]
    md = np.asarray(case["meshDensity"], dtype=np.float64)
    coe = np.asarray(case["cellsOnEdge"])
    x = (md[coe[:, 0]] + md[coe[:, 1]]) / 2.0
    r4 = np.array([cr_root4(v) for v in x])
    lib4 = np.array([math.pow(v, 0.25) for v in x])
    d2 = 1.0 / r4
    d4 = 1.0 / (np.sqrt(x) * np.sqrt(np.sqrt(x)))
    zg = np.asarray(case["zgrid"])
    K = zg.shape[1] - 1
    zd, xn = float(cfg["config_zd"]), float(cfg["config_xnutr"])
    pii = math.acos(-1.0)
    dss = np.zeros((zg.shape[0], K))
    dss_lib = np.zeros_like(dss)
    for c in range(zg.shape[0]):
        zt = zg[c, K]
        mr, ml = cr_root4(md[c]), math.pow(md[c], 0.25)
        for k in range(K):
            z = 0.5 * (zg[c, k] + zg[c, k + 1])
            if z > zd:
                a = 0.5 * pii * (z - zd) / (zt - zd)
                s, sl = cr_sin(a), math.sin(a)
                dss[c, k] = xn * (s * s) / mr
                dss_lib[c, k] = xn * (sl * sl) / ml
    reg_c = 1.0 / np.array([cr_root4(v) for v in md])
    return dict(meshScalingDel2=d2, meshScalingDel4=d4, meshScalingRegionalEdge=d2, meshScalingRegionalCell=reg_c,
                dss=dss), dict(meshScalingDel2=r4 != lib4, dss=dss != dss_lib)


@pytest.mark.parametrize("mode", ["device", "device_cr"])
@pytest.mark.parametrize("fixture", ["init_x1.642_K8.npz", "init_varres2562_K8.npz"])
def test_model_init_matches_reference(fixture, mode):
    import os
    from mpas_dycore.layout import to_fortran
    mg = _cases()
    case = mg.INIT_CASES[fixture]()
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", fixture))
    assert str(z["checksum"]) == mg.init_inputs_checksum(case), "mesh generator changed: regenerate the fixture"
    ref = {k: z[k] for k in z.files if k != "checksum"}
    nC, nE, ME = case["nCells"], case["nEdges"], case["maxEdges"]
    K = case["nVertLevels"]
    # init_atm's deriv_two is the reference's, bit for bit (test_init_pinned.py)
    assert np.array_equal(np.asarray(case["deriv_two"]).reshape(ref["deriv_two"].shape), ref["deriv_two"])
    c = case
    names = ("edgesOnCell_sign", "edgesOnVertex_sign", "kiteForCell", "advCellsForEdge", "nAdvCellsForEdge",
             "adv_coefs", "adv_coefs_3rd", "meshScalingDel2", "meshScalingDel4", "meshScalingRegionalEdge",
             "meshScalingRegionalCell", "dss", "zb_cell", "zb3_cell", "invAreaCell", "invDvEdge", "invDcEdge",
             "invAreaTriangle")
    got = _device(c, names, mode)
    noc = np.asarray(case["nEdgesOnCell"])
    slot = np.arange(ME)[None, :] < noc[:, None]
    nadv = np.asarray(ref["nAdvCellsForEdge"])
    aslot = np.arange(15)[None, :] < nadv[:, None]
    g = {k: v.reshape(-1) for k, v in got.items()}
    # index / sign arrays
    assert np.array_equal(g["nAdvCellsForEdge"][:nE], nadv)
    adv = g["advCellsForEdge"].reshape(nE + 1, 15)[:nE] - 1
    assert np.array_equal(np.where(aslot, adv, 0), np.where(aslot, ref["advCellsForEdge"], 0))
    for n in ("edgesOnCell_sign", "kiteForCell"):
        a = g[n].reshape(nC + 1, ME)[:nC]
        if n == "kiteForCell":
            a = a - 1  # Fortran 1-based -> the fixture's 0-based
        assert np.array_equal(np.where(slot, a, 0), np.where(slot, ref[n], 0)), n
    assert np.array_equal(g["edgesOnVertex_sign"].reshape(-1, 3)[:-1], ref["edgesOnVertex_sign"])
    for n in ("adv_coefs", "adv_coefs_3rd"):
        a = g[n].reshape(nE + 1, 15)[:nE]
        assert np.array_equal(np.where(aslot, a, 0), np.where(aslot, ref[n], 0)), f"{n} not bit for bit"
    if mode == "device":  # the C library's x**0.25 and sin from the host: every output is the reference's
        from mpas_dycore.init_atm import model_init_libm
        for n in ("meshScalingDel2", "meshScalingDel4"):
            assert np.array_equal(g[n][:nE], np.asarray(ref[n])), f"{n} not bit for bit"
        # the regional scalings (mpas_atm_core.F:979-982): the same 1 / x**0.25 as Del2, and per cell
        assert np.array_equal(g["meshScalingRegionalEdge"][:nE], np.asarray(ref["meshScalingDel2"]))
        assert np.array_equal(g["meshScalingRegionalCell"][:nC],
                              1.0 / model_init_libm(case, case["config"])["meshDensity_root4"])
        assert np.array_equal(g["dss"].reshape(nC + 1, K)[:nC], np.asarray(ref["dss"])), "dss not bit for bit"
        return
    # pow / sin outputs: the correctly rounded values; the reference's where its C library rounds right
    want, lib_off = _expected_scaling(case)
    for n in ("meshScalingDel2", "meshScalingDel4", "meshScalingRegionalEdge"):
        assert np.array_equal(g[n][:nE], want[n]), n
    assert np.array_equal(g["meshScalingRegionalCell"][:nC], want["meshScalingRegionalCell"])
    dss = g["dss"].reshape(nC + 1, K)[:nC]
    assert np.array_equal(dss, want["dss"])
    for n, a in (("meshScalingDel2", g["meshScalingDel2"][:nE]), ("meshScalingDel4", g["meshScalingDel4"][:nE]),
                 ("dss", dss)):
        off = lib_off.get(n, np.zeros(a.shape, bool))
        assert np.array_equal(a[~off], np.asarray(ref[n])[~off]), f"{n} differs from the reference where libm is exact"
        if off.any():
            # 1 ulp in the root: <= 2 ulp in its reciprocal; 1 ulp in the sine, squared, and the root:
            # <= 4 ulp in dss = xnutr sin^2 / root
            ulp = np.spacing(np.abs(np.asarray(ref[n])[off]))
            assert np.all(np.abs(a[off] - np.asarray(ref[n])[off]) <= (4 if n == "dss" else 2) * ulp), n
    # the copies and inverses: what the host restatement computes
    zb = np.asarray(case["zb_cell"]).reshape(nC, ME, K + 1)
    z3 = np.asarray(case["zb3_cell"]).reshape(nC, ME, K + 1)
    s3 = slot[:, :, None]
    assert np.array_equal(np.where(s3, g["zb_cell"].reshape(nC + 1, ME, K + 1)[:nC], 0), np.where(s3, zb, 0))
    assert np.array_equal(np.where(s3, g["zb3_cell"].reshape(nC + 1, ME, K + 1)[:nC], 0), np.where(s3, z3, 0))
    for n in ("invAreaCell", "invDvEdge", "invDcEdge", "invAreaTriangle"):
        want_inv = np.asarray(to_fortran(case, n)).reshape(-1)
        assert np.array_equal(g[n][:-1], want_inv[:-1]), n


def test_model_run_from_device_init(moist_case):
    """A moist run whose mesh precompute came from mpas_dyc_model_init (with the host's C-library x**0.25 and
    sin, Dycore(model_init="device")): every precomputed array and the run equal the host-initialised ones
    bit for bit."""
    from mpas_dycore import Dycore
    case = moist_case
    dt = 2880.0
    runs = []
    for mode in ("host", "device"):
        dy = Dycore(case, device=0, moist_end=3, model_init=mode)
        mesh = {n: dy.get_raw("mesh", n) for n in ("adv_coefs", "adv_coefs_3rd", "zb3_cell", "dss", "meshScalingDel2",
                                                    "meshScalingDel4", "edgesOnCell_sign", "invDcEdge",
                                                    "coeffs_reconstruct")}
        dy.init_diagnostics(dt)
        dy.use_graph(True)
        for it in range(3):
            dy.atm_timestep(dt, it + 1)
            dy.shift_time_levels()
        dy.synchronize()
        runs.append((mesh, {n: dy.get("state", n, 1) for n in ("u", "w", "theta_m", "rho_zz", "scalars")}))
        dy.close()
    (m0, s0), (m1, s1) = runs
    for n in m0:
        assert np.array_equal(m0[n], m1[n]), f"{n}: device model init differs from the host's"
    for n in s0:
        assert np.array_equal(s0[n], s1[n]), n


@pytest.mark.parametrize("fixture", ["init_x1.642_K8.npz", "init_varres2562_K8.npz"])
def test_deriv_two_on_device_matches_reference(fixture):
    """deriv_two's least-squares fits on the device (mpas_dyc_init_deriv_two: amatrix, poly_fit_2 with
    MIGS / ELGS and the edge weights of mpas_atm_advection.F:215-358, 567-741), from the C library's
    tangent-plane coordinates and edge angles (init_atm.deriv_two_inputs): bit for bit the reference's
    deriv_two; and the device model init run on it gives the reference's adv_coefs bit for bit."""
    import os
    from mpas_dycore import Dycore, init_atm
    mg = _cases()
    case = mg.INIT_CASES[fixture]()
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", fixture))
    assert str(z["checksum"]) == mg.init_inputs_checksum(case), "mesh generator changed: regenerate the fixture"
    nE = case["nEdges"]
    dy = Dycore(case, device=0, model_init="device")
    try:
        dy.init_deriv_two(init_atm.deriv_two_inputs(case))
        got = dy.get_raw("mesh", "deriv_two").reshape(nE + 1, 2, 15)
        assert np.array_equal(got[:nE], z["deriv_two"]), \
            f"{int((got[:nE] != z['deriv_two']).sum())} deriv_two weights differ from the reference"
        assert not got[nE].any()
        cfg = case["config"]
        dy._check(dy.lib.mpas_dyc_model_init(dy.h, int(bool(cfg.get("config_h_ScaleWithMesh", True))),
                                             float(cfg["config_zd"]), float(cfg["config_xnutr"])), "model_init")
        aslot = np.arange(15)[None, :] < np.asarray(z["nAdvCellsForEdge"])[:, None]
        for n in ("adv_coefs", "adv_coefs_3rd"):
            a = dy.get_raw("mesh", n).reshape(nE + 1, 15)[:nE]
            assert np.array_equal(np.where(aslot, a, 0), np.where(aslot, z[n], 0)), n
    finally:
        dy.close()


def test_deriv_two_on_device_refuses_bad_inputs(moist_case):
    import ctypes as C
    from mpas_dycore import Dycore
    dy = Dycore(moist_case, device=0)
    try:
        with pytest.raises(ValueError):
            dy.init_deriv_two([np.zeros((3, 3))] * 4)
        assert dy.lib.mpas_dyc_init_deriv_two(dy.h, 5, *[C.c_void_p(1)] * 4) == -1  # no block 5
        assert dy.lib.mpas_dyc_init_deriv_two(dy.h, 0, None, None, None, None) == -1
    finally:
        dy.close()


def test_init_chain_on_device_matches_reference_jw():
    """The init core's arithmetic on the device, chained: deriv_two's fits (mpas_dyc_init_deriv_two) and
    zb / zb3 (mpas_dyc_init_zb, mpas_init_atm_cases.F:1045-1093) from the C library's angles and the JW
    vertical grid, against the reference's init_atm_case_jw on x1.642 x 26 (tests/golden/jw_x1.642_K26.npz):
    bit for bit."""
    import os
    from mpas_dycore import Dycore, init_atm
    mg = _cases()
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "jw_x1.642_K26.npz"))
    m, unit, scaled = mg.jw_inputs()
    assert str(z["checksum"]) == mg.case_checksum(
        {**{k: v for k, v in m.items() if isinstance(v, np.ndarray)}, **unit}), "mesh generator changed: regenerate"
    case = init_atm.build_case({**m, **scaled}, K=26, ns=1)
    nE, K = case["nEdges"], case["nVertLevels"]
    dy = Dycore(case, device=0, model_init="device")
    try:
        dy.init_deriv_two(init_atm.deriv_two_inputs(case))
        dy.init_zb(3)
        for name, n_per in (("deriv_two", 30), ("zb", 2 * (K + 1)), ("zb3", 2 * (K + 1))):
            got = dy.get_raw("mesh", name)[:nE * n_per]
            ref = np.asarray(z["mesh." + name]).ravel()[:nE * n_per]
            assert np.array_equal(got, ref), f"{name}: {int((got != ref).sum())} of {got.size} differ from the reference"
        with pytest.raises(Exception):
            dy.init_zb(5)
    finally:
        dy.close()


def test_reconstruct_coefficients_on_device_match_reference():
    """mpas_dyc_init_reconstruct (mpas_rbf_interp_initialize's vectors + mpas_init_reconstruct,
    mpas_atm_core.F:408-409, run by Dycore(model_init="device")): coeffs_reconstruct bit for bit the
    reference's on x1.642 (tests/golden/reconstruct_x1.642.npz), and equal to the host restatement
    (reconstruct.py) on the var-res mesh with pentagons and heptagons."""
    import os
    from mpas_dycore import Dycore, reconstruct
    from mpas_dycore.cases import jw_case
    mg = _cases()
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "reconstruct_x1.642.npz"))
    case = jw_case(642, K=8, ns=1, cache=False)
    # the fixture's geometry is this mesh's (tests/test_reconstruct.py: the host vectors equal its own)
    assert np.array_equal(reconstruct.initialize_vectors(case)["edgeNormalVectors"], z["edgeNormalVectors"])
    cases = [(case, z["coeffs_reconstruct"]), (mg.INIT_CASES["init_varres2562_K8.npz"](), None)]
    for c, ref in cases:
        nC, ME = c["nCells"], c["maxEdges"]
        if ref is None:
            ref = reconstruct.init_reconstruct(c)
            assert (np.asarray(c["nEdgesOnCell"]) != 6).any()
        dy = Dycore(c, device=0, model_init="device")
        try:
            got = dy.get_raw("mesh", "coeffs_reconstruct").reshape(nC + 1, ME, 3)[:nC]
        finally:
            dy.close()
        mask = np.arange(ME)[None, :] < np.asarray(c["nEdgesOnCell"])[:, None]
        assert np.array_equal(got[mask], ref[mask]), f"{int((got[mask] != ref[mask]).sum())} coefficients differ"
        assert np.all(got[~mask] == 0.0)
