"""init_atm.py (the synthetic-case generator: the JW initial state and the model-init precompute)
pinned to the reference.

The fixtures in tests/golden/init_*.npz hold what the reference computes on our meshes (harness
mode 'init', tools/make_golden.py init): the unmodified core_init_atmosphere/mpas_atm_advection.F
(deriv_two, defc_a, defc_b) and mpas_atm_core.F:927-1288 (edge and vertex signs, kiteForCell,
adv_coefs compression, 3rd-order coupling, mesh scaling, dss).  Both the oracle and the product
consume init_atm's arrays, so without this pin a wrong restatement would pass every parity test.

Bars: index arrays and sign codes bit for bit; zb_cell / zb3_cell (copies), mesh scaling and dss
bit for bit; the least-squares / trigonometric weights (deriv_two, defc_a/b, adv_coefs,
adv_coefs_3rd) to 1e-14 relative to each array's largest entry -- they reach the reference's bits
except for last-place differences of sin/cos (numpy vs the Fortran runtime) that the ill-conditioned
fits carry to ~1e-15.

The JW initial state (tests/golden/jw_x1.642_K26.npz and a live run on x1.2562 x 55): the
reference's init_atm_case_jw (core_init_atmosphere/mpas_init_atm_cases.F:367-1312, with env_qv and
sphere_distance, harness mode 'jw') on the same grid given on the unit sphere.  Bars in _jw_compare.
The reference's JW is dry (its parameter moisture = .false., :454): init_atm's moist profile
(build_case(moist=True), the compiled-out branch restated) has no reference run to pin it.
"""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")
EXACT = ("edgesOnCell_sign", "edgesOnVertex_sign", "advCellsForEdge", "nAdvCellsForEdge", "kiteForCell",
         "meshScalingDel2", "meshScalingDel4", "dss", "zb_cell", "zb3_cell")
WEIGHTS = ("deriv_two", "defc_a", "defc_b", "adv_coefs", "adv_coefs_3rd")
TOL = 1e-14


def _cases():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    import make_golden
    return make_golden


def _compare(case, ref):
    nE, ME = case["nEdgesOnCell"], case["maxEdges"]
    cell_slot = np.arange(ME)[None, :] < nE[:, None]            # slots beyond nEdgesOnCell: never read
    adv_slot = np.arange(15)[None, :] < case["nAdvCellsForEdge"][:, None]
    errs = {}
    for k, b in ref.items():
        if k not in case:
            continue
        a = np.asarray(case[k])
        assert a.shape == b.shape, f"{k}: shape {a.shape} vs reference {b.shape}"
        if k in ("kiteForCell", "defc_a", "defc_b", "edgesOnCell_sign"):
            a, b = np.where(cell_slot, a, 0), np.where(cell_slot, b, 0)
        if k in ("advCellsForEdge", "adv_coefs", "adv_coefs_3rd"):
            a, b = np.where(adv_slot, a, 0), np.where(adv_slot, b, 0)
        if k in EXACT:
            assert np.array_equal(a, b), f"{k}: {int((a != b).sum())} entries differ from the reference"
            errs[k] = 0.0
        else:
            den = np.max(np.abs(b))
            errs[k] = float(np.max(np.abs(a - b)) / den) if den else float(np.max(np.abs(a - b)))
    bad = {k: v for k, v in errs.items() if k in WEIGHTS and not v <= TOL}
    assert not bad, f"above {TOL}: {bad}"
    assert set(WEIGHTS) <= set(errs)
    return errs


@pytest.mark.parametrize("fixture", ["init_x1.642_K8.npz", "init_varres2562_K8.npz"])
def test_init_matches_reference_fixture(fixture):
    mg = _cases()
    case = mg.INIT_CASES[fixture]()
    z = np.load(os.path.join(GOLD, fixture))
    assert str(z["checksum"]) == mg.init_inputs_checksum(case), "mesh generator changed: regenerate the fixture"
    _compare(case, {k: z[k] for k in z.files if k != "checksum"})


def test_init_matches_live_reference_x1_2562():
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    from mpas_dycore.cases import jw_case
    case = jw_case(2562, K=26, ns=1, cache=False)
    errs = _compare(case, ref_runner.run_reference_init(case))
    assert errs["zb_cell"] == 0.0 and errs["zb3_cell"] == 0.0


# ---- the JW initial state: core_init_atmosphere/mpas_init_atm_cases.F:367-1312 (init_atm_case_jw) ----
def _jw_compare(case, ref, ref_d2_case):
    """init_atm's JW state vs the reference's.  Bit for bit: the vertical grid and metrics and the
    base state; theta and rho to the last bit except at <= 0.02 % of the points (1 ulp).  u (the rebalanced wind) to 5e-14.  zb / zb3 bit for bit and w to 1e-13
    given the reference's deriv_two (ref_d2_case), since deriv_two's least-squares fits differ from
    the reference's in the last bit for ~0.2 % of the weights (test_init_matches_reference_fixture)
    and zb3 = dcEdge**2 * (d2 sum 1 - d2 sum 2) / 12 cancels."""
    from conftest import rel_linf
    own = {"mesh.zgrid": "zgrid", "mesh.zz": "zz", "mesh.zxu": "zxu", "mesh.rdzw": "rdzw", "mesh.rdzu": "rdzu",
           "mesh.fzm": "fzm", "mesh.fzp": "fzp", "mesh.cf1": "cf1", "mesh.cf2": "cf2", "mesh.cf3": "cf3",
           "diag.theta": "theta", "diag.rho": "rho", "diag.rho_base": "rho_base", "diag.theta_base": "theta_base"}
    for key, name in own.items():
        r = np.asarray(ref[key]).ravel()
        a = np.asarray(case[name], dtype=np.float64).ravel()[:r.size]
        if name in ("theta", "rho"):
            # the column iteration (mpas_init_atm_cases.F:862-950) reproduces the reference bit for
            # bit except at a few (latitude, level) points (theta 9, rho 19 of 140910 on x1.2562 x 55, 1 ulp)
            # whose cause is not located: every transcendental is the C library's there
            nd = int((a != r).sum())
            assert nd <= max(1, r.size // 5000), f"JW {name}: {nd} of {r.size} values differ"
            assert rel_linf(a, r) <= 1e-15, f"JW {name}: rel Linf {rel_linf(a, r):.3e}"
            continue
        assert np.array_equal(a, r), f"JW {name}: {int((a != r).sum())} of {r.size} values differ from the reference"
    u = rel_linf(np.asarray(case["u"]).reshape(ref["state.u.tl1"].shape), ref["state.u.tl1"])
    assert u <= 5e-14, f"JW u (rebalanced wind): rel Linf {u:.3e}"
    for name in ("zb", "zb3"):
        a = np.asarray(ref_d2_case[name]).reshape(ref["mesh." + name].shape)
        assert np.array_equal(a, ref["mesh." + name]), f"JW {name} (reference deriv_two) differs"
    w = rel_linf(np.asarray(ref_d2_case["w"]).reshape(ref["state.w.tl1"].shape), ref["state.w.tl1"])
    assert w <= 1e-13, f"JW w: rel Linf {w:.3e}"
    d2 = rel_linf(np.asarray(case["deriv_two"]).reshape(ref["mesh.deriv_two"].shape), ref["mesh.deriv_two"])
    assert d2 <= 1e-14
    return u, w


def test_jw_state_matches_reference_fixture():
    from mpas_dycore.init_atm import build_case
    mg = _cases()
    z = np.load(os.path.join(GOLD, "jw_x1.642_K26.npz"))
    m, unit, scaled = mg.jw_inputs()
    assert str(z["checksum"]) == mg.case_checksum(
        {**{k: v for k, v in m.items() if isinstance(v, np.ndarray)}, **unit}), "mesh generator changed: regenerate"
    ref = {k: z[k] for k in z.files if k != "checksum"}
    case = build_case({**m, **scaled}, K=26, ns=1)
    _jw_compare(case, ref, build_case({**m, **scaled, "deriv_two": ref["mesh.deriv_two"]}, K=26, ns=1))


def test_jw_state_matches_live_reference_x1_2562():
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    from mpas_dycore.init_atm import build_case
    m, unit, scaled = _cases().jw_inputs(level=4, K=55)
    case = build_case({**m, **scaled}, K=55, ns=1)
    ref = ref_runner.run_reference_jw(case, unit)
    _jw_compare(case, ref, build_case({**m, **scaled, "deriv_two": ref["mesh.deriv_two"]}, K=55, ns=1))
