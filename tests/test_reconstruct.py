"""CPU: the numpy restatement of mpas_rbf_interp_initialize + mpas_init_reconstruct
(mpas_dycore/reconstruct.py) reproduces the reference's coefficients bit for bit
(golden fixture from the compiled reference, tools/make_golden.py reconstruct)."""
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reconstruct_x1.642.npz")


def test_init_reconstruct_matches_reference_bitwise():
    from mpas_dycore.cases import jw_case
    from mpas_dycore import reconstruct
    z = np.load(GOLD)
    case = jw_case(642, K=8, ns=1, cache=False)
    v = reconstruct.initialize_vectors(case)
    assert np.array_equal(v["edgeNormalVectors"], z["edgeNormalVectors"])
    assert np.array_equal(v["cellTangentPlane"], z["cellTangentPlane"])
    got = reconstruct.init_reconstruct(case, v)
    noc = case["nEdgesOnCell"]
    mask = np.arange(case["maxEdges"])[None, :] < noc[:, None]
    assert np.array_equal(got[mask], z["coeffs_reconstruct"][mask])
    assert np.all(got[~mask] == 0.0)


def test_reconstruct_of_solid_body_rotation_is_exact_to_rounding():
    """The RBF weights reproduce a tangential solid-body field at cell centres."""
    from mpas_dycore.mesh import build_mesh
    from mpas_dycore import reconstruct
    m = build_mesh(3, lloyd_iters=5)
    coef = reconstruct.init_reconstruct(m)
    xe = np.stack([m["xEdge"], m["yEdge"], m["zEdge"]], -1)
    om = np.array([0.0, 0.0, 1.0])
    vel_e = np.cross(om, xe)
    n = reconstruct.initialize_vectors(m)["edgeNormalVectors"]
    un = np.sum(vel_e * n, axis=-1)
    eoc, noc = m["edgesOnCell"], m["nEdgesOnCell"]
    mask = np.arange(m["maxEdges"])[None, :] < noc[:, None]
    rec = np.einsum("cij,ci->cj", coef * mask[:, :, None], np.where(mask, un[eoc], 0.0))
    xc = np.stack([m["xCell"], m["yCell"], m["zCell"]], -1)
    exact = np.cross(om, xc)
    assert np.max(np.abs(rec - exact)) / np.max(np.abs(exact)) < 2e-2
