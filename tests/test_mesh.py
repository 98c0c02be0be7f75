"""Mesh generator: MPAS conventions the dycore relies on."""
import numpy as np
import pytest

from mpas_dycore.mesh import build_mesh, _normalize


@pytest.fixture(scope="module", params=[2, 3])
def mesh(request):
    return build_mesh(request.param, lloyd_iters=20)


def _xyz(m, what):
    R = m["sphere_radius"]
    return np.stack([m["x" + what], m["y" + what], m["z" + what]], 1) / R


def test_counts_and_euler(mesh):
    nC, nE, nV = mesh["nCells"], mesh["nEdges"], mesh["nVertices"]
    r = {162: 2, 642: 3}[nC]
    assert (nC, nE, nV) == (10 * 4 ** r + 2, 30 * 4 ** r, 20 * 4 ** r)
    assert nC - nE + nV == 2
    assert np.bincount(mesh["nEdgesOnCell"])[5] == 12          # 12 pentagons, rest hexagons
    assert (mesh["nEdgesOnCell"] >= 5).all() and (mesh["nEdgesOnCell"] <= 6).all()


def test_areas_tile_the_sphere(mesh):
    R = mesh["sphere_radius"]
    A = 4 * np.pi * R * R
    assert abs(mesh["areaCell"].sum() / A - 1) < 1e-12
    assert abs(mesh["areaTriangle"].sum() / A - 1) < 1e-12
    assert np.allclose(mesh["kiteAreasOnVertex"].sum(1), mesh["areaTriangle"], rtol=1e-12)
    assert (mesh["kiteAreasOnVertex"] > 0).all()


def test_edge_orientation_conventions(mesh):
    xc, xv, xe = _xyz(mesh, "Cell"), _xyz(mesh, "Vertex"), _xyz(mesh, "Edge")
    c1, c2 = mesh["cellsOnEdge"].T
    v1, v2 = mesh["verticesOnEdge"].T
    n = xc[c2] - xc[c1]
    t = np.cross(xe, n)
    assert (np.sum((xv[v2] - xv[v1]) * t, 1) > 0).all()       # vertex 2 left of the normal
    # edgesOnCell(i) joins verticesOnCell(i) and verticesOnCell(i+1); cellsOnCell(i) across it
    for c in range(mesh["nCells"]):
        ne = mesh["nEdgesOnCell"][c]
        for i in range(ne):
            e = mesh["edgesOnCell"][c, i]
            assert {mesh["verticesOnCell"][c, i], mesh["verticesOnCell"][c, (i + 1) % ne]} == set(mesh["verticesOnEdge"][e])
            assert set(mesh["cellsOnEdge"][e]) == {c, mesh["cellsOnCell"][c, i]}


def test_trisk_weights(mesh, min_dv_dc=0.0):
    """Thuburn et al. (2009): v accuracy for solid-body rotation and energy antisymmetry.
    min_dv_dc: the accuracy bar applies to edges at least that long relative to dcEdge (the
    variable-resolution mesh opens its near-degenerate edges only to 5 % of dcEdge, where the
    reconstruction is less accurate; the antisymmetry is exact everywhere)."""
    xc, xe = _xyz(mesh, "Cell"), _xyz(mesh, "Edge")
    c1, c2 = mesh["cellsOnEdge"].T
    n = _normalize(xc[c2] - xc[c1] - np.sum((xc[c2] - xc[c1]) * xe, 1)[:, None] * xe)
    t = np.cross(xe, n)
    U = np.cross(_normalize(np.array([0.3, 0.2, 1.0])), xe)
    u, vt = np.sum(U * n, 1), np.sum(U * t, 1)
    eoe, w = mesh["edgesOnEdge"], mesh["weightsOnEdge"]
    v = np.sum(np.where(eoe >= 0, w * u[np.maximum(eoe, 0)], 0.0), 1)
    ok = mesh["dvEdge"] / mesh["dcEdge"] >= min_dv_dc
    assert np.abs(v - vt)[ok].max() / np.abs(vt).max() < 0.05
    dc, dv = mesh["dcEdge"], mesh["dvEdge"]
    W = {}
    for e in range(mesh["nEdges"]):
        for j in range(mesh["nEdgesOnEdge"][e]):
            W[(e, eoe[e, j])] = w[e, j] * dc[e] / dv[eoe[e, j]]
    err = max(abs(W[(a, b)] + W[(b, a)]) for (a, b) in W)
    assert err < 1e-14


def test_sfc_locality(mesh):
    """Cells are Hilbert-ordered: neighbours are close in index space (coalesced gathers)."""
    c1, c2 = mesh["cellsOnEdge"].T
    assert np.median(np.abs(c1 - c2)) < mesh["nCells"] / 8


@pytest.fixture(scope="module")
def vr_mesh():
    from mpas_dycore.mesh import build_varres_mesh
    return build_varres_mesh(2562, ratio=4.0, lloyd_iters=30)


def test_varres_mesh_conventions(vr_mesh):
    """Variable-resolution SCVT: valid Voronoi topology with 5/6/7-gons, MPAS orientation
    conventions, positive kites, near-exact tiling and antisymmetric TRiSK weights."""
    m = vr_mesh
    assert m["nCells"] - m["nEdges"] + m["nVertices"] == 2
    counts = np.bincount(m["nEdgesOnCell"])
    assert m["maxEdges"] == 7 and counts[5] > 0 and counts[7] > 0 and counts[6] > 0.8 * m["nCells"]
    assert (m["kiteAreasOnVertex"] > 0).all()
    R = m["sphere_radius"]
    assert abs(m["areaCell"].sum() / (4 * np.pi * R * R) - 1) < 2e-3
    assert m["dcEdge"].max() / m["dcEdge"].min() > 3.0           # really variable resolution
    test_edge_orientation_conventions(m)
    test_trisk_weights(m)


def test_large_varres_start_has_no_degenerate_edges():
    """The icosahedral start of the large variable-resolution meshes (build_varres_mesh,
    start="icosahedral"): no nearly co-circular quads, dvEdge / dcEdge well away from 0."""
    from mpas_dycore.mesh import build_varres_mesh
    m = build_varres_mesh(10242, ratio=20.0, lloyd_iters=4, start="icosahedral")
    assert m["nCells"] == 10242
    r = m["dvEdge"] / m["dcEdge"]
    assert r.min() > 0.3
    assert m["dcEdge"].max() / m["dcEdge"].min() > 10.0
    test_trisk_weights(m)
