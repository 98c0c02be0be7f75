"""Quasi-uniform icosahedral Voronoi (C-grid) mesh generator with MPAS conventions.

The reference vendors no meshes and no mesh generator (MPAS-Tools is external,
SURVEY.md §7 "Meshes"), so the synthetic x1.N meshes used by the parity tests
and the benchmark are generated here.  Every convention the dycore relies on is
taken from how the reference *uses* the fields:

* ``u(k,e)`` is positive from ``cellsOnEdge(1,e)`` to ``cellsOnEdge(2,e)``
  (``mpas_atm_core.F:1040-1048``, divergence in
  ``mpas_atm_time_integration.F:5626-5640``).
* ``verticesOnEdge(2,e)`` lies to the left of the normal: k x n points from
  vertex 1 to vertex 2 (``mpas_atm_core.F:1026-1030`` + vorticity at
  ``mpas_atm_time_integration.F:5606-5620``).
* ``edgesOnCell(i,c)`` joins ``verticesOnCell(i,c)`` and ``verticesOnCell(i+1,c)``
  and ``cellsOnCell(i,c)`` lies across it, counter-clockwise
  (``core_init_atmosphere/mpas_atm_advection.F:290-323, 898-946``).
* ``kiteAreasOnVertex(j,v)`` is the kite of ``cellsOnVertex(j,v)``
  (``mpas_atm_core.F:1055-1072``).
* ``edgesOnEdge/weightsOnEdge`` are the TRiSK reconstruction (Thuburn et al.
  2009, Ringler et al. 2010) of the tangential velocity, positive along k x n.

All arrays here are 0-based numpy arrays (index -1 = "no neighbour"); the
Fortran/C-ABI layer converts to MPAS 1-based + garbage-slot indexing.
Cells are ordered along a 3-D Hilbert space-filling curve so neighbour gathers
are local in memory (north_star: "index arrays reordered by SFC").
"""
from __future__ import annotations

import os
import sys

import numpy as np

SPHERE_RADIUS = 6371229.0  # mpas_constants.F: a = 6371229


# --------------------------------------------------------------------------
# spherical geometry helpers (vectorised)
# --------------------------------------------------------------------------
def _normalize(x):
    return x / np.linalg.norm(x, axis=-1, keepdims=True)


def arc_length(a, b):
    """Great-circle distance between unit vectors (robust atan2 form)."""
    cr = np.linalg.norm(np.cross(a, b), axis=-1)
    dt = np.sum(a * b, axis=-1)
    return np.arctan2(cr, dt)


def tri_area(a, b, c):
    """Spherical triangle area on the unit sphere (Van Oosterom-Strackee)."""
    num = np.abs(np.sum(a * np.cross(b, c), axis=-1))
    den = 1.0 + np.sum(a * b, axis=-1) + np.sum(b * c, axis=-1) + np.sum(c * a, axis=-1)
    return 2.0 * np.arctan2(num, den)


def latlon(x):
    lat = np.arcsin(np.clip(x[..., 2], -1.0, 1.0))
    lon = np.arctan2(x[..., 1], x[..., 0])
    lon = np.where(lon < 0.0, lon + 2.0 * np.pi, lon)
    return lat, lon


# --------------------------------------------------------------------------
# icosahedral geodesic Delaunay triangulation
# --------------------------------------------------------------------------
def _icosahedron():
    p = (1.0 + 5 ** 0.5) / 2.0
    v = np.array([[-1, p, 0], [1, p, 0], [-1, -p, 0], [1, -p, 0],
                  [0, -1, p], [0, 1, p], [0, -1, -p], [0, 1, -p],
                  [p, 0, -1], [p, 0, 1], [-p, 0, -1], [-p, 0, 1]], dtype=np.float64)
    f = np.array([[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11],
                  [1, 5, 9], [5, 11, 4], [11, 10, 2], [10, 7, 6], [7, 1, 8],
                  [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9],
                  [4, 9, 5], [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]], dtype=np.int64)
    return _normalize(v), f


def _subdivide(v, f):
    e = np.sort(np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]]), axis=1)
    key = e[:, 0] * len(v) + e[:, 1]
    ukey, inv = np.unique(key, return_inverse=True)
    a, b = ukey // len(v), ukey % len(v)
    mid = _normalize(v[a] + v[b])
    nf = len(f)
    m01 = len(v) + inv[:nf]
    m12 = len(v) + inv[nf:2 * nf]
    m20 = len(v) + inv[2 * nf:]
    f0, f1, f2 = f[:, 0], f[:, 1], f[:, 2]
    nf_ = np.concatenate([np.stack([f0, m01, m20], 1), np.stack([f1, m12, m01], 1),
                          np.stack([f2, m20, m12], 1), np.stack([m01, m12, m20], 1)])
    return np.concatenate([v, mid]), nf_


def _hilbert3d_keys(x, bits=16):
    """3-D Hilbert index of points in [-1,1]^3 (Skilling's transpose algorithm)."""
    n = 1 << bits
    q = np.clip(((x + 1.0) * 0.5 * (n - 1)).round().astype(np.int64), 0, n - 1)
    X = [q[:, 0].copy(), q[:, 1].copy(), q[:, 2].copy()]
    M = 1 << (bits - 1)
    Q = M
    while Q > 1:
        P = Q - 1
        for i in range(3):
            hi = (X[i] & Q) != 0
            X[0] = np.where(hi, X[0] ^ P, X[0])
            t = np.where(hi, 0, (X[0] ^ X[i]) & P)
            X[0] ^= t
            X[i] ^= t
        Q >>= 1
    for i in range(1, 3):
        X[i] ^= X[i - 1]
    t = np.zeros_like(X[0])
    Q = M
    while Q > 1:
        t = np.where((X[2] & Q) != 0, t ^ (Q - 1), t)
        Q >>= 1
    for i in range(3):
        X[i] ^= t
    key = np.zeros(len(x), dtype=np.int64)
    for b in range(bits - 1, -1, -1):
        for i in range(3):
            key = (key << 1) | ((X[i] >> b) & 1)
    return key


def _circumcenters(p, f):
    a, b, c = p[f[:, 0]], p[f[:, 1]], p[f[:, 2]]
    cc = _normalize(np.cross(b - a, c - a))
    s = np.sign(np.sum(cc * a, axis=1))
    return cc * s[:, None]


# --------------------------------------------------------------------------
# mesh construction
# --------------------------------------------------------------------------
def build_mesh(level: int, lloyd_iters: int = 0, radius: float = SPHERE_RADIUS, sfc: bool = True) -> dict:
    """Build an x1.(10*4**level+2) mesh.  Returns a dict of 0-based arrays."""
    p, f = _icosahedron()
    for _ in range(level):
        p, f = _subdivide(p, f)
    # orient faces counter-clockwise seen from outside
    a, b, c = p[f[:, 0]], p[f[:, 1]], p[f[:, 2]]
    flip = np.sum(np.cross(b - a, c - a) * a, axis=1) < 0
    f[flip] = f[flip][:, [0, 2, 1]]

    # Lloyd (centroidal) relaxation with fixed topology
    for _ in range(lloyd_iters):
        p = _lloyd_step(p, f)

    if sfc:
        order = np.argsort(_hilbert3d_keys(p), kind="stable")
        rank = np.empty_like(order)
        rank[order] = np.arange(len(order))
        p = p[order]
        f = rank[f]
    return _topology_and_geometry(p, f, radius)


def _lloyd_step(p, f, density=None):
    """One Lloyd step: every generator moves to the (density-weighted) centroid of its
    Voronoi cell, integrated over the fan of triangles (generator, v_j, v_j+1)."""
    vc = _circumcenters(p, f)
    cnt, vof = _cells_vertices_ccw(p, f)
    W = vof.shape[1]
    num = np.zeros_like(p)
    idx = np.arange(len(p))
    for j in range(W):
        ok = j < cnt
        v0 = vof[ok, j]
        v1 = vof[ok, (j + 1) % W]
        v1 = np.where((j + 1) < cnt[ok], v1, vof[ok, 0])
        tA, tB, tC = p[idx[ok]], vc[v0], vc[v1]
        ar = tri_area(tA, tB, tC)
        cen = _normalize(tA + tB + tC)
        if density is not None:
            ar = ar * density(cen)
        num[idx[ok]] += ar[:, None] * cen
    return _normalize(num)


def _delaunay(p):
    """Spherical Delaunay triangulation = convex hull of the unit generators, faces CCW."""
    from scipy.spatial import ConvexHull
    f = ConvexHull(p).simplices.astype(np.int64)
    a, b, c = p[f[:, 0]], p[f[:, 1]], p[f[:, 2]]
    flip = np.sum(np.cross(b - a, c - a) * a, axis=1) < 0
    f[flip] = f[flip][:, [0, 2, 1]]
    return f


def varres_density(center_latlon=(30.0, -90.0), radius_deg=20.0, width_deg=10.0, ratio=20.0):
    """MPAS-style refinement density rho(x) = (1-g)/2 (tanh((beta - d)/alpha) + 1) + g with
    g = ratio^-4, so the cell spacing dx ~ rho^-1/4 varies by ``ratio`` between the
    refined disc (radius beta around the centre) and the far field."""
    lat, lon = np.radians(center_latlon[0]), np.radians(center_latlon[1])
    xc = np.array([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)])
    beta, alpha, g = np.radians(radius_deg), np.radians(width_deg), float(ratio) ** -4

    def rho(x):
        d = np.arccos(np.clip(x @ xc, -1.0, 1.0))
        return (1.0 - g) / 2.0 * (np.tanh((beta - d) / alpha) + 1.0) + g
    return rho


def _fibonacci_sphere(n):
    i = np.arange(n) + 0.5
    z = 1.0 - 2.0 * i / n
    r = np.sqrt(1.0 - z * z)
    phi = np.pi * (3.0 - np.sqrt(5.0)) * i
    return np.stack([r * np.cos(phi), r * np.sin(phi), z], axis=1)


def _schmidt(p, center_latlon, c):
    """Schmidt transform: colatitude theta about the centre -> 2 atan(tan(theta/2) / c),
    which refines the spacing by c near the centre and coarsens it by c at the antipode."""
    lat, lon = np.radians(center_latlon[0]), np.radians(center_latlon[1])
    zc = np.array([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)])
    a = np.cross(zc, [0.0, 0.0, 1.0]) if abs(zc[2]) < 0.9 else np.cross(zc, [1.0, 0.0, 0.0])
    xa = a / np.linalg.norm(a)
    ya = np.cross(zc, xa)
    pz, px, py = p @ zc, p @ xa, p @ ya
    th = np.arccos(np.clip(pz, -1.0, 1.0))
    ph = np.arctan2(py, px)
    th2 = 2.0 * np.arctan(np.tan(th / 2.0) / c)
    return (np.sin(th2) * np.cos(ph))[:, None] * xa + (np.sin(th2) * np.sin(ph))[:, None] * ya + np.cos(th2)[:, None] * zc


def _icosahedral_points(n: int) -> np.ndarray:
    """Generators of an n-times subdivided icosahedron (10 n^2 + 2 points): each face's
    barycentric grid, projected to the sphere, shared edge / corner points once."""
    v, f = _icosahedron()
    i, j = np.meshgrid(np.arange(n + 1), np.arange(n + 1), indexing="ij")
    keep = (i + j) <= n
    i, j = i[keep].astype(np.float64), j[keep].astype(np.float64)
    k = n - i - j
    pts = np.concatenate([(i[:, None] * v[a] + j[:, None] * v[b] + k[:, None] * v[c]) / n for a, b, c in f])
    p = _normalize(pts)
    _, first = np.unique(np.round(p * 1e9).astype(np.int64), axis=0, return_index=True)
    return p[np.sort(first)]


def build_varres_mesh(ncells: int, ratio: float = 20.0, lloyd_iters: int = 10, seed: int = 20250415,
                      radius: float = SPHERE_RADIUS, sfc: bool = True, start: str | None = None,
                      **density_kw) -> dict:
    """Variable-resolution spherical centroidal Voronoi mesh (BASELINE.json configs[4]:
    x20.835586-like 60-3 km meshes).  A Fibonacci lattice of ``ncells`` generators is
    pulled towards the refinement centre by a Schmidt transform (stretch sqrt(ratio)),
    then relaxed by density-weighted Lloyd iterations on the spherical Delaunay
    triangulation, which is rebuilt every step so the topology (pentagons / hexagons /
    heptagons in the transition zone) is free to change.

    start = "icosahedral" (the default above 200000 cells) begins instead from the n-times
    subdivided icosahedron with 10 n^2 + 2 ~ ncells points (n = 289: 835212 cells): a few Lloyd
    iterations from the Fibonacci lattice leave tens of thousands of nearly co-circular quads at
    that size (Voronoi edges of ~1e-6 of the spacing, which make the dycore blow up within a
    step), while the stretched icosahedral lattice relaxes to dvEdge / dcEdge >= 0.35 -- at the
    price of hexagons only (the 5/6/7-gon paths are covered by the smaller Fibonacci meshes)."""
    rho = varres_density(ratio=ratio, **density_kw)
    center = density_kw.get("center_latlon", (30.0, -90.0))
    if start is None:
        start = "icosahedral" if ncells > 200000 else "fibonacci"
    if start == "icosahedral":
        p0 = _icosahedral_points(max(1, int(round(np.sqrt((ncells - 2) / 10.0)))))
    else:
        p0 = _fibonacci_sphere(ncells)
    p = _schmidt(p0, center, np.sqrt(ratio))
    for it in range(lloyd_iters):
        p = _lloyd_step(p, _delaunay(p), rho)
        if ncells > 200000:  # long builds report progress (a silent GPU-box job looks hung)
            print(f"varres mesh: Lloyd iteration {it + 1}/{lloyd_iters}", file=sys.__stderr__, flush=True)
    if start == "icosahedral":  # a safety net: the stretched lattice relaxes without such quads
        p = _untangle_cocircular(p)
    f = _delaunay(p)
    if sfc:
        order = np.argsort(_hilbert3d_keys(p), kind="stable")
        rank = np.empty_like(order)
        rank[order] = np.arange(len(order))
        p = p[order]
        f = rank[f]
    m = _topology_and_geometry(p, f, radius)
    m["meshDensity"] = rho(p)
    return m


DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
X20_835586 = os.path.join(DATA, "x20.835586_generators.npz")


def varres_from_generators(path: str = X20_835586, radius: float = SPHERE_RADIUS, sfc: bool = True) -> dict:
    """A variable-resolution mesh from stored generators (tools/make_varres_mesh.py: the BASELINE.json
    configs[4] 60-3 km SCVT of 835586 cells, Lloyd-relaxed offline): the spherical Delaunay
    triangulation of the generators, Hilbert-ordered, with the MPAS topology and geometry, and the
    meshDensity of the density it was relaxed for."""
    z = np.load(path, allow_pickle=False)
    p = _normalize(z["xyz_q30"].astype(np.float64) / 2.0 ** 30)
    rho = varres_density(tuple(float(x) for x in z["center"]), float(z["radius_deg"]), float(z["width_deg"]),
                         float(z["ratio"]))
    f = _delaunay(p)
    if sfc:
        order = np.argsort(_hilbert3d_keys(p), kind="stable")
        rank = np.empty_like(order)
        rank[order] = np.arange(len(order))
        p = p[order]
        f = rank[f]
    m = _topology_and_geometry(p, f, radius)
    m["meshDensity"] = rho(p)
    return m


def _untangle_cocircular(p, min_ratio=0.05, step=0.15, rounds=10):
    """Density-weighted Lloyd iterations leave some nearly co-circular generator quads in the
    refinement's transition zone: their two Delaunay triangles have almost the same circumcentre,
    so the Voronoi edge between them is ~1e-6 of the cell spacing (a 4-valent vertex in all but
    name).  Such an edge makes the dycore's 1/dvEdge operators (del4 mixing, vorticity) blow up.
    Pulling the edge's two generators towards each other by ``step`` of their distance makes that
    diagonal clearly Delaunay and opens the edge; repeated until every Voronoi edge is at least
    ``min_ratio`` of its cell-centre distance (MPAS quasi-uniform meshes: ~0.33)."""
    for _ in range(rounds):
        f = _delaunay(p)
        vc = _circumcenters(p, f)
        pairs = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]])
        face = np.concatenate([np.arange(len(f))] * 3)
        s = np.sort(pairs, axis=1)
        o = np.lexsort((s[:, 1], s[:, 0]))
        s, face = s[o], face[o]
        a, b = s[0::2], s[1::2]
        fa, fb = face[0::2], face[1::2]
        dv = np.linalg.norm(vc[fa] - vc[fb], axis=1)
        dc = np.linalg.norm(p[a[:, 0]] - p[a[:, 1]], axis=1)
        bad = dv < min_ratio * dc
        if len(p) > 200000:
            print(f"varres mesh: {int(bad.sum())} near-degenerate Voronoi edges", file=sys.__stderr__, flush=True)
        if not np.any(bad):
            break
        i, j = a[bad, 0], a[bad, 1]
        d = p[j] - p[i]
        q = p.copy()
        np.add.at(q, i, step * d)
        np.add.at(q, j, -step * d)
        p = _normalize(q)
    return p


def _cells_vertices_ccw(p, f, width=None):
    """For each cell, its incident faces (=Voronoi vertices) sorted CCW; -1 padded to
    ``width`` (default: the largest cell degree)."""
    nC = len(p)
    cell = f.reshape(-1)
    face = np.repeat(np.arange(len(f)), 3)
    vc = _circumcenters(p, f)
    c = p[cell]
    # local tangent basis
    ez = np.array([0.0, 0.0, 1.0])
    e1 = np.cross(ez, c)
    bad = np.linalg.norm(e1, axis=1) < 1e-8
    e1[bad] = np.cross(np.array([1.0, 0.0, 0.0]), c[bad])
    e1 = _normalize(e1)
    e2 = np.cross(c, e1)
    d = vc[face] - c
    ang = np.arctan2(np.sum(d * e2, axis=1), np.sum(d * e1, axis=1))
    o = np.lexsort((ang, cell))
    cell_s, face_s = cell[o], face[o]
    cnt = np.bincount(cell_s, minlength=nC)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    pos = np.arange(len(cell_s)) - start[cell_s]
    vof = -np.ones((nC, int(cnt.max()) if width is None else width), dtype=np.int64)
    vof[cell_s, pos] = face_s
    return cnt, _walk_fans(f, cnt, vof, nC)


def _walk_fans(f, cnt, vof, nC):
    """Re-derive every cell's CCW face order by walking its triangle fan from the first face of
    the angle sort: the face after (a, b, c) around a is the one holding the directed edge a -> c.
    Where the angle sort is right this reproduces it; where two circumcentres nearly coincide
    (co-circular generators: a near-zero Voronoi edge) the sort can swap them, and consecutive
    faces then share no edge -- cellsOnCell / edgesOnCell would be broken for that cell."""
    nF = len(f)
    src = f.reshape(-1)
    dst = f[:, [1, 2, 0]].reshape(-1)
    keys = src * nC + dst
    order = np.argsort(keys)
    keys_s, face_of = keys[order], np.repeat(np.arange(nF), 3)[order]
    out = vof.copy()
    cells = np.arange(nC)
    cur = vof[:, 0]
    for j in range(1, vof.shape[1]):
        live = j < cnt
        fc = f[np.where(live, cur, 0)]
        # c: the vertex before `cell` in face cur (CCW), i.e. f[(pos + 2) % 3]
        pos = np.argmax(fc == cells[:, None], axis=1)
        c = fc[np.arange(nC), (pos + 2) % 3]
        k = np.searchsorted(keys_s, cells * nC + c)
        nxt = face_of[np.minimum(k, len(keys_s) - 1)]
        cur = np.where(live, nxt, cur)
        out[:, j] = np.where(live, cur, out[:, j])
    return out


def _topology_and_geometry(p, f, radius):
    # vertex (triangle) order: by the sorted cell triple, like the edges' (first cell, second
    # cell) order below, so vertices follow the cells' Hilbert order too -- the vertex gathers
    # of the diagnostics (edgesOnVertex, verticesOnCell, verticesOnEdge) stay local in memory
    fs = np.sort(f, axis=1)
    f = f[np.lexsort((fs[:, 2], fs[:, 1], fs[:, 0]))]
    nC, nV = len(p), len(f)
    xv = _circumcenters(p, f)
    nEoC, voc = _cells_vertices_ccw(p, f)
    maxEdges = voc.shape[1]  # 6 for icosahedral meshes; 7+ for variable-resolution SCVTs

    # edges: unique (cell,cell) pairs of the Delaunay triangles
    pairs = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]])
    pface = np.concatenate([np.arange(nV)] * 3)
    s = np.sort(pairs, axis=1)
    key = s[:, 0] * nC + s[:, 1]
    o = np.argsort(key, kind="stable")
    key_s = key[o]
    assert np.all(key_s[0::2] == key_s[1::2]), "non-manifold triangulation"
    ekey = key_s[0::2]
    faceA, faceB = pface[o][0::2], pface[o][1::2]
    c1, c2 = ekey // nC, ekey % nC
    nE = len(ekey)
    # edge order: by first cell (already sorted since key sorted by (c1,c2)) -> SFC-local
    cellsOnEdge = np.stack([c1, c2], 1)
    xc = p
    xe = _normalize(xc[c1] + xc[c2])
    # verticesOnEdge: vertex 2 to the left of normal n (c1->c2):  (k x n) . (v2 - v1) > 0
    n = xc[c2] - xc[c1]
    n = _normalize(n - np.sum(n * xe, axis=1)[:, None] * xe)
    t = np.cross(xe, n)
    vA, vB = faceA, faceB
    swap = np.sum((xv[vB] - xv[vA]) * t, axis=1) < 0
    v1 = np.where(swap, vB, vA)
    v2 = np.where(swap, vA, vB)
    verticesOnEdge = np.stack([v1, v2], 1)

    # lookup edge id from sorted cell pair
    def edge_of(ca, cb):
        lo, hi = np.minimum(ca, cb), np.maximum(ca, cb)
        return np.searchsorted(ekey, lo * nC + hi)

    # cell connectivity: vertices CCW; edge i joins vertex i and i+1
    verticesOnCell = voc.copy()
    edgesOnCell = -np.ones((nC, maxEdges), dtype=np.int64)
    cellsOnCell = -np.ones((nC, maxEdges), dtype=np.int64)
    for i in range(maxEdges):
        has = i < nEoC
        va = voc[:, i]
        vb = np.where(i + 1 < nEoC, voc[:, (i + 1) % maxEdges], voc[:, 0])
        # the edge shared by faces va and vb is the cell pair (this cell, other)
        # other cell = the vertex common to faces va, vb that is not this cell
        cc = np.arange(nC)
        fa, fb = f[np.where(has, va, 0)], f[np.where(has, vb, 0)]
        other = -np.ones(nC, dtype=np.int64)
        for ia in range(3):
            for ib in range(3):
                m = (fa[:, ia] == fb[:, ib]) & (fa[:, ia] != cc)
                other = np.where(m, fa[:, ia], other)
        eid = edge_of(cc, np.where(other >= 0, other, 0))
        edgesOnCell[:, i] = np.where(has, eid, -1)
        cellsOnCell[:, i] = np.where(has, other, -1)

    # a closed mesh: every edge of a cell joins it to the neighbour listed beside it
    slot = np.arange(maxEdges)[None, :] < nEoC[:, None]
    ce = cellsOnEdge[np.where(slot, edgesOnCell, 0)]
    own = np.arange(nC)[:, None]
    ok = (cellsOnCell >= 0) & (((ce[..., 0] == own) & (ce[..., 1] == cellsOnCell))
                               | ((ce[..., 1] == own) & (ce[..., 0] == cellsOnCell)))
    assert np.all(ok | ~slot), f"inconsistent cell connectivity in {int((~ok & slot).sum())} slots"

    # vertex connectivity: cells of the (CCW) Delaunay face, edge j between cell j and j+1
    cellsOnVertex = f.copy()
    edgesOnVertex = np.stack([edge_of(f[:, j], f[:, (j + 1) % 3]) for j in range(3)], 1)

    # geometry (unit sphere, then scaled)
    dcEdge = arc_length(xc[c1], xc[c2])
    dvEdge = arc_length(xv[v1], xv[v2])
    # kites: kite(j, v) of cell cellsOnVertex(j,v) = tri(c, e_prev, v) + tri(c, v, e_next)
    kite = np.zeros((nV, 3))
    for j in range(3):
        cj = f[:, j]
        e_next = edgesOnVertex[:, j]            # between cell j and j+1
        e_prev = edgesOnVertex[:, (j + 2) % 3]  # between cell j-1 and j
        kite[:, j] = tri_area(xc[cj], xe[e_prev], xv) + tri_area(xc[cj], xv, xe[e_next])
    areaTriangle = kite.sum(1)
    areaCell = np.zeros(nC)
    np.add.at(areaCell, f.reshape(-1), kite.reshape(-1))

    latCell, lonCell = latlon(xc)
    latVertex, lonVertex = latlon(xv)
    latEdge, lonEdge = latlon(xe)
    # angleEdge: angle of the edge normal w.r.t. local east (MPAS convention)
    ez = np.array([0.0, 0.0, 1.0])
    east = np.cross(ez, xe)
    bad = np.linalg.norm(east, axis=1) < 1e-12
    east[bad] = np.array([1.0, 0.0, 0.0])
    east = _normalize(east)
    north = np.cross(xe, east)
    angleEdge = np.arctan2(np.sum(n * north, axis=1), np.sum(n * east, axis=1))

    R = radius
    mesh = dict(
        nCells=nC, nEdges=nE, nVertices=nV, maxEdges=maxEdges, maxEdges2=2 * maxEdges, vertexDegree=3,
        sphere_radius=R,
        xCell=xc[:, 0] * R, yCell=xc[:, 1] * R, zCell=xc[:, 2] * R,
        xEdge=xe[:, 0] * R, yEdge=xe[:, 1] * R, zEdge=xe[:, 2] * R,
        xVertex=xv[:, 0] * R, yVertex=xv[:, 1] * R, zVertex=xv[:, 2] * R,
        latCell=latCell, lonCell=lonCell, latEdge=latEdge, lonEdge=lonEdge,
        latVertex=latVertex, lonVertex=lonVertex, angleEdge=angleEdge,
        nEdgesOnCell=nEoC.astype(np.int64), edgesOnCell=edgesOnCell, cellsOnCell=cellsOnCell,
        verticesOnCell=verticesOnCell, cellsOnEdge=cellsOnEdge, verticesOnEdge=verticesOnEdge,
        cellsOnVertex=cellsOnVertex, edgesOnVertex=edgesOnVertex,
        dcEdge=dcEdge * R, dvEdge=dvEdge * R, areaCell=areaCell * R * R,
        areaTriangle=areaTriangle * R * R, kiteAreasOnVertex=kite * R * R,
        meshDensity=np.ones(nC), indexToCellID=np.arange(1, nC + 1),
    )
    _trisk(mesh)
    return mesh


def _trisk(m):
    """edgesOnEdge / weightsOnEdge (Thuburn et al. 2009 TRiSK weights).

    For edge e and each of its cells c (c1 then c2), the other edges e' of c are
    visited counter-clockwise starting after e; R accumulates the kite fractions
    of the vertices passed.  v_e = sum_j weightsOnEdge(j,e) * u(edgesOnEdge(j,e)).
    Validated by tests/test_mesh.py (solid-body rotation and energy antisymmetry).
    """
    nE, maxE = m["nEdges"], m["maxEdges"]
    nEoC, eoc, voc = m["nEdgesOnCell"], m["edgesOnCell"], m["verticesOnCell"]
    coe, cov, kite = m["cellsOnEdge"], m["cellsOnVertex"], m["kiteAreasOnVertex"]
    area, dc, dv = m["areaCell"], m["dcEdge"], m["dvEdge"]
    eoe = -np.ones((nE, 2 * maxE), dtype=np.int64)
    w = np.zeros((nE, 2 * maxE))
    neoe = np.zeros(nE, dtype=np.int64)
    # kite fraction of cell c at its i-th vertex
    kfrac = np.zeros((m["nCells"], maxE))
    for i in range(maxE):
        v = voc[:, i]
        ok = v >= 0
        vv = np.where(ok, v, 0)
        kk = np.zeros(m["nCells"])
        for j in range(3):
            kk = np.where(cov[vv, j] == np.arange(m["nCells"]), kite[vv, j], kk)
        kfrac[:, i] = np.where(ok, kk / area, 0.0)
    # edge sign on cell: +1 if cell is cellsOnEdge(1)
    for side in range(2):
        c = coe[:, side]
        n = nEoC[c]
        # position of e within edgesOnCell(c)
        pos = np.zeros(nE, dtype=np.int64)
        for i in range(maxE):
            pos = np.where(eoc[c, i] == np.arange(nE), i, pos)
        Racc = np.zeros(nE)
        sgn_e = 1.0 if side == 0 else -1.0   # outward-normal sign of e relative to c
        for j in range(1, maxE):
            act = j < n
            ii = (pos + j) % np.maximum(n, 1)
            e2 = eoc[c, ii]
            # vertex passed between previous edge and e2 is verticesOnCell(ii) (edge ii joins v_ii, v_ii+1)
            Racc = Racc + np.where(act, kfrac[c, ii], 0.0)
            s2 = np.where(coe[np.where(act, e2, 0), 0] == c, 1.0, -1.0)  # outward sign of e2 on c
            val = sgn_e * s2 * (0.5 - Racc) * dv[np.where(act, e2, 0)] / dc
            col = neoe.copy()
            eoe[np.arange(nE)[act], col[act]] = e2[act]
            w[np.arange(nE)[act], col[act]] = val[act]
            neoe = neoe + act
    m["edgesOnEdge"] = eoe
    m["weightsOnEdge"] = w
    m["nEdgesOnEdge"] = neoe


# arrays of a mesh / case whose second axis is the maxEdges (maxEdges2) slot
MAX_EDGES_ARRAYS = ("edgesOnCell", "cellsOnCell", "verticesOnCell", "kiteForCell", "edgesOnCell_sign", "defc_a",
                    "defc_b", "coeffs_reconstruct", "zb_cell", "zb3_cell")
MAX_EDGES2_ARRAYS = ("edgesOnEdge", "weightsOnEdge")


def pad_max_edges(m: dict, max_edges: int = 10, max_edges2: int = 20, fill: str = "none") -> dict:
    """The same mesh (or case) declared with larger maxEdges / maxEdges2, as MPAS-distributed mesh files
    declare them (maxEdges = 10, maxEdges2 = 20: "the largest number of neighbors that a primal mesh
    cell may have", core_atmosphere/Registry.xml:13-16).  Slots past nEdgesOnCell / nEdgesOnEdge are
    never read by the reference; they hold ``fill``: "none" -- index -1 (0 in the 1-based file), real
    0 -- or "repeat" -- the row's last used entry repeated (index arrays; reals stay 0), the two
    conventions MPAS mesh tools have written."""
    out = dict(m)
    out["maxEdges"], out["maxEdges2"] = int(max_edges), int(max_edges2)
    for names, n_new, cnt in ((MAX_EDGES_ARRAYS, max_edges, "nEdgesOnCell"),
                              (MAX_EDGES2_ARRAYS, max_edges2, "nEdgesOnEdge")):
        for n in names:
            if n not in m:
                continue
            a = np.asarray(m[n])
            if a.shape[1] > n_new:
                raise ValueError(f"{n} has {a.shape[1]} slots, more than {n_new}")
            pad_shape = (a.shape[0], n_new - a.shape[1]) + a.shape[2:]
            is_index = np.issubdtype(a.dtype, np.integer) and n != "kiteForCell"
            pad = np.full(pad_shape, -1 if is_index else 0, dtype=a.dtype)
            b = np.concatenate([a, pad], axis=1)
            if is_index or n == "kiteForCell":
                used = np.asarray(m[cnt])
                slot = np.arange(n_new)[None, :]
                if fill == "repeat":
                    last = b[np.arange(b.shape[0]), np.maximum(used - 1, 0)]
                    b = np.where(slot < used[:, None], b, last[:, None])
                elif n != "kiteForCell":
                    b = np.where(slot < used[:, None], b, -1)
            out[n] = b
    return out
