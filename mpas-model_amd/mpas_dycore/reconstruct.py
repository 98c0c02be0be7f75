"""Mesh coefficients of the cell-centre velocity reconstruction.

This module restates two reference routines in numpy, vectorised over cells:
  * mpas_initialize_vectors (operators/mpas_vector_operations.F:652-771), which
    mpas_rbf_interp_initialize calls;
  * mpas_init_reconstruct (operators/mpas_vector_reconstruction.F:51-181).
Together they produce ``coeffs_reconstruct(R3, maxEdges, nCells)``: the
per-cell weights that map edge-normal velocities to a 3-D vector at the cell
centre. The atmosphere core computes them once at init (mpas_atm_core.F:408-409).
The per-step reconstruction itself runs on the GPU (k_reconstruct).

Operation order follows the Fortran, so the weights are reproducible:
  * Fortran ``sum()`` over R3 is ((a1 + a2) + a3);
  * ``**2`` is x*x;
  * the RBF is the inverse multiquadric 1/sqrt(1 + r²) (evaluate_rbf, :1369);
  * the linear solves are the reference's scaled-pivot elimination,
    elgs + mpas_legs (mpas_rbf_interpolation.F:1670-1846).
All of these run per cell, batched over cells with the same edge count.
"""
from __future__ import annotations

import numpy as np


def _sum3(a):
    return (a[..., 0] + a[..., 1]) + a[..., 2]


def _unit(v):
    """mpas_unit_vec_in_r3 (mpas_vector_operations.F:96-101)."""
    mag = np.sqrt((v[..., 0] ** 2 + v[..., 1] ** 2) + v[..., 2] ** 2)
    return v / mag[..., None]


def _cross(a, b):
    """mpas_cross_product_in_r3 (mpas_vector_operations.F:118-120)."""
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
                     a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], axis=-1)


def initialize_vectors(case: dict) -> dict:
    """edgeNormalVectors (nE,3), cellTangentPlane (nC,2,3), localVerticalUnitVectors (nC,3)
    on a sphere without boundaries (mpas_vector_operations.F:697-769)."""
    xc = np.stack([case["xCell"], case["yCell"], case["zCell"]], axis=-1).astype(np.float64)
    vert = _unit(xc.copy())
    coe = np.asarray(case["cellsOnEdge"])
    n = _unit(xc[coe[:, 1]] - xc[coe[:, 0]])
    e1 = np.asarray(case["edgesOnCell"])[:, 0]
    rhat = vert
    ndr = _sum3(n[e1] * rhat)
    xhat = _unit(n[e1] - ndr[:, None] * rhat)
    yhat = _unit(_cross(rhat, xhat))
    return dict(edgeNormalVectors=n, cellTangentPlane=np.stack([xhat, yhat], axis=1), localVerticalUnitVectors=vert)


CHUNK = 8192  # systems per batch: the batch's arrays stay in cache (each system is independent)


def _legs_batched(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """elgs + mpas_legs for a batch of systems A (m,N,N) and right-hand sides B (m,N,R); returns
    X (m,N,R).  The elimination (elgs) depends on A only, so it runs once for the R right-hand
    sides that the reference solves one call each -- same operations on each, same bits."""
    if A.shape[0] > CHUNK:
        return np.concatenate([_legs_batched(A[i:i + CHUNK], B[i:i + CHUNK]) for i in range(0, A.shape[0], CHUNK)])
    A = A.copy()
    B = B.copy()
    m, N, _ = A.shape
    rows = np.arange(m)
    indx = np.tile(np.arange(N), (m, 1))
    C = np.zeros((m, N))
    for i in range(N):  # row scale factors C(I) = max_j |A(I,J)| (sequential max from 0.0)
        c1 = np.zeros(m)
        for j in range(N):
            c1 = np.maximum(c1, np.abs(A[:, i, j]))
        C[:, i] = c1
    for j in range(N - 1):
        pi1 = np.zeros(m)
        k = np.full(m, j)
        for i in range(j, N):
            ii = indx[:, i]
            pi = np.abs(A[rows, ii, j]) / C[rows, ii]
            better = pi > pi1
            pi1 = np.where(better, pi, pi1)
            k = np.where(better, i, k)
        itmp = indx[:, j].copy()
        indx[:, j] = indx[rows, k]
        indx[rows, k] = itmp
        jj = indx[:, j]
        for i in range(j + 1, N):
            ii = indx[:, i]
            pj = A[rows, ii, j] / A[rows, jj, j]
            A[rows, ii, j] = pj
            for kk in range(j + 1, N):
                A[rows, ii, kk] = A[rows, ii, kk] - pj * A[rows, jj, kk]
    for i in range(N - 1):
        for j in range(i + 1, N):
            B[rows, indx[:, j]] = B[rows, indx[:, j]] - A[rows, indx[:, j], i][:, None] * B[rows, indx[:, i]]
    X = np.zeros((m, N, B.shape[2]))
    X[:, N - 1] = B[rows, indx[:, N - 1]] / A[rows, indx[:, N - 1], N - 1][:, None]
    for i in range(N - 2, -1, -1):
        xi = B[rows, indx[:, i]]
        for j in range(i + 1, N):
            xi = xi - A[rows, indx[:, i], j][:, None] * X[:, j]
        X[:, i] = xi / A[rows, indx[:, i], i][:, None]
    return X


def _rbf(r2):
    """evaluate_rbf (mpas_rbf_interpolation.F:1369-1376): inverse multiquadric."""
    return 1 / np.sqrt(1 + r2)


def init_reconstruct(case: dict, vectors: dict | None = None) -> np.ndarray:
    """coeffs_reconstruct as an element-major (nCells, maxEdges, 3) array
    (mpas_vector_reconstruction.F:112-177 with
    mpas_rbf_interp_func_3D_plane_vec_const_dir_comp_coeffs, mpas_rbf_interpolation.F:1079-1145)."""
    if vectors is None:
        vectors = initialize_vectors(case)
    nC, ME = case["nCells"], case["maxEdges"]
    noc = np.asarray(case["nEdgesOnCell"])
    eoc = np.asarray(case["edgesOnCell"])
    xc = np.stack([case["xCell"], case["yCell"], case["zCell"]], axis=-1).astype(np.float64)
    xe = np.stack([case["xEdge"], case["yEdge"], case["zEdge"]], axis=-1).astype(np.float64)
    nrm = vectors["edgeNormalVectors"]
    tp = vectors["cellTangentPlane"]
    out = np.zeros((nC, ME, 3))
    for pc in np.unique(noc):
        cells = np.flatnonzero(noc == pc)
        m = cells.size
        e = eoc[cells, :pc]                              # (m, pc)
        center = xc[cells]                               # (m, 3)
        loc = xe[e]                                      # (m, pc, 3)
        nor = nrm[e]                                     # (m, pc, 3)
        # alpha = mean distance from the centre to the edge points (sequential sum, :141-145)
        alpha = np.zeros(m)
        for i in range(pc):
            d = center - loc[:, i]
            alpha = alpha + np.sqrt(_sum3(d * d))
        alpha = alpha / pc
        b1, b2 = tp[cells, 0], tp[cells, 1]              # (m, 3) plane basis
        ps = np.stack([_sum3(loc * b1[:, None]), _sum3(loc * b2[:, None])], axis=-1)   # (m, pc, 2)
        pu = np.stack([_sum3(nor * b1[:, None]), _sum3(nor * b2[:, None])], axis=-1)
        pd = np.stack([_sum3(center * b1), _sum3(center * b2)], axis=-1)                # (m, 2)
        a2 = alpha * alpha
        N = pc + 2
        M = np.zeros((m, N, N))
        rhs = np.zeros((m, N, 2))
        for j in range(pc):  # mpas_set_up_vector_dirichlet_rbf_matrix_and_rhs (:1546-1556)
            for i in range(j, pc):
                d = ps[:, i] - ps[:, j]
                r2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) / a2
                dot = pu[:, i, 0] * pu[:, j, 0] + pu[:, i, 1] * pu[:, j, 1]
                M[:, i, j] = _rbf(r2) * dot
                M[:, j, i] = M[:, i, j]
        for j in range(pc):
            d = pd - ps[:, j]
            r2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) / a2
            rhs[:, j, :] = _rbf(r2)[:, None] * pu[:, j, :]
        for i in range(pc):  # constant vector in the plane (:1117-1123)
            M[:, i, pc:pc + 2] = pu[:, i, :]
            M[:, pc:pc + 2, i] = pu[:, i, :]
        rhs[:, pc, 0] = 1.0
        rhs[:, pc + 1, 1] = 1.0
        cc = _legs_batched(M, rhs)
        c1, c2 = cc[:, :, 0], cc[:, :, 1]
        for i in range(3):  # coefficients(:,i) = b1(i) c1 + b2(i) c2 (:1131-1134)
            out[cells, :pc, i] = b1[:, i][:, None] * c1[:, :pc] + b2[:, i][:, None] * c2[:, :pc]
    return out
