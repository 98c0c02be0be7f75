"""Field registry: MPAS names, pools, horizontal location and index semantics.

Names follow core_atmosphere/Registry.xml (var_struct mesh/state/diag/tend,
Registry.xml:1127-1779).  Arrays on the Python side are element-major numpy
arrays, e.g. ``u`` has shape (nEdges, K) -- the transpose of the Fortran
``u(K, nEdges+1)`` without the garbage slot -- so a row is one contiguous
column of K levels, exactly the layout used in HBM (k is the fast axis).
"""
from __future__ import annotations

# name -> horizontal location of the LEADING numpy axis
LOCATION = {}
for n in ("latCell lonCell xCell yCell zCell areaCell invAreaCell meshDensity nEdgesOnCell indexToCellID "
          "edgesOnCell cellsOnCell verticesOnCell kiteForCell edgesOnCell_sign defc_a defc_b zgrid zz dss "
          "zb_cell zb3_cell theta rho scalars rho_base theta_base w coeffs_reconstruct t_init "
          "bdyMaskCell nearestRelaxationCell meshScalingRegionalCell specZoneMaskCell "
          "meshDensity_root4 dss_sin").split():
    LOCATION[n] = "cell"
for n in ("latEdge lonEdge xEdge yEdge zEdge dcEdge dvEdge invDcEdge invDvEdge angleEdge fEdge "
          "meshScalingDel2 meshScalingDel4 nEdgesOnEdge nAdvCellsForEdge cellsOnEdge verticesOnEdge "
          "edgesOnEdge advCellsForEdge weightsOnEdge adv_coefs adv_coefs_3rd zxu deriv_two zb zb3 u "
          "bdyMaskEdge meshScalingRegionalEdge specZoneMaskEdge meshDensityEdge_root4").split():
    LOCATION[n] = "edge"
for n in ("latVertex lonVertex xVertex yVertex zVertex areaTriangle invAreaTriangle fVertex "
          "cellsOnVertex edgesOnVertex edgesOnVertex_sign kiteAreasOnVertex").split():
    LOCATION[n] = "vertex"

# index arrays -> which element set they point into (0-based in numpy, -1 = none)
INDEX_TARGET = {
    "edgesOnCell": "edge", "cellsOnCell": "cell", "verticesOnCell": "vertex",
    "cellsOnEdge": "cell", "verticesOnEdge": "vertex", "edgesOnEdge": "edge",
    "advCellsForEdge": "cell", "cellsOnVertex": "cell", "edgesOnVertex": "edge",
    "nearestRelaxationCell": "cell",
}
# small-integer arrays stored 0-based in numpy but 1-based in MPAS (not element indices)
ONE_BASED_SMALL = {"kiteForCell"}
COUNTS = {"nEdgesOnCell", "nEdgesOnEdge", "nAdvCellsForEdge", "indexToCellID"}

VERTICAL_1D = ("fzm", "fzp", "rdzw", "rdzu", "u_init", "v_init")
SCALARS_0D = ("cf1", "cf2", "cf3")


def count_of(case: dict, loc: str) -> int:
    return {"cell": case["nCells"], "edge": case["nEdges"], "vertex": case["nVertices"]}[loc]
