"""Element-major numpy <-> MPAS Fortran memory image (garbage slot, 1-based indices)."""
import numpy as np

from mpas_dycore.layout import to_fortran


def test_index_and_real_conversion(small_case):
    c = small_case
    eoc = to_fortran(c, "edgesOnCell")
    assert eoc.dtype == np.int32 and eoc.shape == (c["nCells"] + 1, c["maxEdges"])
    assert eoc[:-1].min() >= 1 and eoc.max() <= c["nEdges"] + 1
    assert (eoc[-1] == c["nEdges"] + 1).all()                       # garbage row -> garbage slot
    pent = np.nonzero(c["nEdgesOnCell"] == 5)[0][0]
    assert eoc[pent, 5] == c["nEdges"] + 1                          # missing neighbour -> n+1
    assert (to_fortran(c, "kiteForCell")[:-1] >= 1).all()
    u = to_fortran(c, "u")
    assert u.shape == (c["nEdges"] + 1, c["nVertLevels"]) and (u[-1] == 0).all()
    np.testing.assert_array_equal(u[:-1], c["u"])
    zb = to_fortran(c, "zb_cell")
    assert zb.shape == (c["nCells"] + 1, c["maxEdges"], c["nVertLevels"] + 1)
