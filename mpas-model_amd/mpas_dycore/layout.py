"""Element-major numpy arrays <-> MPAS Fortran memory images.

A Fortran pool array ``x(K, n+1)`` is, in memory, the C-order array
``[n+1][K]`` -- exactly the HBM layout of the device fields.  Element-major
numpy arrays (n, ...) therefore only need the garbage row n+1 appended and,
for index arrays, the 0-based -> 1-based shift with "missing" -> n+1
(mpas_block_creator.F:1445, 1471).
"""
from __future__ import annotations

import numpy as np

from . import fields as F

LOC_N = {"cell": "nCells", "edge": "nEdges", "vertex": "nVertices"}


def to_fortran(case: dict, name: str) -> np.ndarray:
    a = np.asarray(case[name])
    if name in F.INDEX_TARGET:
        n_tgt = case[LOC_N[F.INDEX_TARGET[name]]]
        a = np.where(a >= 0, a + 1, n_tgt + 1).astype(np.int32)
    elif name in F.ONE_BASED_SMALL:
        a = (a + 1).astype(np.int32)
    elif a.dtype.kind in "iu":
        a = a.astype(np.int32)
    else:
        a = a.astype(np.float64)
    loc = F.LOCATION.get(name)
    if loc is not None:
        n = case[LOC_N[loc]]
        if a.shape[0] != n:
            raise ValueError(f"{name}: leading dim {a.shape[0]} != {LOC_N[loc]}={n}")
        pad = np.zeros((1,) + a.shape[1:], dtype=a.dtype)
        if name in F.INDEX_TARGET:
            pad[...] = case[LOC_N[F.INDEX_TARGET[name]]] + 1
        a = np.concatenate([a, pad], axis=0)
    return np.ascontiguousarray(a)


def from_fortran(buf: np.ndarray, n: int, inner_shape=()) -> np.ndarray:
    """Fortran image with garbage slot -> element-major (n, *inner_shape)."""
    return buf.reshape((n + 1,) + tuple(inner_shape))[:n]
