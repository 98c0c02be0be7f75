"""MPAS mesh / initial-condition files <-> dycore cases.

The reference reads its mesh and initial state from the `input` stream of
core_atmosphere (Registry.xml:398-470, file `x1.N.init.nc`, produced by
init_atmosphere from `x1.N.grid.nc` / `x1.N.static.nc`), through PIO
(framework/mpas_io.F, mpas_io_streams.F).  This module maps those files onto the
flat case dict that `Dycore` uploads (init_atm.build_case's layout):

* `read_mesh(path)`  -- the horizontal mesh of any MPAS grid/static/init file;
* `read_init(path, config)` -- mesh + vertical grid + initial state of an init file,
  then the dycore's model-init precompute (init_atm.model_init, the restatement of
  mpas_atm_core.F:311-463, 927-1288), i.e. what atm_mpas_init_block does before
  the first atm_timestep;
* `write_mesh` / `write_init` -- the reverse, in the same variable names, dimension
  names and index conventions, so files round-trip and can be handed to MPAS tools.

Conventions (as in the files MPAS writes): netCDF arrays are the C-order view of the
Fortran arrays (`cellsOnEdge(TWO, nEdges)` -> `[nEdges, TWO]`), element indices are
1-based with 0 for "none"; the case dict holds them 0-based with -1 for "none".
Time-dependent fields carry a leading `Time` record dimension; the first record is
the initial state.  Scalars (`var_array scalars`, Registry.xml) are one variable per
constituent (qv, qc, ...), stacked on the last axis in the order given.
"""
from __future__ import annotations

import numpy as np

from . import ncio

MESH_INDEX = {  # name -> target set, for the 1-based <-> 0-based conversion
    "cellsOnEdge": "cell", "edgesOnCell": "edge", "edgesOnEdge": "edge", "cellsOnCell": "cell",
    "verticesOnCell": "vertex", "verticesOnEdge": "vertex", "edgesOnVertex": "edge", "cellsOnVertex": "cell",
}
MESH_COUNTS = ("nEdgesOnCell", "nEdgesOnEdge", "indexToCellID", "indexToEdgeID", "indexToVertexID")
MESH_REAL = {
    "cell": ("latCell", "lonCell", "xCell", "yCell", "zCell", "areaCell", "meshDensity"),
    "edge": ("latEdge", "lonEdge", "xEdge", "yEdge", "zEdge", "dvEdge", "dcEdge", "angleEdge", "fEdge"),
    "vertex": ("latVertex", "lonVertex", "xVertex", "yVertex", "zVertex", "areaTriangle", "fVertex"),
}
MESH_2D = {  # name -> netCDF dimensions (C order)
    "cellsOnEdge": ("nEdges", "TWO"), "verticesOnEdge": ("nEdges", "TWO"),
    "edgesOnCell": ("nCells", "maxEdges"), "cellsOnCell": ("nCells", "maxEdges"),
    "verticesOnCell": ("nCells", "maxEdges"), "edgesOnEdge": ("nEdges", "maxEdges2"),
    "weightsOnEdge": ("nEdges", "maxEdges2"), "edgesOnVertex": ("nVertices", "vertexDegree"),
    "cellsOnVertex": ("nVertices", "vertexDegree"), "kiteAreasOnVertex": ("nVertices", "vertexDegree"),
}
# input-stream fields of the vertical grid and model-init inputs (Registry.xml:447-469)
INIT_FIXED = {
    "zgrid": ("nCells", "nVertLevelsP1"), "zz": ("nCells", "nVertLevels"), "zxu": ("nEdges", "nVertLevels"),
    "zb": ("nEdges", "TWO", "nVertLevelsP1"), "zb3": ("nEdges", "TWO", "nVertLevelsP1"),
    "dss": ("nCells", "nVertLevels"), "rdzw": ("nVertLevels",), "rdzu": ("nVertLevels",),
    "dzu": ("nVertLevels",), "fzm": ("nVertLevels",), "fzp": ("nVertLevels",),
    "u_init": ("nVertLevels",), "v_init": ("nVertLevels",), "qv_init": ("nVertLevels",),
    "t_init": ("nCells", "nVertLevels"), "deriv_two": ("nEdges", "TWO", "FIFTEEN"),
    "defc_a": ("nCells", "maxEdges"), "defc_b": ("nCells", "maxEdges"),
    "coeffs_reconstruct": ("nCells", "maxEdges", "R3"),
}
INIT_STATE = {
    "u": ("nEdges", "nVertLevels"), "w": ("nCells", "nVertLevelsP1"), "rho": ("nCells", "nVertLevels"),
    "theta": ("nCells", "nVertLevels"), "rho_base": ("nCells", "nVertLevels"),
    "theta_base": ("nCells", "nVertLevels"),
}
# the constituents of a WSM6-like scalar set, in the order of the reference's moist species
DEFAULT_SCALARS = ("qv", "qc", "qr", "qi", "qs", "qg")


def _count(loc, m):
    return {"cell": m["nCells"], "edge": m["nEdges"], "vertex": m["nVertices"]}[loc]


def read_mesh(path_or_ds) -> dict:
    """Horizontal mesh of an MPAS grid/static/init file as a 0-based mesh dict."""
    ds = ncio.read(path_or_ds) if isinstance(path_or_ds, str) else path_or_ds
    m = dict(nCells=ds.dims["nCells"], nEdges=ds.dims["nEdges"], nVertices=ds.dims["nVertices"],
             maxEdges=ds.dims["maxEdges"], maxEdges2=ds.dims["maxEdges2"],
             vertexDegree=ds.dims.get("vertexDegree", 3))
    r = ds.attrs.get("sphere_radius", None)
    m["sphere_radius"] = float(np.asarray(r).ravel()[0]) if r is not None else 6371229.0
    if str(ds.attrs.get("on_a_sphere", "YES")).strip().upper() != "YES":
        raise ValueError("only spherical meshes (on_a_sphere = YES) are supported")
    for loc, names in MESH_REAL.items():
        for n in names:
            if n in ds:
                m[n] = np.asarray(ds[n], dtype=np.float64)
    for n in ("weightsOnEdge", "kiteAreasOnVertex"):
        m[n] = np.asarray(ds[n], dtype=np.float64)
    for n in MESH_COUNTS:
        if n in ds:
            m[n] = np.asarray(ds[n], dtype=np.int64)
    for n, tgt in MESH_INDEX.items():
        a = np.asarray(ds[n], dtype=np.int64)
        nt = _count(tgt, m)
        m[n] = np.where((a >= 1) & (a <= nt), a - 1, -1)
    if "meshDensity" not in m:
        m["meshDensity"] = np.ones(m["nCells"])
    if "indexToCellID" not in m:
        m["indexToCellID"] = np.arange(1, m["nCells"] + 1)
    return m


def _mesh_dataset(m: dict, ds: ncio.Dataset | None = None) -> ncio.Dataset:
    ds = ds or ncio.Dataset(unlimited="Time")
    ds.attrs.update(on_a_sphere="YES", sphere_radius=float(m.get("sphere_radius", 6371229.0)), is_periodic="NO",
                    mesh_spec="1.0", source="mpas-model_amd")
    for d in ("nCells", "nEdges", "nVertices", "maxEdges", "maxEdges2", "vertexDegree"):
        ds.dims[d] = int(m.get(d, 3))
    ds.dims["TWO"] = 2
    for loc, names in MESH_REAL.items():
        for n in names:
            if n in m:
                ds.add(n, ({"cell": "nCells", "edge": "nEdges", "vertex": "nVertices"}[loc],), m[n])
    for n in MESH_COUNTS:
        loc = {"nEdgesOnCell": "nCells", "nEdgesOnEdge": "nEdges", "indexToCellID": "nCells",
               "indexToEdgeID": "nEdges", "indexToVertexID": "nVertices"}[n]
        if n in m:
            ds.add(n, (loc,), np.asarray(m[n], dtype=np.int32))
        elif n == "indexToEdgeID" or n == "indexToVertexID":
            ds.add(n, (loc,), np.arange(1, ds.dims[loc] + 1, dtype=np.int32))
    for n, dims in MESH_2D.items():
        a = np.asarray(m[n])
        if n in MESH_INDEX:
            a = np.where(a >= 0, a + 1, 0).astype(np.int32)
        ds.add(n, dims, a)
    return ds


def write_mesh(path: str, m: dict, version: int = 2) -> None:
    """A grid file (the mesh fields of x1.N.grid.nc)."""
    ncio.write(path, _mesh_dataset(m), version=version)


def write_init(path: str, case: dict, scalar_names=None, version: int = 2,
               xtime: str = "0000-01-01_00:00:00") -> None:
    """An init file: mesh, vertical grid, model-init inputs and the initial state (Time record 0)."""
    ds = _mesh_dataset(case)
    K = case["nVertLevels"]
    ds.dims.update(nVertLevels=K, nVertLevelsP1=K + 1, FIFTEEN=15, R3=3, StrLen=64)
    for n in ("cf1", "cf2", "cf3"):
        ds.add(n, (), np.float64(case[n]))
    for n, dims in INIT_FIXED.items():
        if n in case:
            ds.add(n, dims, np.asarray(case[n], dtype=np.float64))
    for n, dims in INIT_STATE.items():
        ds.add(n, ("Time",) + dims, np.asarray(case[n], dtype=np.float64)[None])
    ns = case["num_scalars"]
    names = list(scalar_names or DEFAULT_SCALARS[:ns])
    if len(names) < ns:
        names += [f"scalar{i + 1}" for i in range(len(names), ns)]
    for i, n in enumerate(names[:ns]):
        ds.add(n, ("Time", "nCells", "nVertLevels"), np.ascontiguousarray(case["scalars"][:, :, i])[None])
    ds.add("xtime", ("Time", "StrLen"), np.frombuffer(xtime.encode().ljust(64), dtype="S1")[None])
    ds.add("initial_time", ("StrLen",), np.frombuffer(xtime.encode().ljust(64), dtype="S1"))
    ncio.write(path, ds, version=version)


def read_init(path: str, config: dict | None = None, scalar_names=None, record: int = 0) -> dict:
    """An MPAS init file as a dycore case: the input-stream fields of record ``record`` plus the
    model-init precompute.  ``config`` holds namelist values (init_atm.DEFAULT_CONFIG keys);
    ``scalar_names`` the constituents to carry, default every one of qv, qc, qr, qi, qs, qg present."""
    from .init_atm import DEFAULT_CONFIG, model_init

    ds = ncio.read(path)
    case = read_mesh(ds)
    K = ds.dims["nVertLevels"]
    case["nVertLevels"] = K
    for n in ("cf1", "cf2", "cf3"):
        case[n] = np.float64(np.asarray(ds[n]).ravel()[0])
    for n in INIT_FIXED:
        if n in ds:
            case[n] = np.asarray(ds[n], dtype=np.float64)
    for n in INIT_STATE:
        a = np.asarray(ds[n], dtype=np.float64)
        case[n] = np.ascontiguousarray(a[record] if ds.vars[n].dims[0] == ds.unlimited else a)
    names = [n for n in (scalar_names or DEFAULT_SCALARS) if n in ds]
    if scalar_names and len(names) != len(scalar_names):
        raise KeyError(f"scalars missing from {path}: {sorted(set(scalar_names) - set(names))}")
    if not names:
        raise KeyError(f"{path} holds none of the scalars {list(scalar_names or DEFAULT_SCALARS)}")
    case["scalars"] = np.ascontiguousarray(
        np.stack([np.asarray(ds[n], dtype=np.float64)[record] for n in names], axis=-1))
    case["num_scalars"] = len(names)
    case["scalar_names"] = names
    cfg = dict(DEFAULT_CONFIG)
    if config:
        cfg.update(config)
    # vertical-grid / model-init inputs the dycore needs beyond the mesh (init_atm.model_init)
    missing = [n for n in ("zgrid", "zz", "zxu", "zb", "zb3", "deriv_two", "rdzw", "rdzu", "fzm", "fzp")
               if n not in case]
    if missing:
        raise KeyError(f"{path} is not an init file: missing {missing}")
    case = model_init(case, cfg)
    if "config_dt" in cfg:
        case["dt"] = float(cfg["config_dt"])
    return case
