"""Synthetic benchmark / test cases of BASELINE.json (SURVEY.md §8d "Synthetic inputs").

x1.N quasi-uniform icosahedral meshes with the JW baroclinic-wave state; dt and
config_len_disp scale with resolution as SURVEY.md §8d lists them:
2562 -> 2880 s / 480 km, 10242 -> 1440 s / 240 km, 163842 -> 360 s / 60 km.
Cases are cached as .npz files (they take tens of seconds to build at 163842).
"""
from __future__ import annotations

import os
import pickle
import sys

import numpy as np

from .init_atm import build_case
from .mesh import build_mesh, build_varres_mesh

CACHE = os.environ.get("MPAS_DYCORE_CACHE", "/tmp/mpas_dycore_cache")

LEVEL_OF = {162: 2, 642: 3, 2562: 4, 10242: 5, 40962: 6, 163842: 7, 655362: 8}

# the last mesh built in this process: the dry and moist cases of one resolution share it
_MESH_MEMO: dict = {}


def _mesh(level: int, lloyd_iters: int) -> dict:
    key = (level, lloyd_iters)
    if key not in _MESH_MEMO:
        _MESH_MEMO.clear()
        _MESH_MEMO[key] = build_mesh(level, lloyd_iters=lloyd_iters)
    return _MESH_MEMO[key]


def level_for(ncells: int) -> int:
    return LEVEL_OF[ncells]


def jw_dt(level: int) -> float:
    return 360.0 * 2 ** (7 - level)


def jw_len_disp(level: int) -> float:
    return 60000.0 * 2 ** (7 - level)


def jw_case(ncells: int, K: int = 56, ns: int = 1, moist: bool = False, order: int = 2,
            lloyd_iters: int = 20, cache: bool = True) -> dict:
    level = level_for(ncells)
    key = f"jw_l{level}_K{K}_ns{ns}_m{int(moist)}_o{order}_ll{lloyd_iters}_v6"
    path = os.path.join(CACHE, key + ".pkl")
    if cache and os.path.isfile(path):
        with open(path, "rb") as f:  # our own cache file, written below
            return pickle.load(f)
    m = _mesh(level, lloyd_iters)
    cfg = dict(config_len_disp=jw_len_disp(level), config_dt=jw_dt(level), config_time_integration_order=order)
    case = build_case(m, K=K, ns=ns, moist=moist, config=cfg)
    case["dt"] = jw_dt(level)
    if cache:
        os.makedirs(CACHE, exist_ok=True)
        tmp = path + f".{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            pickle.dump(case, f, protocol=pickle.HIGHEST_PROTOCOL)
        os.replace(tmp, path)
    return case


def varres_case(ncells: int, ratio: float = 20.0, K: int = 56, ns: int = 1, moist: bool = False,
                lloyd_iters: int | None = None, cache: bool = True, order: int = 2) -> dict:
    """JW state on a variable-resolution SCVT (BASELINE.json configs[4]).

    ncells = 835586 with ratio 20: the 60-3 km mesh of configs[4] from its stored generators
    (mesh.varres_from_generators, Lloyd-relaxed offline by tools/make_varres_mesh.py); other sizes
    are generated here (mesh.build_varres_mesh).  dt and config_len_disp follow the finest spacing,
    as MPAS variable-resolution runs do (dt ~ 5 s per km of the finest cells, len_disp = finest
    spacing); ``order`` = config_time_integration_order (3 for the BASELINE runs)."""
    from .mesh import X20_835586, varres_from_generators
    stored = ncells == 835586 and ratio == 20.0 and os.path.isfile(X20_835586)
    if lloyd_iters is None:
        lloyd_iters = 40 if ncells <= 200000 else 6
    key = (f"vr_x20.835586_K{K}_ns{ns}_m{int(moist)}_o{order}_v7" if stored else
           f"vr_n{ncells}_r{ratio:g}_K{K}_ns{ns}_m{int(moist)}_ll{lloyd_iters}_o{order}_v6")
    path = os.path.join(CACHE, key + ".pkl")
    if cache and os.path.isfile(path):
        with open(path, "rb") as f:  # our own cache file, written below
            return pickle.load(f)
    m = varres_from_generators(X20_835586) if stored else build_varres_mesh(ncells, ratio=ratio,
                                                                               lloyd_iters=lloyd_iters)
    dx_min = float(m["dcEdge"].min())
    dt = float(max(1.0, round(5.0 * dx_min / 1000.0)))
    cfg = dict(config_len_disp=dx_min, config_dt=dt, config_time_integration_order=order)
    if ncells > 200000:
        print(f"varres case: mesh done ({m['nCells']} cells), building the JW state", file=sys.__stderr__, flush=True)
    case = build_case(m, K=K, ns=ns, moist=moist, config=cfg)
    case["dt"] = dt
    if cache and ncells <= 400000:  # larger cases are rebuilt rather than pickled to /tmp
        os.makedirs(CACHE, exist_ok=True)
        tmp = path + f".{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            pickle.dump(case, f, protocol=pickle.HIGHEST_PROTOCOL)
        os.replace(tmp, path)
    return case


def regional_lbc(case: dict, interior_deg: float = 40.0, interval_end: float = 10800.0) -> tuple[dict, dict]:
    """A limited-area configuration on a global case (config_apply_lbcs): the cells farther than
    ``interior_deg`` from (0N, 0E) form the boundary zones, ring by ring outward -- bdyMaskCell 1..5
    relaxation, 6 and 7 (and everything beyond) specified -- as a regional mesh's masks count them
    (mpas_atm_boundaries.F:10-12).  Edges take the smaller mask of their two cells.  Also sets
    specZoneMask* and nearestRelaxationCell as mpas_atm_setup_bdy_masks does (:426-495; here every
    specified cell gets its nearest relaxation cell of mask 5, so no read falls outside the mesh)
    and meshScalingRegional* as atm_compute_mesh_scaling (mpas_atm_core.F:967-981).  Returns the
    case with these fields and the driving data of the lbc pool: lbc_<f>_s (interval-end state) and
    lbc_<f>_t (tendency) for u, ru, rho_zz, rtheta_m and scalars, element-major, plus
    ``interval_end`` = seconds from the first step's start to the LBC interval end."""
    import numpy as np
    from .init_atm import _pow
    c = dict(case)
    nC, nE = c["nCells"], c["nEdges"]
    lat, lon = np.asarray(c["latCell"]), np.asarray(c["lonCell"])
    ang = np.degrees(np.arccos(np.clip(np.cos(lat) * np.cos(lon), -1.0, 1.0)))
    mask = np.full(nC, 99, dtype=np.int64)
    mask[ang < interior_deg] = 0
    coc, noc = np.asarray(c["cellsOnCell"]), np.asarray(c["nEdgesOnCell"])
    ring = np.flatnonzero(mask == 0)
    for r in range(1, 8):
        nb = coc[ring]
        nb = nb[np.arange(coc.shape[1])[None, :] < noc[ring][:, None]]
        nb = np.unique(nb[nb >= 0])
        ring = nb[mask[nb] == 99]
        mask[ring] = r
    mask[mask == 99] = 7
    coe = np.asarray(c["cellsOnEdge"])
    emask = np.minimum(mask[coe[:, 0]], mask[coe[:, 1]])
    c["bdyMaskCell"] = mask.astype(np.int32)
    c["bdyMaskEdge"] = emask.astype(np.int32)
    c["specZoneMaskCell"] = (mask > 5).astype(np.float64)
    c["specZoneMaskEdge"] = (emask > 5).astype(np.float64)
    xyz = np.stack([np.asarray(c["xCell"]), np.asarray(c["yCell"]), np.asarray(c["zCell"])], 1)
    relax = np.flatnonzero(mask == 5)
    near = np.full(nC, -1, dtype=np.int64)
    for i in np.flatnonzero(mask > 5):
        d2 = ((xyz[relax] - xyz[i]) ** 2).sum(1)
        near[i] = relax[np.argmin(d2)]
    c["nearestRelaxationCell"] = near
    md = np.asarray(c.get("meshDensity", np.ones(nC)), dtype=np.float64)
    c["meshScalingRegionalCell"] = 1.0 / _pow(md, 0.25)
    c["meshScalingRegionalEdge"] = 1.0 / _pow((md[coe[:, 0]] + md[coe[:, 1]]) / 2.0, 0.25)
    # driving data: the initial state with a smooth perturbation at the interval end, and the
    # tendency that leads there
    K, ns = c["nVertLevels"], c["num_scalars"]
    zz = np.asarray(c["zz"])
    rho_zz = np.asarray(c["rho"]) / zz
    sc = np.asarray(c["scalars"]).reshape(nC, K, ns)
    theta_m = np.asarray(c["theta"]) * (1.0 + 461.6 / 287.0 * sc[:, :, 0])
    u = np.asarray(c["u"])
    ru = u * 0.5 * (rho_zz[coe[:, 0]] + rho_zz[coe[:, 1]])
    lonE, latE = np.asarray(c["lonEdge"]), np.asarray(c["latEdge"])
    pc, pe = 0.003 * np.cos(lon)[:, None], 0.003 * np.cos(lonE)[:, None]
    tc, te = 1e-7 * np.sin(lat)[:, None], 1e-7 * np.sin(latE)[:, None]
    lbc = {"interval_end": float(interval_end)}
    for name, base, p_, t_ in (("u", u, pe, te), ("ru", ru, pe, te), ("rho_zz", rho_zz, pc, tc),
                               ("rtheta_m", rho_zz * theta_m, pc, tc)):
        lbc[f"lbc_{name}_s"] = base * (1.0 + p_)
        lbc[f"lbc_{name}_t"] = base * t_
    lbc["lbc_scalars_s"] = sc * (1.0 + 3.0 * pc[:, :, None])
    lbc["lbc_scalars_t"] = sc * tc[:, :, None]
    return c, lbc
