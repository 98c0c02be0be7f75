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
    key = f"jw_l{level}_K{K}_ns{ns}_m{int(moist)}_o{order}_ll{lloyd_iters}_v4"
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
                lloyd_iters: int | None = None, cache: bool = True) -> dict:
    """JW state on a variable-resolution SCVT (BASELINE.json configs[4] analogue).

    dt and config_len_disp follow the finest spacing, as MPAS variable-resolution runs do
    (dt ~ 5 s per km of the finest cells, len_disp = finest spacing)."""
    if lloyd_iters is None:
        lloyd_iters = 40 if ncells <= 200000 else 6
    key = f"vr_n{ncells}_r{ratio:g}_K{K}_ns{ns}_m{int(moist)}_ll{lloyd_iters}_v5"
    path = os.path.join(CACHE, key + ".pkl")
    if cache and os.path.isfile(path):
        with open(path, "rb") as f:  # our own cache file, written below
            return pickle.load(f)
    m = build_varres_mesh(ncells, ratio=ratio, lloyd_iters=lloyd_iters)
    dx_min = float(m["dcEdge"].min())
    dt = float(max(1.0, round(5.0 * dx_min / 1000.0)))
    cfg = dict(config_len_disp=dx_min, config_dt=dt)
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
