"""Host-side mirror of the reference dycore interface over the C ABI.

The reference's operator API is the Fortran module ``atm_time_integration``
(mpas_atm_time_integration.F): the core driver calls ``atm_timestep`` each
step (mpas_atm_core.F:873), ``atm_init_coupled_diagnostics`` and
``atm_compute_solve_diagnostics`` at init (mpas_atm_core.F:390,399), and
shifts state time levels after each step (mpas_atm_core.F:671).  ``Dycore``
exposes exactly those operations; fields are addressed by (pool, name,
timeLevel) as in ``mpas_pool_get_array`` (mpas_pool_routines.F:4282), and
travel as element-major numpy arrays (the transpose-free view of the Fortran
(K, n+1) memory image).  Errors raise ``DycoreError`` (the reference aborts
through MPAS_LOG_CRIT, mpas_log.F:612).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from . import fields as F
from .layout import LOC_N, to_fortran

STATE_INPUTS = ("u", "w", "scalars")
DIAG_INPUTS = ("theta", "rho", "rho_base", "theta_base")
_SKIP = set(STATE_INPUTS) | set(DIAG_INPUTS) | {"xCell", "yCell", "zCell", "xEdge", "yEdge", "zEdge", "xVertex",
                                                "yVertex", "zVertex", "latCell", "lonCell", "latEdge", "lonEdge",
                                                "latVertex", "lonVertex", "areaCell", "areaTriangle",
                                                "meshDensity", "indexToCellID", "deriv_two", "zb", "zb3"}


class DycoreError(RuntimeError):
    pass


class Dycore:
    """One block of the MI355X dycore (all cells owned unless ``solve`` counts are given)."""

    def __init__(self, case: dict, device: int = 0, solve: tuple | None = None, moist_end: int = 1):
        self.lib = _lib.load()
        self.case = case
        self.K = case["nVertLevels"]
        self.ns = case["num_scalars"]
        self.n = {"cell": case["nCells"], "edge": case["nEdges"], "vertex": case["nVertices"]}
        d = _lib.Dims()
        d.nCells, d.nEdges, d.nVertices = case["nCells"], case["nEdges"], case["nVertices"]
        d.nVertLevels, d.maxEdges, d.maxEdges2 = self.K, case["maxEdges"], case["maxEdges2"]
        d.num_scalars = self.ns
        if solve is None:
            solve = (case["nCells"], case["nEdges"], case["nVertices"])
        d.nCellsSolve, d.nEdgesSolve, d.nVerticesSolve = solve
        d.moist_start, d.moist_end, d.index_qv = 1, moist_end, 1
        cfg = _lib.make_config(case["config"])
        h = C.c_void_p()
        rc = self.lib.mpas_dyc_create(C.byref(d), C.byref(cfg), int(device), C.byref(h))
        if rc != 0 or not h.value:
            raise DycoreError(f"mpas_dyc_create failed ({rc})")
        self.h = h
        self._upload_case(case)

    # -------------------------------------------------------------- fields
    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.mpas_dyc_last_error(self.h)
            raise DycoreError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def set_raw(self, pool: str, name: str, fortran_image: np.ndarray, time_level: int = 1):
        a = np.ascontiguousarray(fortran_image)
        self._check(self.lib.mpas_dyc_set_field(self.h, pool.encode(), name.encode(), time_level,
                                                a.ctypes.data_as(C.c_void_p), a.nbytes), f"set {pool}.{name}")

    def set(self, pool: str, name: str, arr, time_level: int = 1):
        """Upload an element-major array (0-based indices for index fields)."""
        self.set_raw(pool, name, to_fortran({**self.case, name: arr}, name), time_level)

    def get(self, pool: str, name: str, time_level: int = 1) -> np.ndarray:
        """Download a real field as element-major (n, inner) numpy (garbage slot dropped)."""
        nb = self.lib.mpas_dyc_field_bytes(self.h, pool.encode(), name.encode())
        if nb <= 0:
            raise DycoreError(f"unknown field {pool}.{name}")
        buf = np.empty(nb // 8, dtype=np.float64)
        self._check(self.lib.mpas_dyc_get_field(self.h, pool.encode(), name.encode(), time_level,
                                                buf.ctypes.data_as(C.c_void_p), buf.nbytes), f"get {pool}.{name}")
        loc = _loc_of(pool, name)
        if loc is None:
            return buf
        n1 = self.n[loc] + 1
        if name in ("scalars", "scalars_tend"):
            return buf.reshape(n1, self.K, self.ns)[:-1]
        return buf.reshape(n1, buf.size // n1)[:-1]

    def _upload_case(self, case: dict):
        for name in case:
            if name in _SKIP:
                continue
            if name in F.LOCATION or name in F.VERTICAL_1D:
                if name in F.VERTICAL_1D:
                    self.set_raw("mesh", name, np.asarray(case[name], dtype=np.float64))
                else:
                    self.set_raw("mesh", name, to_fortran(case, name))
            elif name in F.SCALARS_0D:
                self.set_raw("mesh", name, np.asarray([case[name]], dtype=np.float64))
        for name in STATE_INPUTS:
            self.set_raw("state", name, to_fortran(case, name), 1)
        for name in DIAG_INPUTS:
            self.set_raw("diag", name, to_fortran(case, name))

    # -------------------------------------------------------- operators
    def init_diagnostics(self, dt: float):
        """atm_init_coupled_diagnostics + atm_compute_solve_diagnostics (mpas_atm_core.F:387-404)."""
        self._check(self.lib.mpas_dyc_init_diagnostics(self.h, float(dt)), "init_diagnostics")

    def atm_timestep(self, dt: float, itimestep: int = 1):
        """atm_timestep -> atm_srk3 (mpas_atm_time_integration.F:87-139); asynchronous."""
        self._check(self.lib.mpas_dyc_timestep(self.h, float(dt), int(itimestep)), "atm_timestep")

    def shift_time_levels(self):
        self._check(self.lib.mpas_dyc_shift_time_levels(self.h), "shift_time_levels")

    def synchronize(self):
        self._check(self.lib.mpas_dyc_synchronize(self.h), "synchronize")

    def use_graph(self, on: bool = True):
        self._check(self.lib.mpas_dyc_use_graph(self.h, 1 if on else 0), "use_graph")

    def time_acoustic_step(self, dts: float, small_step: int = 2, reps: int = 10):
        ms = C.c_double()
        ks = (C.c_double * 3)()
        self._check(self.lib.mpas_dyc_time_acoustic_step(self.h, float(dts), int(small_step), int(reps),
                                                         C.byref(ms), ks), "time_acoustic_step")
        return ms.value, list(ks)

    def acoustic_bytes(self) -> float:
        return self.lib.mpas_dyc_acoustic_bytes(self.h)

    def close(self):
        if getattr(self, "h", None):
            self.lib.mpas_dyc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# horizontal location of device fields not in fields.LOCATION
_LOCS = {}
for _n in ("theta_m", "rho_zz", "rho_p", "rtheta_p", "exner", "pressure_p", "kdiff", "ke", "divergence", "rw",
           "wwAvg", "cqw", "h_divergence", "pv_cell", "rho_pp", "rtheta_pp", "rw_p", "exner_base", "pressure_base",
           "rtheta_base", "coftz", "cofwz", "cofwr", "cofwt", "a_tri", "alpha_tri", "gamma_tri", "rw_save",
           "tend_rtheta_adv", "rho_p_save", "rtheta_p_save", "rho_zz_old_split", "rtheta_pp_old", "wwAvg_split",
           "scalars_tend", "rthdynten", "rt_diabatic_tend", "theta_euler", "w_euler"):
    _LOCS[_n] = "cell"
for _n in ("ru", "ruAvg", "ru_p", "ru_save", "cqu", "rho_edge", "v", "pv_edge", "gradPVn", "gradPVt",
           "ruAvg_split", "u_euler"):
    _LOCS[_n] = "edge"
for _n in ("vorticity", "pv_vertex"):
    _LOCS[_n] = "vertex"


def _loc_of(pool: str, name: str):
    if pool == "tend" and name == "u":
        return "edge"
    if name in _LOCS:
        return _LOCS[name]
    return F.LOCATION.get(name)
