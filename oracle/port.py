"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the C restatement (oracle/c/atm_port.c)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_ref", "libatm_port.so")

_I = C.POINTER(C.c_int32)
_D = C.POINTER(C.c_double)


class AcousticArgs(C.Structure):
    _fields_ = [("nCells", C.c_int32), ("nEdges", C.c_int32), ("nCellsSolve", C.c_int32), ("K", C.c_int32),
                ("maxEdges", C.c_int32),
                ("cellsOnEdge", _I), ("edgesOnCell", _I), ("nEdgesOnCell", _I),
                ("edgesOnCell_sign", _D), ("invDcEdge", _D), ("dvEdge", _D), ("invAreaCell", _D),
                ("specZoneMaskEdge", _D), ("specZoneMaskCell", _D),
                ("zz", _D), ("zxu", _D), ("dss", _D), ("fzm", _D), ("fzp", _D), ("rdzw", _D),
                ("theta_m", _D), ("rho_zz", _D), ("w", _D), ("exner", _D), ("cqu", _D),
                ("cofwr", _D), ("cofwz", _D), ("cofwt", _D), ("coftz", _D), ("cofrz", _D), ("a_tri", _D),
                ("alpha_tri", _D), ("gamma_tri", _D),
                ("tend_ru", _D), ("tend_rho", _D), ("tend_rt", _D), ("tend_rw", _D), ("rw", _D), ("rw_save", _D),
                ("ru_p", _D), ("ruAvg", _D), ("rho_pp", _D), ("rtheta_pp", _D), ("rtheta_pp_old", _D),
                ("rw_p", _D), ("wwAvg", _D)]


def available() -> bool:
    return os.path.isfile(LIB)


def acoustic_substep(mesh: dict, fields: dict, dts, small_step, epssm, smdiv, len_disp, nthreads=0) -> dict:
    """mesh: element-major arrays (0-based indices); fields: name -> element-major array (no garbage row).
    Returns the updated fields (copies)."""
    lib = C.CDLL(LIB)
    lib.atm_port_acoustic_substep.argtypes = [C.POINTER(AcousticArgs), C.c_double, C.c_int, C.c_double,
                                              C.c_double, C.c_double, C.c_int]
    keep = []

    def garb(a, dtype=np.float64, fill=0):
        a = np.asarray(a, dtype=dtype)
        pad = np.full((1,) + a.shape[1:], fill, dtype=dtype)
        b = np.ascontiguousarray(np.concatenate([a, pad], 0))
        keep.append(b)
        return b

    def flat(a, dtype=np.float64):
        b = np.ascontiguousarray(np.asarray(a, dtype=dtype))
        keep.append(b)
        return b

    nC, nE = mesh["nCells"], mesh["nEdges"]
    args = AcousticArgs()
    args.nCells, args.nEdges, args.nCellsSolve, args.K, args.maxEdges = nC, nE, nC, mesh["K"], mesh["maxEdges"]
    coe = np.where(mesh["cellsOnEdge"] >= 0, mesh["cellsOnEdge"], nC)
    eoc = np.where(mesh["edgesOnCell"] >= 0, mesh["edgesOnCell"], nE)
    args.cellsOnEdge = garb(coe, np.int32, nC).ctypes.data_as(_I)
    args.edgesOnCell = garb(eoc, np.int32, nE).ctypes.data_as(_I)
    args.nEdgesOnCell = garb(mesh["nEdgesOnCell"], np.int32).ctypes.data_as(_I)
    for n in ("edgesOnCell_sign", "invAreaCell", "zz", "dss"):
        setattr(args, n, garb(mesh[n]).ctypes.data_as(_D))
    for n in ("invDcEdge", "dvEdge", "zxu"):
        setattr(args, n, garb(mesh[n]).ctypes.data_as(_D))
    args.specZoneMaskEdge = garb(np.zeros(nE)).ctypes.data_as(_D)
    args.specZoneMaskCell = garb(np.zeros(nC)).ctypes.data_as(_D)
    for n in ("fzm", "fzp", "rdzw", "cofrz"):
        src = mesh if n in mesh else fields
        setattr(args, n, flat(src[n]).ctypes.data_as(_D))
    outs = {}
    for n in ("theta_m", "rho_zz", "w", "exner", "cqu", "cofwr", "cofwz", "cofwt", "coftz", "a_tri", "alpha_tri",
              "gamma_tri", "tend_ru", "tend_rho", "tend_rt", "tend_rw", "rw", "rw_save", "ru_p", "ruAvg", "rho_pp",
              "rtheta_pp", "rtheta_pp_old", "rw_p", "wwAvg"):
        b = garb(fields[n])
        outs[n] = b
        setattr(args, n, b.ctypes.data_as(_D))
    lib.atm_port_acoustic_substep(C.byref(args), float(dts), int(small_step), float(epssm), float(smdiv),
                                  float(len_disp), int(nthreads))
    return {n: outs[n][:-1].copy() for n in ("ru_p", "ruAvg", "rho_pp", "rtheta_pp", "rtheta_pp_old", "rw_p", "wwAvg")}
