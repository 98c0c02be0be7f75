#!/usr/bin/env python3
"""Dump the x1.N mesh index streams the gather kernels read (in the library's device form: 0-based,
missing -> the garbage element, maxEdges2 slots packed to 10) and run tools/gather_floor on them.

    python tools/gather_floor.py [--ncells 163842] [--levels 56] [--ns 1] [--reps 20] [--rounds 5]
"""
import argparse
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpas-model_amd"))


def dump(case, out):
    os.makedirs(out, exist_ok=True)
    nC, nE, nV, K = case["nCells"], case["nEdges"], case["nVertices"], case["nVertLevels"]

    def idx(a, n_tgt, width):
        a = np.asarray(a)[:, :width]
        a = np.where((a >= 0) & (a < n_tgt), a, n_tgt).astype(np.int32)
        return np.concatenate([a, np.full((1, width), n_tgt, np.int32)])

    def real(a, width):
        a = np.asarray(a, dtype=np.float64)[:, :width]
        return np.concatenate([a, np.zeros((1, width))])
    files = {
        "advCellsForEdge.i32": idx(case["advCellsForEdge"], nC, 15),
        "nAdvCellsForEdge.i32": np.append(np.asarray(case["nAdvCellsForEdge"]), 0).astype(np.int32),
        "cellsOnEdge.i32": idx(case["cellsOnEdge"], nC, 2),
        "edgesOnEdge.i32": idx(case["edgesOnEdge"], nE, 10),
        "nEdgesOnEdge.i32": np.append(np.asarray(case["nEdgesOnEdge"]), 0).astype(np.int32),
        "adv_coefs.f64": real(case["adv_coefs"], 15),
        "adv_coefs_3rd.f64": real(case["adv_coefs_3rd"], 15),
        "weightsOnEdge.f64": real(case["weightsOnEdge"], 10),
    }
    # k_build_cell_rec's records: [0, 7) edgesOnCell, [7, 14) the cell across each edge, [14] nEdgesOnCell
    ne = np.asarray(case["nEdgesOnCell"])
    eoc = np.asarray(case["edgesOnCell"])[:, :7]
    coe = np.asarray(case["cellsOnEdge"])
    rec = np.zeros((nC + 1, 16), np.int32)
    rec[:, :7] = nE
    rec[:, 7:14] = nC
    for m in range(eoc.shape[1]):
        live = m < ne
        e = np.where(live, eoc[:, m], 0)
        other = np.where(coe[e, 0] == np.arange(nC), coe[e, 1], coe[e, 0])
        rec[:nC, m] = np.where(live, e, nE)
        rec[:nC, 7 + m] = np.where(live & (other >= 0), other, nC)
    rec[:nC, 14] = ne
    rec[nC, 14] = 0
    files["cell_rec.i32"] = rec
    for n, a in files.items():
        np.ascontiguousarray(a).tofile(os.path.join(out, n))
    return nC, nE, nV, K


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ncells", type=int, default=163842)
    ap.add_argument("--levels", type=int, default=56)
    ap.add_argument("--ns", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--dir", default="/tmp/gather_floor")
    a = ap.parse_args()
    from mpas_dycore.cases import jw_case
    case = jw_case(a.ncells, K=a.levels, ns=1, order=3)
    nC, nE, nV, K = dump(case, a.dir)
    with open(os.path.join(a.dir, "meta.txt"), "w") as f:
        f.write(f"{nC} {nE} {nV} {K} {a.ns}\n")
    exe = os.path.join(ROOT, "tools", "gather_floor")
    r = subprocess.run([exe, a.dir, str(a.reps), str(a.rounds)], capture_output=True, text=True)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
