#!/usr/bin/env python3
"""Write a synthetic x1.N JW case as an MPAS init file (mpas_dycore.mpas_files.write_init), optionally
declaring maxEdges / maxEdges2 as MPAS-distributed meshes do (10, 20), for bench.py --init.

    python tools/write_init.py --ncells 163842 --levels 56 --max-edges 10,20 /tmp/x1.163842.init.nc
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpas-model_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--ncells", type=int, default=163842)
    ap.add_argument("--levels", type=int, default=56)
    ap.add_argument("--order", type=int, default=3)
    ap.add_argument("--max-edges", default=None, metavar="ME[,ME2]")
    ap.add_argument("--fill", default="none", choices=("none", "repeat"))
    a = ap.parse_args()
    from mpas_dycore import mpas_files
    from mpas_dycore.cases import jw_case
    from mpas_dycore.mesh import pad_max_edges
    case = jw_case(a.ncells, K=a.levels, ns=1, order=a.order)
    if a.max_edges:
        me = [int(x) for x in a.max_edges.split(",")]
        case = pad_max_edges(case, me[0], me[1] if len(me) > 1 else 2 * me[0], a.fill)
    mpas_files.write_init(a.out, case, version=5)
    print(f"{a.out}: {case['nCells']} cells x {case['nVertLevels']} levels, maxEdges {case['maxEdges']}, "
          f"maxEdges2 {case['maxEdges2']}, dt {case['dt']:g} s, len_disp {case['config']['config_len_disp']:g} m")


if __name__ == "__main__":
    main()
