#!/usr/bin/env python3
"""Whole-dt roofline table: every kernel of one atm_timestep, its algorithmic bytes per launch
(SURVEY.md §8d's rule), its measured time, and the PMC-counted HBM traffic.

    python tools/kernel_roofline.py KERNEL_STATS.csv PMC.json STEPS [NCELLS LEVELS [NS]] > profiles/r03_kernel_roofline.csv

With NS > 1 (the moist transport, scalar-major scalars): the monotone pipeline's kernels (k_mono_*
but k_mono_prep) run one launch per pair of scalars (MonoFlux2, a second set of scratch), so their
scalars / scalars_tend count 2 of NS scalar columns and their per-scalar scratch twice.

Algorithmic bytes of a launch = the sum, over the arrays the kernel reads and over those it writes
(tools/kernel_access.py, resolved per template variant below), of the array's size over the
elements of its location the launch covers.  Each distinct array counts once per read and once per
write; neighbour gathers count nothing extra ("neighbour gathers assumed
cache-reused").  One block, so every launch covers all cells / edges / vertices (owned = all).
The PMC bytes come from tools/pmc_summary.py (FETCH_SIZE x calibration + WRITE_SIZE, per
dispatch, eager launches).  Columns:
  kernel, calls_per_dt, us_per_call, alg_bytes, alg_TBps, alg_frac (of 8 TB/s), pmc_bytes,
  pmc_TBps, pmc_frac, pmc_over_alg, ms_per_dt
"""
import csv
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from kernel_access import access_map  # noqa: E402

PEAK = 8.0e12
DYCORE = os.path.join(os.path.dirname(HERE), "mpas-model_amd", "csrc", "dycore.hip")

# Ptrs member -> registry "pool.name" (state fields carry their time level in the member name)
ALIAS = {"u1": "state.u", "u2": "state.u", "w1": "state.w", "w2": "state.w", "w2_rd": "state.w",
         "theta_m1": "state.theta_m", "theta_m2": "state.theta_m", "rho_zz1": "state.rho_zz",
         "rho_zz2": "state.rho_zz", "rho_zz2_rd": "state.rho_zz", "scalars1": "state.scalars",
         "scalars2": "state.scalars", "rw_rd": "diag.rw", "tend_u": "tend.u", "tend_u_euler": "tend.u_euler",
         "tend_w": "tend.w", "tend_w_euler": "tend.w_euler", "tend_theta": "tend.theta_m",
         "tend_theta_euler": "tend.theta_euler", "tend_rho": "tend.rho_zz", "rt_diabatic_tend": "tend.rt_diabatic_tend",
         "scalars_tend": "tend.scalars_tend"}

# What a template variant / launch flag switches off (member names), and the fields of helper
# paths that only other configurations take (regional masks, physics, wide stencils).
NOT_DEFAULT = {"bdyMaskCell", "bdyMaskEdge", "tend_ru_physics", "tend_rtheta_physics", "tend_rho_physics",
               "rt_diabatic_tend", "bnd_pairs", "bnd_edges", "bnd_cells", "edge_bnd", "cell_bnd", "lbc_tmp"}
VARIANT = {
    # rk_step > 1: no PGF / del2 / rk1 filters (4770-4790, 4849-4944)
    "k_dyn_edges_p<false": {"drop": {"cqu", "zxu", "pressure_p", "zz", "dpdz", "divergence", "vorticity", "kdiff",
                                     "meshScalingDel2", "delsq_u", "invDvEdge", "verticesOnEdge"},
                            "drop_w": {"tend_u_euler", "delsq_u"}},
    # rk1 SPLIT: the PGF part goes to k_dyn_edges_pgf_p
    "k_dyn_edges_p<true": {"drop": {"cqu", "zxu", "pressure_p", "zz", "dpdz", "divergence", "vorticity", "kdiff",
                                    "meshScalingDel2", "delsq_u", "invDvEdge", "verticesOnEdge", "tend_u_euler"},
                           "drop_w": {"tend_u_euler", "delsq_u"}},
    "k_dyn_cells3_r<6, false": {"drop": {"delsq_theta", "delsq_w", "dpdz", "pressure_p", "t_init", "zgrid",
                                         "cqw", "meshScalingDel4", "rdzu", "tend_rtheta_physics"},
                                "drop_w": {"tend_theta_euler", "tend_w_euler", "rthdynten", "tend_rtheta_adv"}},
    # rk1 reads tend_w_euler / tend_theta_euler (k_dyn_cells2's del2 terms) and rw_save; not ru_save
    "k_dyn_cells3_r<6, true": {"drop": {"ru_save", "tend_rtheta_physics"},
                               "drop_w": {"rthdynten", "tend_rtheta_adv"}},
    "k_acoustic_cells_r<6, false": {"drop": {"rho_base", "rho_p_save", "rtheta_base", "rtheta_p_save", "exner_base"},
                                    "drop_w": {"exner", "pressure_p", "rho_p", "rho_zz2", "rtheta_p", "rw", "theta_m2",
                                               "w2"}},
    "k_acoustic_cells_r<6, true": {"drop_w": {"rho_pp", "rw_p", "rtheta_pp"}},
    "k_divdamp_p<true": {},
    "k_acoustic_edges_p<true": {},
    "k_diag_edges_p": {"drop_w": {"gradPVn", "gradPVt"}},
}
EXTRA_READS = {  # pointer arguments, not Ptrs members
    "k_diag_vertices": {"state.u"}, "k_diag_cells_b": {"state.u"}, "k_diag_vertices_p": {"state.u"},
    "k_diag_edges_p": {"state.u", "state.rho_zz"}, "k_reconstruct": {"state.u"}, "k_reconstruct_b": {"state.u"},
}


def _calls(body, fn):
    """Argument lists (top-level comma split) of every call fn(...) in body."""
    out = []
    for m in re.finditer(rf"\b{fn}\(", body):
        depth, k, args, cur = 1, m.end(), [], ""
        while depth:
            ch = body[k]
            if ch == "(":
                depth += 1
            elif ch == ")":
                depth -= 1
            if depth == 1 and ch == "," or depth == 0:
                args.append(cur.strip())
                cur = ""
            else:
                cur += ch
            k += 1
        out.append((m.start(), args))
    return out


def registry(nC, K, ME=6, ME2=10, ns=1):
    """pool.name -> (elements incl. the garbage slot, doubles per element), from build_registry."""
    nE, nV = 3 * nC - 6, 2 * nC - 4
    n = {"L_CELL": nC + 1, "L_EDGE": nE + 1, "L_VERTEX": nV + 1, "L_NONE": 1}
    env = {"K": K, "ME": ME, "ME2": ME2, "ns": ns, "CELL_REC": 16}
    src = open(DYCORE).read()
    body = src[src.index("void build_registry"):src.index("Field* find(")]
    out = {}
    loops = [(m.start(), re.findall(r'"(\w+)"', m.group(1)))
             for m in re.finditer(r"for \(const char\* n : \{([^}]*)\}\)", body)]
    for pos, a in _calls(body, "add"):
        if len(a) < 5 or a[0] != "c":
            continue
        pool, name, loc = a[1].strip('"'), a[2], a[3]
        inner = eval(re.sub(r"\(int64_t\)", "", a[4]), {}, env)
        names = [name.strip('"')]
        if name == "n":  # inside the nearest preceding name loop
            names = max((lp for lp in loops if lp[0] < pos), key=lambda lp: lp[0])[1]
        for nm in names:
            out[f"{pool}.{nm}"] = (n[loc], inner)
    return out


def field_key(member, reg):
    if member in ALIAS:
        return ALIAS[member]
    for pool in ("diag", "mesh", "scratch", "tend_physics", "tend", "lbc"):
        if f"{pool}.{member}" in reg:
            return f"{pool}.{member}"
    return None


PER_SCALAR_FIELDS = {"state.scalars", "tend.scalars_tend"}


def alg_bytes(kernel_full, amap, reg, ns=1):
    base = kernel_full.split("<")[0].replace("void ", "").strip()
    if base not in amap:
        return None
    reads, writes = (set(x) for x in amap[base])
    reads -= NOT_DEFAULT
    writes -= NOT_DEFAULT
    for pre, rule in VARIANT.items():
        if kernel_full.replace("void ", "").startswith(pre):
            reads -= rule.get("drop", set())
            writes -= rule.get("drop_w", set())
    # one entry per distinct array: the two time levels of a state field are two arrays, and a
    # *_rd member names the same array as its field
    def arr(m):
        k = field_key(m, reg)
        return (k, m.rstrip("_rd")[-1] if k and k.startswith("state.") else "")
    keys_r = {arr(m) for m in reads} | {(k, "x") for k in EXTRA_READS.get(base, set())}
    keys_w = {arr(m) for m in writes}
    pair = ns > 1 and base.startswith("k_mono_") and base != "k_mono_prep"

    def size(k):
        b = reg[k][0] * reg[k][1] * (4 if k.split(".")[1] in INT_FIELDS else 8)
        if pair and k in PER_SCALAR_FIELDS:
            return b * 2 // ns  # two of the ns scalars
        if pair and k.startswith("scratch."):
            return 2 * b  # the pair's second set of scratch
        return b
    tot = 0
    for k, tag in keys_r:
        if k and k in reg:
            tot += size(k)
    for k, tag in keys_w:
        if k and k in reg:
            tot += size(k)
    return tot


INT_FIELDS = {"nEdgesOnCell", "edgesOnCell", "cellsOnCell", "verticesOnCell", "kiteForCell", "cellsOnEdge",
              "verticesOnEdge", "nEdgesOnEdge", "edgesOnEdge", "nAdvCellsForEdge", "advCellsForEdge",
              "cellsOnVertex", "edgesOnVertex", "cell_rec"}


def main():
    stats, pmc_path, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    nC = int(sys.argv[4]) if len(sys.argv) > 4 else 163842
    K = int(sys.argv[5]) if len(sys.argv) > 5 else 56
    ns = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    reg = registry(nC, K, ns=ns)
    amap = access_map()
    pmc = {}
    if os.path.isfile(pmc_path):
        for r in json.load(open(pmc_path))["kernels"]:
            pmc[r["kernel"].replace("void ", "")] = r["read_bytes"] + r["write_bytes"]
    rows = list(csv.DictReader(open(stats)))
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls_per_dt", "us_per_call", "alg_bytes", "alg_TBps", "alg_frac", "pmc_bytes", "pmc_TBps",
                "pmc_frac", "pmc_over_alg", "ms_per_dt"])
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        name = r["Name"].split("(")[0].replace("mpas::", "").replace("void ", "").strip()
        calls = int(r["Calls"]) / steps
        us = float(r["AverageNs"]) / 1e3
        if name.startswith("__amd") or "init" in name or "build" in name or calls < 0.5:
            continue
        # launches over a halo / boundary remainder (one element on one block) have no whole-array count
        b = alg_bytes(name, amap, reg, ns) if us >= 20.0 else None
        pb = pmc.get(name)
        row = [name, f"{calls:.2f}", f"{us:.1f}"]
        if b:
            row += [f"{b:.4g}", f"{b / (us * 1e-6) / 1e12:.2f}", f"{b / (us * 1e-6) / PEAK:.3f}"]
        else:
            row += ["", "", ""]
        if pb:
            row += [f"{pb:.4g}", f"{pb / (us * 1e-6) / 1e12:.2f}", f"{pb / (us * 1e-6) / PEAK:.3f}",
                    f"{pb / b:.2f}" if b else ""]
        else:
            row += ["", "", "", ""]
        row.append(f"{calls * us / 1e3:.3f}")
        w.writerow(row)


if __name__ == "__main__":
    main()
