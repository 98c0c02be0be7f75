#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE dycore.

Runs the unmodified reference atm_srk3 (oracle/_ref/mpas_ref_harness, built from
/root/reference by oracle/Makefile) on deterministic synthetic cases and stores
inputs/outputs as compressed npz (data only -- no reference source).

  tests/golden/acoustic_x1.162_K16.npz
      one atm_advance_acoustic_step + atm_divergence_damping_3d (small_step=2) on a
      mid-run state: every input the kernel reads (pre_*) and every field it updates
      (post_*), plus the mesh arrays it needs (0-based indices).
  tests/golden/srk3_x1.642_K26_ns3.npz
      moist JW + two tracer blobs (num_scalars=3): reference prognostics after 1 and
      10 atm_timestep calls (u, w, theta_m, rho_zz, scalars) and an input checksum.

  tests/golden/reconstruct_x1.642.npz
      mpas_rbf_interp_initialize + mpas_init_reconstruct outputs (edgeNormalVectors,
      cellTangentPlane, coeffs_reconstruct) on x1.642.
  tests/golden/init_x1.642_K8.npz, tests/golden/init_varres2562_K8.npz
      the reference's mesh-dependent precompute (harness mode 'init': deriv_two, defc_a/b from
      core_init_atmosphere/mpas_atm_advection.F; signs, kiteForCell, adv_coefs compression,
      3rd-order coupling, mesh scaling, dss from mpas_atm_core.F:927-1288) on the quasi-uniform
      and the variable-resolution test meshes, with a checksum of the mesh it ran on.
  tests/golden/jw_x1.642_K26.npz
      the reference's init_atm_case_jw (core_init_atmosphere/mpas_init_atm_cases.F:367-1312, harness
      mode 'jw') on x1.642 given on the unit sphere: vertical grid, metrics, the dry JW state with
      the rebalanced wind, zb / zb3, deriv_two; with a checksum of the grid it ran on.

Usage: python tools/make_golden.py [acoustic|srk3|reconstruct|init|jw ...]   (needs oracle/_ref built)
"""
from __future__ import annotations

import hashlib
import os
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpas-model_amd"))
sys.path.insert(0, ROOT)

from mpas_dycore.cases import jw_case  # noqa: E402
from oracle import ref_runner  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")

ACOUSTIC_PRE = ["diag.ru_p", "diag.ruAvg", "diag.rho_pp", "diag.rtheta_pp", "diag.rtheta_pp_old", "diag.rw_p",
                "diag.wwAvg", "state.theta_m.tl1", "state.rho_zz.tl2", "state.w.tl2", "diag.exner", "diag.cqu",
                "diag.cofwr", "diag.cofwz", "diag.cofwt", "diag.coftz", "diag.cofrz", "diag.a_tri", "diag.alpha_tri",
                "diag.gamma_tri", "tend.u", "tend.rho_zz", "tend.theta_m", "tend.w", "diag.rw", "diag.rw_save"]
ACOUSTIC_POST = ["diag.ru_p", "diag.ruAvg", "diag.rho_pp", "diag.rtheta_pp", "diag.rtheta_pp_old", "diag.rw_p",
                 "diag.wwAvg"]
ACOUSTIC_MESH = ["zz", "zxu", "dss", "fzm", "fzp", "rdzw", "cellsOnEdge", "edgesOnCell", "nEdgesOnCell",
                 "edgesOnCell_sign", "invDcEdge", "dvEdge", "invAreaCell"]
STATE = ["state.u.tl1", "state.w.tl1", "state.theta_m.tl1", "state.rho_zz.tl1", "state.scalars.tl1"]


def case_checksum(case: dict) -> str:
    h = hashlib.sha256()
    for k in sorted(case):
        v = case[k]
        if isinstance(v, np.ndarray):
            h.update(k.encode())
            h.update(np.ascontiguousarray(v).tobytes())
    return h.hexdigest()


def acoustic_fixture():
    case = jw_case(162, K=16, ns=1, cache=False)
    wd = "/tmp/golden_acoustic"
    shutil.rmtree(wd, ignore_errors=True)
    res, _ = ref_runner.run_reference(case, nsteps=2, dt=case["dt"], dump_steps=[2], nthreads=1, workdir=wd)
    pre = res[2]
    dts = case["dt"] / case["config"]["config_dynamics_split_steps"] / case["config"]["config_number_of_sub_steps"]
    post = ref_runner.run_reference_kernel(case, os.path.join(wd, "out", "step_0002"), "acoustic", dts=dts,
                                           small_step=2, nthreads=1)
    out = dict(nCells=case["nCells"], nEdges=case["nEdges"], K=case["nVertLevels"], maxEdges=case["maxEdges"],
               dts=dts, small_step=2, epssm=case["config"]["config_epssm"], smdiv=case["config"]["config_smdiv"],
               len_disp=case["config"]["config_len_disp"])
    for k in ACOUSTIC_PRE:
        out["pre_" + k] = pre[k]
    for k in ACOUSTIC_POST:
        out["post_" + k] = post[k]
    for k in ACOUSTIC_MESH:
        out["mesh_" + k] = np.asarray(case[k])
    os.makedirs(GOLD, exist_ok=True)
    np.savez_compressed(os.path.join(GOLD, "acoustic_x1.162_K16.npz"), **out)
    shutil.rmtree(wd, ignore_errors=True)


def srk3_fixture():
    case = jw_case(642, K=26, ns=3, moist=True, cache=False)
    res, _ = ref_runner.run_reference(case, nsteps=10, dt=case["dt"], dump_steps=[1, 10], nthreads=4)
    out = dict(checksum=case_checksum(case), dt=case["dt"])
    for s in (1, 10):
        for k in STATE:
            out[f"step{s}_{k}"] = res[s][k]
    np.savez_compressed(os.path.join(GOLD, "srk3_x1.642_K26_ns3.npz"), **out)


JW_EXACT = ("mesh.zgrid", "mesh.zz", "mesh.zxu", "mesh.rdzw", "mesh.rdzu", "mesh.fzm", "mesh.fzp", "mesh.cf1",
            "mesh.cf2", "mesh.cf3", "diag.theta", "diag.rho", "diag.rho_base", "diag.theta_base")
JW_CLOSE = ("state.u.tl1", "state.w.tl1", "mesh.zb", "mesh.zb3", "mesh.deriv_two", "mesh.fEdge", "mesh.fVertex")


def jw_inputs(level: int = 3, K: int = 26):
    """The JW pin's mesh: the x1.N grid on the unit sphere (what the reference reads) and scaled as
    init_atm_case_jw scales it (what init_atm reads)."""
    from mpas_dycore.cases import _mesh
    m = _mesh(level, 20)
    unit, scaled = ref_runner.unit_sphere(m)
    return m, unit, scaled


def jw_fixture():
    """init_atm_case_jw of the reference (harness mode 'jw') on x1.642, K = 26: the vertical grid and
    metrics, the dry JW state with the rebalanced wind, zb / zb3 and deriv_two."""
    from mpas_dycore.init_atm import build_case
    m, unit, scaled = jw_inputs()
    case = build_case({**m, **scaled}, K=26, ns=1)
    ref = ref_runner.run_reference_jw(case, unit)
    out = {"checksum": case_checksum({**{k: v for k, v in m.items() if isinstance(v, np.ndarray)}, **unit})}
    for k in JW_EXACT + JW_CLOSE:
        out[k] = np.asarray(ref[k])
    np.savez_compressed(os.path.join(GOLD, "jw_x1.642_K26.npz"), **out)


def reconstruct_fixture():
    """mpas_rbf_interp_initialize + mpas_init_reconstruct outputs of the reference on x1.642."""
    case = jw_case(642, K=8, ns=1, cache=False)
    res, _ = ref_runner.run_reference(case, nsteps=1, dt=case["dt"], dump_steps=[0], nthreads=2)
    r0 = res[0]
    nC, nE, ME = case["nCells"], case["nEdges"], case["maxEdges"]
    np.savez_compressed(os.path.join(GOLD, "reconstruct_x1.642.npz"),
                        checksum=case_checksum(case),
                        coeffs_reconstruct=r0["mesh.coeffs_reconstruct"].reshape(nC + 1, ME, 3)[:-1],
                        edgeNormalVectors=r0["mesh.edgeNormalVectors"].reshape(nE + 1, 3)[:-1],
                        cellTangentPlane=r0["mesh.cellTangentPlane"].reshape(nC + 1, 2, 3)[:-1])


INIT_CASES = {
    "init_x1.642_K8.npz": lambda: jw_case(642, K=8, ns=1, cache=False),
    "init_varres2562_K8.npz": lambda: __import__("mpas_dycore.cases", fromlist=["varres_case"]).varres_case(
        2562, ratio=4.0, K=8, ns=1, lloyd_iters=30, cache=False),
}
# the model-init outputs' inputs: the mesh the routines read (their checksum pins the fixture's mesh)
INIT_INPUTS = ["xCell", "yCell", "zCell", "xVertex", "yVertex", "zVertex", "cellsOnCell", "edgesOnCell",
               "verticesOnCell", "cellsOnEdge", "verticesOnEdge", "cellsOnVertex", "edgesOnVertex", "nEdgesOnCell",
               "dcEdge", "dvEdge", "meshDensity", "zgrid", "zb", "zb3"]


def init_inputs_checksum(case: dict) -> str:
    return case_checksum({k: np.asarray(case[k]) for k in INIT_INPUTS})


def init_fixture():
    for fn, make in INIT_CASES.items():
        case = make()
        ref = ref_runner.run_reference_init(case)
        out = {"checksum": init_inputs_checksum(case)}
        for k, v in ref.items():
            if k not in ("zb_cell", "zb3_cell"):  # copies of zb / zb3, checked live (and large)
                out[k] = v
        np.savez_compressed(os.path.join(GOLD, fn), **out)


if __name__ == "__main__":
    if not ref_runner.available():
        sys.exit("build the oracle first: make -C oracle")
    only = sys.argv[1:]
    if not only or "acoustic" in only:
        acoustic_fixture()
    if not only or "srk3" in only:
        srk3_fixture()
    if not only or "reconstruct" in only:
        reconstruct_fixture()
    if not only or "init" in only:
        init_fixture()
    if not only or "jw" in only:
        jw_fixture()
    for f in sorted(os.listdir(GOLD)):
        print(f, os.path.getsize(os.path.join(GOLD, f)))
