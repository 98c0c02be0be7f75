"""TEST INFRASTRUCTURE ONLY -- runs the compiled reference dycore (the oracle).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module.  It writes a synthetic case (built by mpas_dycore.init_atm) in the
raw Fortran layout read by oracle/harness/mpas_ref_harness.F90, runs the
harness binary built from /root/reference by oracle/Makefile, and reads the
dumped pools back as element-major numpy arrays.

Parity is pinned to the reference itself: the binary is the UNMODIFIED
mpas_atm_time_integration.F (atm_srk3 and every *_work routine it calls).
"""
from __future__ import annotations

import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
HARNESS = os.path.join(HERE, "_ref", "mpas_ref_harness")
# the reference dycore built with -DDO_PHYSICS, physics_get_tend replaced by a test double that
# hands over prescribed tendencies (make -C oracle phys; shims/mpas_atmphys_todynamics_stub.F90)
PHYS_HARNESS = os.path.join(HERE, "_ref", "mpas_ref_harness_phys")
# the same harness driver linked against the Fortran drop-in module + libmpas_dycore.so
# (make -C oracle dropin): the product behind the reference's own Fortran API, not an oracle
DROPIN_HARNESS = os.path.join(HERE, "_ref", "mpas_dropin_harness")
# the drop-in built with -DDO_PHYSICS over the same physics test doubles as PHYS_HARNESS
DROPIN_PHYS_HARNESS = os.path.join(HERE, "_ref", "mpas_dropin_harness_phys")

_LOC_N = {"cell": "nCells", "edge": "nEdges", "vertex": "nVertices"}


def _big_stack():
    import resource
    _, hard = resource.getrlimit(resource.RLIMIT_STACK)
    try:
        resource.setrlimit(resource.RLIMIT_STACK, (hard, hard))
    except (ValueError, OSError):
        pass


def available(binary: str = HARNESS) -> bool:
    return os.path.isfile(binary) and os.access(binary, os.X_OK)


def _fields():
    import sys
    pkg = os.path.join(os.path.dirname(HERE), "mpas-model_amd")
    if pkg not in sys.path:
        sys.path.insert(0, pkg)
    from mpas_dycore import fields
    return fields


def to_fortran(case: dict, name: str) -> np.ndarray:
    """Element-major numpy -> Fortran (..., n+1) memory image (shared with the product's upload path)."""
    _fields()
    from mpas_dycore.layout import to_fortran as tf
    return tf(case, name)


def write_physics_inputs(case: dict, d: str, physics: dict):
    """Prescribed physics tendencies in the Fortran images the DO_PHYSICS harness reads:
    element-major tend_ru_physics (nEdges, K), tend_rtheta_physics / tend_rho_physics (nCells, K),
    scalars_tend (nCells, K, ns) -> (K, n+1) / (ns, K, nCells+1) with a zero garbage slot."""
    K, ns = case["nVertLevels"], case["num_scalars"]
    shapes = {"tend_ru_physics": (case["nEdges"], K), "tend_rtheta_physics": (case["nCells"], K),
              "tend_rho_physics": (case["nCells"], K), "scalars_tend": (case["nCells"], K, ns)}
    for n, shp in shapes.items():
        a = np.asarray(physics[n], dtype=np.float64).reshape(shp)
        img = np.zeros((shp[0] + 1,) + shp[1:])
        img[:-1] = a
        img.tofile(os.path.join(d, n + "_in.bin"))


def lbc_images(case: dict, lbc: dict) -> dict:
    """cases.regional_lbc's element-major driving data -> {(name, time level): Fortran image}, time
    level 1 = tendency, 2 = interval-end state (the reference's lbc pool)."""
    out = {}
    for name in ("u", "ru", "rho_zz", "rtheta_m", "scalars"):
        for tl, suf in ((1, "t"), (2, "s")):
            a = np.asarray(lbc[f"lbc_{name}_{suf}"], dtype=np.float64)
            img = np.zeros((a.shape[0] + 1,) + a.shape[1:])
            img[:-1] = a
            out[(f"lbc_{name}", tl)] = img
    return out


def write_lbc_inputs(case: dict, d: str, lbc: dict):
    """The lbc pool as the harness reads it (lbc.lbc_<f>.tl<N>.bin) and the regional namelist switches."""
    for (name, tl), img in lbc_images(case, lbc).items():
        img.tofile(os.path.join(d, f"lbc.{name}.tl{tl}.bin"))
    with open(os.path.join(d, "harness.nml")) as f:
        nml = f.read()
    iv = repr(float(lbc["interval_end"])).replace("e", "d")
    with open(os.path.join(d, "harness.nml"), "w") as f:
        f.write(nml.replace("&harness\n", f"&harness\n config_apply_lbcs_in=.true., lbc_interval_end={iv},\n"))


def write_fields(case: dict, d: str):
    """Every mesh / state / diag array of the case as its Fortran memory image, one .bin per field."""
    F = _fields()
    os.makedirs(d, exist_ok=True)
    names = [n for n in case if n in F.LOCATION or n in F.VERTICAL_1D or n in F.SCALARS_0D]
    for n in names:
        if n in F.SCALARS_0D:
            np.asarray([case[n]], dtype=np.float64).tofile(os.path.join(d, n + ".bin"))
        elif n in F.VERTICAL_1D:
            np.asarray(case[n], dtype=np.float64).tofile(os.path.join(d, n + ".bin"))
        else:
            to_fortran(case, n).tofile(os.path.join(d, n + ".bin"))


def write_inputs(case: dict, d: str, nsteps: int, dt: float, dump_steps=(), nthreads: int = 0,
                 moist_end: int = 1, convection_scheme: str = "off", print_minmax: int = 0,
                 dump_only=(), fields: bool = True, nblocks: int = 1, microp_scheme: str = "off"):
    os.makedirs(d, exist_ok=True)
    if fields:
        write_fields(case, d)
    cfg = case["config"]
    ds = list(dump_steps) + [-1] * (16 - len(dump_steps))

    def fl(x):
        return ".true." if x else ".false."

    nml = f"""&harness
 nCells={case['nCells']}, nEdges={case['nEdges']}, nVertices={case['nVertices']},
 nVertLevels_in={case['nVertLevels']}, maxEdges_in={case['maxEdges']}, maxEdges2_in={case['maxEdges2']},
 num_scalars_in={case['num_scalars']}, nsteps={nsteps}, moist_end={moist_end}, nthreads_req={nthreads},
 dump_steps={','.join(str(x) for x in ds)},
 dt={dt!r}, sphere_radius={case['sphere_radius']!r},
 config_time_integration_order={cfg['config_time_integration_order']},
 config_number_of_sub_steps={cfg['config_number_of_sub_steps']},
 config_dynamics_split_steps={cfg['config_dynamics_split_steps']},
 config_number_rayleigh_damp_u_levels={cfg['config_number_rayleigh_damp_u_levels']},
 config_split_dynamics_transport={fl(cfg['config_split_dynamics_transport'])},
 config_scalar_advection={fl(cfg['config_scalar_advection'])},
 config_positive_definite={fl(cfg['config_positive_definite'])},
 config_monotonic={fl(cfg['config_monotonic'])}, config_mix_full={fl(cfg['config_mix_full'])},
 config_rayleigh_damp_u={fl(cfg['config_rayleigh_damp_u'])},
 config_h_mom_eddy_visc2={cfg['config_h_mom_eddy_visc2']!r}, config_h_mom_eddy_visc4={cfg['config_h_mom_eddy_visc4']!r},
 config_v_mom_eddy_visc2={cfg['config_v_mom_eddy_visc2']!r},
 config_h_theta_eddy_visc2={cfg['config_h_theta_eddy_visc2']!r}, config_h_theta_eddy_visc4={cfg['config_h_theta_eddy_visc4']!r},
 config_v_theta_eddy_visc2={cfg['config_v_theta_eddy_visc2']!r},
 config_len_disp={cfg['config_len_disp']!r}, config_visc4_2dsmag={cfg['config_visc4_2dsmag']!r},
 config_del4u_div_factor={cfg['config_del4u_div_factor']!r}, config_coef_3rd_order={cfg['config_coef_3rd_order']!r},
 config_smagorinsky_coef={cfg['config_smagorinsky_coef']!r}, config_epssm={cfg['config_epssm']!r},
 config_smdiv={cfg['config_smdiv']!r}, config_apvm_upwinding={cfg['config_apvm_upwinding']!r},
 config_mpas_cam_coef={cfg['config_mpas_cam_coef']!r},
 config_rayleigh_damp_u_timescale_days={cfg['config_rayleigh_damp_u_timescale_days']!r},
 config_horiz_mixing='{cfg['config_horiz_mixing']}', config_convection_scheme='{convection_scheme}',
 config_microp_scheme='{microp_scheme}'
/
"""
    if print_minmax:
        nml = nml.replace("&harness\n", f"&harness\n print_minmax={print_minmax},\n")
    if dump_only:
        nml = nml.replace("&harness\n", f"&harness\n dump_only='{','.join(dump_only)}',\n")
    if nblocks > 1:
        nml = nml.replace("&harness\n", f"&harness\n nblocks={nblocks},\n")
    nml = nml.replace("e+", "d+").replace("e-", "d-")
    with open(os.path.join(d, "harness.nml"), "w") as f:
        f.write(nml)


# Fortran shapes of dumped real fields, (leading dims..., location) -> element-major reshape
def read_dump(case: dict, stepdir: str) -> dict:
    """Read every pool.field[.tlN].bin of a dump directory into element-major arrays
    (garbage slot dropped).  Keys are 'pool.name' or 'pool.name.tlN'."""
    K, ns = case["nVertLevels"], case["num_scalars"]
    nC, nE, nV = case["nCells"], case["nEdges"], case["nVertices"]
    out = {}
    text = {}
    for fn in sorted(os.listdir(stepdir)):
        if fn.endswith(".txt"):  # character fields (state.xtime.tlN)
            with open(os.path.join(stepdir, fn)) as f:
                text[fn[:-4]] = f.read().strip()
            continue
        if not fn.endswith(".bin"):
            continue
        key = fn[:-4]
        a = np.fromfile(os.path.join(stepdir, fn), dtype=np.float64)
        out[key] = a
    # reshape the hot-path prognostic/diagnostic fields by size
    shaped = {}
    for key, a in out.items():
        n = a.size
        for (rows, cols) in ((nC + 1, K), (nC + 1, K + 1), (nE + 1, K), (nV + 1, K), (nC + 1, K * ns)):
            if n == rows * cols:
                b = a.reshape(rows, cols)[:-1]
                if cols == K * ns and ns > 1 and "scalars" in key:
                    b = b.reshape(rows - 1, K, ns)
                shaped[key] = b
                break
        else:
            shaped[key] = a
    shaped.update(text)
    return shaped


def run_reference(case: dict, nsteps: int, dt: float, dump_steps=None, nthreads: int = 0,
                  workdir: str | None = None, moist_end: int = 1, timeout: int = 3000, binary: str = HARNESS,
                  physics: dict | None = None, print_minmax: int = 0, dump_only=(), env_extra: dict | None = None,
                  with_total: bool = False, lbc: dict | None = None):
    """Run the reference dycore; returns ({step: {field: array}}, [step wall times]) -- and, with
    ``lbc`` (cases.regional_lbc's driving data) runs with config_apply_lbcs, the lbc pool and masks.
    ``with_total``, the wall time of the whole time loop including its final wait for the device
    ({"total": s, "after2": s of steps 3.. } when the run has more than 2 steps).
    ``binary=DROPIN_HARNESS`` runs the same driver on the drop-in module instead.
    ``physics`` (dict of write_physics_inputs' arrays, optional keys "convection_scheme" and
    "microp_scheme" -- "mp_test_double" selects the microphysics test double of
    shims/mpas_atmphys_driver_microphysics_stub.F90) runs the DO_PHYSICS build with those tendencies
    handed over by physics_get_tend every step.
    ``dump_only`` (e.g. ["state.u", "state.w"]) limits the dumps to those fields (full-size runs).
    ``print_minmax`` turns on summarize_timestep's namelist switches (1 global_minmax_vel,
    2 detailed_minmax_vel, 4 global_minmax_sca); the reference's log text is then res["log"]."""
    if physics is not None and binary == HARNESS:
        binary = PHYS_HARNESS
    if not available(binary):
        raise RuntimeError(f"{binary} not built (make -C oracle)")
    if dump_steps is None:
        dump_steps = [nsteps]
    own = workdir is None
    tmp = tempfile.mkdtemp(prefix="mpasref_") if own else workdir
    ind, outd = os.path.join(tmp, "in"), os.path.join(tmp, "out")
    write_inputs(case, ind, nsteps, dt, dump_steps, nthreads, moist_end,
                 (physics or {}).get("convection_scheme", "off"), print_minmax, dump_only,
                 microp_scheme=(physics or {}).get("microp_scheme", "off"))
    if physics is not None:
        write_physics_inputs(case, ind, physics)
    if lbc is not None:
        write_lbc_inputs(case, ind, lbc)
    env = dict(os.environ)
    if nthreads:
        env["OMP_NUM_THREADS"] = str(nthreads)
    env.update(env_extra or {})
    # the reference's automatic arrays (nCells-sized locals in the *_work routines) live on the
    # stack: large meshes need the main thread's stack unlimited and big OpenMP thread stacks
    env.setdefault("OMP_STACKSIZE", "1G")
    r = subprocess.run([binary, ind, outd], cwd=tmp, env=env, capture_output=True, text=True, timeout=timeout,
                       preexec_fn=_big_stack)
    if r.returncode != 0:
        raise RuntimeError(f"{os.path.basename(binary)} failed ({r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
    res = {}
    for s in dump_steps:
        sd = os.path.join(outd, f"step_{s:04d}")
        res[s] = read_dump(case, sd)
    if print_minmax:
        logs = sorted(fn for fn in os.listdir(tmp) if fn.startswith("log.") and fn.endswith(".out"))
        res["log"] = "".join(open(os.path.join(tmp, fn)).read() for fn in logs)
    times, total = [], None
    with open(os.path.join(outd, "timing.txt")) as f:
        for line in f:
            if line.startswith("step"):
                times.append(float(line.split()[2]))
            elif line.startswith("total"):
                total = float(line.split()[1])
            elif line.startswith("after2"):   # steps 3.. (both time-level parities warm), device wait included
                total = {"total": total, "after2": float(line.split()[1])}
    if own:
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)
    return (res, times, total) if with_total else (res, times)


# mode 'init': the reference's mesh-dependent precompute (mpas_atm_advection.F deriv_two / defc_a /
# defc_b; mpas_atm_core.F:927-1288 signs, adv_coef compression, 3rd-order coupling, mesh scaling,
# damping coefficients).  Outputs: name -> (location, Fortran leading dims, is_int).
INIT_OUTPUTS = {
    "deriv_two": ("edge", (15, 2), False), "defc_a": ("cell", ("ME",), False), "defc_b": ("cell", ("ME",), False),
    "edgesOnCell_sign": ("cell", ("ME",), False), "edgesOnVertex_sign": ("vertex", (3,), False),
    "kiteForCell": ("cell", ("ME",), True), "zb_cell": ("cell", ("K1", "ME"), False),
    "zb3_cell": ("cell", ("K1", "ME"), False), "adv_coefs": ("edge", (15,), False),
    "adv_coefs_3rd": ("edge", (15,), False), "advCellsForEdge": ("edge", (15,), True),
    "nAdvCellsForEdge": ("edge", (), True), "meshScalingDel2": ("edge", (), False),
    "meshScalingDel4": ("edge", (), False), "dss": ("cell", ("K",), False), "advCells": ("cell", (21,), True),
}


def run_reference_init(case: dict, nthreads: int = 1, timeout: int = 600) -> dict:
    """Run the reference's model-init precompute on the case's mesh (harness mode 'init') and return
    its outputs as element-major arrays (index arrays 0-based, a missing entry -1).  The inputs are
    the mesh geometry and connectivity, zgrid, meshDensity, zb / zb3; every output above is
    withheld from the harness, so it starts from zeros as the reference does."""
    import shutil
    tmp = tempfile.mkdtemp(prefix="mpasrefi_")
    try:
        ind, outd = os.path.join(tmp, "in"), os.path.join(tmp, "out")
        write_inputs({k: v for k, v in case.items() if k not in INIT_OUTPUTS}, ind, 0, 1.0, [], nthreads)
        with open(os.path.join(ind, "harness.nml")) as f:
            nml = f.read()
        with open(os.path.join(ind, "harness.nml"), "w") as f:
            f.write(nml.replace("&harness\n", "&harness\n mode='init',\n"))
        env = dict(os.environ, OMP_NUM_THREADS=str(nthreads))
        r = subprocess.run([HARNESS, ind, outd], cwd=tmp, env=env, capture_output=True, text=True, timeout=timeout,
                           preexec_fn=_big_stack)
        if r.returncode != 0:
            raise RuntimeError(f"reference init run failed ({r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
        dims = {"ME": case["maxEdges"], "K": case["nVertLevels"], "K1": case["nVertLevels"] + 1}
        out = {}
        for name, (loc, lead, is_int) in INIT_OUTPUTS.items():
            a = np.fromfile(os.path.join(outd, "step_0000", f"mesh.{name}.bin"), dtype=np.int32 if is_int else np.float64)
            inner = tuple(dims.get(x, x) for x in lead)
            a = a.reshape((case[_LOC_N[loc]] + 1,) + inner[::-1])[:-1]
            out[name] = a.astype(np.int64) - 1 if is_int and name != "nAdvCellsForEdge" else a
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


# mode 'jw': the reference's JW initial state (core_init_atmosphere init_atm_case_jw, :367-1312) on
# the case's mesh.  The reference scales a unit-sphere grid (:474-489), so lengths go in divided by
# the sphere radius and areas by its square.  Outputs: everything the routine computes.
JW_OUTPUTS = ("u", "w", "theta", "rho", "rho_base", "theta_base", "scalars", "zgrid", "zz", "zxu", "rdzw", "rdzu",
              "fzm", "fzp", "cf1", "cf2", "cf3", "zb", "zb3", "deriv_two", "defc_a", "defc_b", "fEdge", "fVertex",
              "dss")
_UNIT_LENGTH = ("xCell", "yCell", "zCell", "xEdge", "yEdge", "zEdge", "xVertex", "yVertex", "zVertex", "dvEdge",
                "dcEdge")
_UNIT_AREA = ("areaCell", "areaTriangle", "kiteAreasOnVertex")


def unit_sphere(mesh: dict) -> tuple[dict, dict]:
    """(unit-sphere grid, the same grid scaled as init_atm_case_jw scales it, :474-489): lengths
    divided by the sphere radius and multiplied back, areas by its square (R**2 is exact for an
    integral radius).  Our restatement run on the scaled fields and the reference run on the unit
    ones then see the same geometry bit for bit."""
    R = float(mesh["sphere_radius"])
    unit = {k: np.asarray(mesh[k], dtype=np.float64) / R for k in _UNIT_LENGTH}
    unit.update({k: np.asarray(mesh[k], dtype=np.float64) / (R * R) for k in _UNIT_AREA})
    scaled = {k: unit[k] * R for k in _UNIT_LENGTH}
    scaled.update({k: unit[k] * (R * R) for k in _UNIT_AREA})
    return unit, scaled


def run_reference_jw(case: dict, unit: dict | None = None, nthreads: int = 1, timeout: int = 600) -> dict:
    """Run init_atm_case_jw (harness mode 'jw') on the case's mesh, given on the unit sphere
    (``unit``, from unit_sphere(); default: the case's lengths / R and areas / R**2); returns its
    dumps keyed 'pool.name' (state fields as 'state.<name>.tlN'), element-major where the shape is
    known, else the flat Fortran image."""
    import shutil
    R = float(case["sphere_radius"])
    inp = {k: v for k, v in case.items() if k not in JW_OUTPUTS}
    if unit is None:
        unit = unit_sphere(case)[0]
    inp.update(unit)
    for k in ("u", "w", "theta", "rho", "rho_base", "theta_base", "scalars"):  # zero inputs of the shapes
        inp[k] = np.zeros_like(np.asarray(case[k], dtype=np.float64))
    tmp = tempfile.mkdtemp(prefix="mpasjw_")
    try:
        ind, outd = os.path.join(tmp, "in"), os.path.join(tmp, "out")
        write_inputs(inp, ind, 0, 1.0, [], nthreads)
        with open(os.path.join(ind, "harness.nml")) as f:
            nml = f.read()
        with open(os.path.join(ind, "harness.nml"), "w") as f:
            f.write(nml.replace("&harness\n", "&harness\n mode='jw',\n"))
        env = dict(os.environ, OMP_NUM_THREADS=str(nthreads))
        r = subprocess.run([HARNESS, ind, outd], cwd=tmp, env=env, capture_output=True, text=True, timeout=timeout,
                           preexec_fn=_big_stack)
        if r.returncode != 0:
            raise RuntimeError(f"reference JW init failed ({r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
        out = read_dump(case, os.path.join(outd, "step_0000"))
        K, nE = case["nVertLevels"], case["nEdges"]
        for name, shape in (("mesh.zb", (nE + 1, 2, K + 1)), ("mesh.zb3", (nE + 1, 2, K + 1)),
                            ("mesh.deriv_two", (nE + 1, 2, 15))):
            out[name] = np.asarray(out[name]).reshape(shape)[:-1]
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def write_block_inputs(blocks: list, d: str):
    """The blocks of one process (mpas_dycore.decomp) for the harness's multi-block mode: per block
    <d>/block<i>/ with its fields, block.nml (dims, owned counts) and its local-copy exchange lists
    copy_<loc>_<layer>_<j>.bin (1-based srcList here, then destList in block j, MPAS exchList order)."""
    local = {b.part: i for i, b in enumerate(blocks)}
    for i, b in enumerate(blocks):
        bd = os.path.join(d, f"block{i}")
        write_fields(b.case, bd)
        nc, ne, nv = b.solve
        with open(os.path.join(bd, "block.nml"), "w") as f:
            f.write(f"&block\n nCells={b.case['nCells']}, nEdges={b.case['nEdges']}, nVertices={b.case['nVertices']},\n"
                    f" nCellsSolve_in={nc}, nEdgesSolve_in={ne}, nVerticesSolve_in={nv}\n/\n")
        for loc, layer, peer, idx in b.send:
            pb = blocks[local[peer]]
            dst = [x for (l2, y2, q2, x) in pb.recv if l2 == loc and y2 == layer and q2 == b.part]
            if len(dst) != 1 or len(dst[0]) != len(idx):
                raise ValueError(f"block {b.part} -> {peer} {loc} layer {layer}: send/recv lists disagree")
            lists = np.concatenate([np.asarray(idx, np.int32) + 1, np.asarray(dst[0], np.int32) + 1])
            lists.astype(np.int32).tofile(os.path.join(bd, f"copy_{loc}_{layer}_{local[peer]}.bin"))


def run_reference_blocks(case: dict, blocks: list, nsteps: int, dt: float, dump_steps=None, nthreads: int = 0,
                         moist_end: int = 1, timeout: int = 3000, dump_only=(), binary: str = HARNESS,
                         env_extra: dict | None = None):
    """The reference dycore on several blocks in one process (mpas_dmpar local copies between them):
    returns ({step: [per-block {field: array}]}, [step wall times]).  ``binary=DROPIN_HARNESS``
    runs the same driver on the drop-in module (its domain context then holds every block)."""
    import shutil
    if not available(binary):
        raise RuntimeError(f"{binary} not built (make -C oracle)")
    dump_steps = [nsteps] if dump_steps is None else dump_steps
    tmp = tempfile.mkdtemp(prefix="mpasrefb_")
    try:
        ind, outd = os.path.join(tmp, "in"), os.path.join(tmp, "out")
        write_inputs(case, ind, nsteps, dt, dump_steps, nthreads, moist_end, dump_only=dump_only, fields=False,
                     nblocks=len(blocks))
        write_block_inputs(blocks, ind)
        env = dict(os.environ)
        if nthreads:
            env["OMP_NUM_THREADS"] = str(nthreads)
        env.setdefault("OMP_STACKSIZE", "1G")
        env.update(env_extra or {})
        r = subprocess.run([binary, ind, outd], cwd=tmp, env=env, capture_output=True, text=True, timeout=timeout,
                           preexec_fn=_big_stack)
        if r.returncode != 0:
            raise RuntimeError(f"multi-block reference failed ({r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
        res = {s: [read_dump(b.case, os.path.join(outd, f"step_{s:04d}", f"block{i}")) for i, b in enumerate(blocks)]
               for s in dump_steps}
        times = []
        with open(os.path.join(outd, "timing.txt")) as f:
            for line in f:
                if line.startswith("step"):
                    times.append(float(line.split()[2]))
        return res, times
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def run_reference_kernel(case: dict, restore_dir: str, mode: str, dts: float = 0.0, small_step: int = 2,
                         rk_step: int = 1, nthreads: int = 1, timeout: int = 600) -> dict:
    """Run one reference routine ('acoustic' = atm_advance_acoustic_step + atm_divergence_damping_3d)
    on a state restored from a previous dump directory; returns the dumped pools."""
    import shutil
    tmp = tempfile.mkdtemp(prefix="mpasrefk_")
    try:
        ind, outd = os.path.join(tmp, "in"), os.path.join(tmp, "out")
        write_inputs(case, ind, 0, 1.0, [], nthreads)
        for fn in os.listdir(restore_dir):
            if fn.endswith(".bin"):
                shutil.copy(os.path.join(restore_dir, fn), os.path.join(ind, fn))
        with open(os.path.join(ind, "harness.nml")) as f:
            nml = f.read()
        extra = f" mode='{mode}', kernel_small_step={small_step}, kernel_rk_step={rk_step}, kernel_dts={dts!r},\n"
        nml = nml.replace("&harness\n", "&harness\n" + extra.replace("e+", "d+").replace("e-", "d-"))
        with open(os.path.join(ind, "harness.nml"), "w") as f:
            f.write(nml)
        env = dict(os.environ, OMP_NUM_THREADS=str(nthreads))
        r = subprocess.run([HARNESS, ind, outd], cwd=tmp, env=env, capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0:
            raise RuntimeError(f"reference kernel run failed ({r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
        return read_dump(case, os.path.join(outd, "step_0000"))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


# ---- the reference's domain decomposition (harness/decomp_harness.F90, make -C oracle decomp) ----
DECOMP_HARNESS = os.path.join(HERE, "_ref", "decomp_harness")
MPIRUN = "/opt/conda/bin/mpirun"


def _nml(v):
    if isinstance(v, bool):
        return ".true." if v else ".false."
    if isinstance(v, float):
        return repr(v).replace("e", "d") if "e" in repr(v) else repr(v) + "d0"
    return str(v)


def run_reference_decomp(case: dict, part, nprocs: int = 1, timeout: int = 600, binary: str = DECOMP_HARNESS,
                         plan: dict | None = None) -> dict:
    """mpas_block_decomp.F + mpas_block_creator.F on the case's mesh and cell partition ``part``
    (0-based block per cell, written as graph.info.part.N).  With ``nprocs`` > 1 the harness runs
    under mpirun, one task per block.  Returns {block id: {"<loc>_index": global 0-based ids in
    local order, "<loc>_solve": end of owned and of each halo layer, "<loc>_<kind>_<layer>": list of
    (endPointID, srcList, destList) with MPAS's 1-based local indices / buffer positions}}."""
    import shutil
    part = np.asarray(part, dtype=np.int64)
    nblocks = int(part.max()) + 1
    tmp = tempfile.mkdtemp(prefix="mpasdec_")
    try:
        ind, outd = os.path.join(tmp, "in"), os.path.join(tmp, "out")
        os.makedirs(ind)
        for name in ("nEdgesOnCell", "cellsOnCell", "edgesOnCell", "verticesOnCell", "cellsOnEdge", "cellsOnVertex"):
            a = np.asarray(case[name], dtype=np.int64)
            (a + (0 if name == "nEdgesOnCell" else 1)).astype(np.int32).tofile(os.path.join(ind, f"{name}.bin"))
        with open(os.path.join(ind, f"graph.info.part.{nblocks}"), "w") as f:
            f.write("\n".join(str(int(x)) for x in part) + "\n")
        with open(os.path.join(ind, "decomp.nml"), "w") as f:
            f.write(f"&decomp\n nCells={case['nCells']}, nEdges={case['nEdges']}, nVertices={case['nVertices']},\n"
                    f" maxEdges={case['maxEdges']}, nblocks={nblocks}, nHalos=2\n/\n")
            if plan is not None:
                f.write("&plan\n" + ",\n".join(f" {k}={_nml(v)}" for k, v in plan.items()) + "\n/\n")
        cmd = [binary, ind, outd]
        if nprocs > 1:
            cmd = [MPIRUN, "-np", str(nprocs)] + cmd
        r = subprocess.run(cmd, cwd=tmp, capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0:
            raise RuntimeError(f"decomp_harness failed ({r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
        out = {}
        for bdir in sorted(os.listdir(outd)):
            if bdir.startswith("plan_task"):  # dropin_plan_harness: the drop-in's plan of each task
                out.setdefault("plans", {})[int(bdir[len("plan_task"):-4])] = _read_plan(os.path.join(outd, bdir))
                continue
            b = int(bdir[len("block"):])
            res = {}
            for fn in sorted(os.listdir(os.path.join(outd, bdir))):
                a = np.fromfile(os.path.join(outd, bdir, fn), dtype=np.int32)
                key = fn[:-4]
                if key.endswith("_index"):
                    res[key] = a.astype(np.int64) - 1
                elif key.endswith("_solve"):
                    res[key] = a.astype(np.int64)
                else:
                    nodes, i = [], 0
                    while i < a.size:
                        ep, n = int(a[i]), int(a[i + 1])
                        nodes.append((ep, a[i + 2:i + 2 + n].astype(np.int64), a[i + 2 + n:i + 2 + 2 * n].astype(np.int64)))
                        i += 2 + 2 * n
                    res[key] = nodes
            out[b] = res
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


# ---- the Fortran drop-in's multi-task plan (harness/decomp_harness.F90 -DDROPIN_PLAN, make -C oracle dropin_plan) ----
DROPIN_PLAN_HARNESS = os.path.join(HERE, "_ref", "dropin_plan_harness")


def _read_plan(path):
    """A plan file of atm_dycore_plan_exchanges: (id checksum, messages as tuples (point, direction,
    block, peer_rank, peer_block, count), plan keys)."""
    ident, msgs, keys = None, [], []
    with open(path) as f:
        for line in f:
            tag, _, rest = line.rstrip("\n").partition(" ")
            if tag == "id":
                ident = int(rest)
            elif tag == "msg":
                msgs.append(tuple(int(x) for x in rest.split()))
            elif tag == "key":
                keys.append(rest.strip())
    return ident, msgs, keys


def run_dropin_plan(case: dict, part, nprocs: int, plan: dict, timeout: int = 600) -> dict:
    """The drop-in's domain-context path on `nprocs` MPI tasks without a GPU: the reference's
    decomposition of `part` (as run_reference_decomp), each task's blocks handed to
    atm_dycore_plan_exchanges.  Returns run_reference_decomp's dict plus "plans": {task: (id
    checksum, messages, keys)}."""
    cmd_binary = DROPIN_PLAN_HARNESS
    return run_reference_decomp(case, part, nprocs=nprocs, timeout=timeout, binary=cmd_binary, plan=plan)
