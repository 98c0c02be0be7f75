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
# what atm_mpas_init_block precomputes (mpas_atm_core.F:311-358, 927-1288; mpas_dyc_model_init) and what
# it reads beyond the dycore's own mesh fields
MODEL_INIT_OUT = ("invAreaCell", "invDvEdge", "invDcEdge", "invAreaTriangle", "edgesOnVertex_sign",
                  "edgesOnCell_sign", "zb_cell", "zb3_cell", "kiteForCell", "nAdvCellsForEdge", "advCellsForEdge",
                  "adv_coefs", "adv_coefs_3rd", "meshScalingDel2", "meshScalingDel4", "meshScalingRegionalCell",
                  "meshScalingRegionalEdge", "dss")
MODEL_INIT_IN = ("deriv_two", "zb", "zb3", "meshDensity", "areaCell", "areaTriangle")
# and mpas_rbf_interp_initialize + mpas_init_reconstruct (mpas_atm_core.F:408-409; mpas_dyc_init_reconstruct)
RECONSTRUCT_IN = ("xCell", "yCell", "zCell", "xEdge", "yEdge", "zEdge")
DIAG_INPUTS = ("theta", "rho", "rho_base", "theta_base")
_SKIP = set(STATE_INPUTS) | set(DIAG_INPUTS) | {"xCell", "yCell", "zCell", "xEdge", "yEdge", "zEdge", "xVertex",
                                                "yVertex", "zVertex",
                                                "latVertex", "lonVertex", "areaCell", "areaTriangle",
                                                "meshDensity", "indexToCellID", "deriv_two", "zb", "zb3"}


def _host_allgather_fn(group, nranks: int):
    """mpas_dyc_comm_init_host's all-gather over a torch.distributed group: every rank's bytes, in rank
    order (CPU tensors, so gloo carries them)."""
    import torch
    import torch.distributed as dist

    def fn(send, recv, nbytes, user):
        try:
            mine = torch.frombuffer(bytearray(C.string_at(send, nbytes)), dtype=torch.uint8) if nbytes else \
                torch.zeros(0, dtype=torch.uint8)
            outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(nranks)]
            dist.all_gather(outs, mine, group=group)
            buf = b"".join(bytes(o.numpy().tobytes()) for o in outs)
            C.memmove(recv, buf, len(buf))
            return 0
        except Exception:  # noqa: BLE001 -- reported to the library as a failed all-gather
            return 1

    return _lib.ALLGATHER_FN(fn)


class DycoreError(RuntimeError):
    pass


def _make_dims(cases, solves, moist_end):
    dims = (_lib.Dims * len(cases))()
    for d, c, sv in zip(dims, cases, solves):
        d.nCells, d.nEdges, d.nVertices = c["nCells"], c["nEdges"], c["nVertices"]
        d.nVertLevels, d.maxEdges, d.maxEdges2 = c["nVertLevels"], c["maxEdges"], c["maxEdges2"]
        d.num_scalars = c["num_scalars"]
        if sv is None:
            sv = (c["nCells"], c["nEdges"], c["nVertices"])
        d.nCellsSolve, d.nEdgesSolve, d.nVerticesSolve = (int(x) for x in sv)
        d.moist_start, d.moist_end, d.index_qv = 1, moist_end, 1
    return dims


def _install_lists(lib, h, blocks, placement, check, positional_rank=None, include_self=False):
    """Every block's send / receive lists (mpas_multihalo_exchange_list) into the context.
    positional_rank (this process's rank): the lists with other ranks go in as mpas_dmpar keeps them
    for tasks of several blocks -- positions in one buffer per task pair (decomp.positional_lists,
    mpas_dyc_set_exchange_positions); include_self: this rank's own block pairs too."""
    code = {"cell": _lib.CELL, "edge": _lib.EDGE, "vertex": _lib.VERTEX}
    if positional_rank is not None:
        from .decomp import positional_lists
        pos = positional_lists(blocks, placement, positional_rank, include_self=include_self)
        for ib, (b, lst) in enumerate(zip(blocks, pos)):
            for dname, loc, layer, pr, idx, p in lst:
                a = np.ascontiguousarray(idx + 1, dtype=np.int32)
                p = np.ascontiguousarray(p, dtype=np.int32)
                check(lib.mpas_dyc_set_exchange_positions(h, ib, code[loc], int(layer),
                                                          _lib.SEND if dname == "send" else _lib.RECV, int(pr),
                                                          a.ctypes.data_as(C.c_void_p), p.ctypes.data_as(C.c_void_p),
                                                          int(a.size)), "set_exchange_positions")
            for direction, lists in ((_lib.SEND, b.send), (_lib.RECV, b.recv)):
                for loc, layer, peer, idx in lists:
                    pr, pb = placement[peer]
                    if pr != positional_rank or include_self:
                        continue
                    a = np.ascontiguousarray(np.asarray(idx, dtype=np.int32) + 1)
                    check(lib.mpas_dyc_set_exchange_list(h, ib, code[loc], int(layer), direction, int(pr), int(pb),
                                                         a.ctypes.data_as(C.c_void_p), int(a.size)), "set_exchange_list")
        return
    for ib, b in enumerate(blocks):
        for direction, lists in ((_lib.SEND, b.send), (_lib.RECV, b.recv)):
            for loc, layer, peer, idx in lists:
                pr, pb = placement[peer]
                a = np.ascontiguousarray(np.asarray(idx, dtype=np.int32) + 1)
                check(lib.mpas_dyc_set_exchange_list(h, ib, code[loc], int(layer), direction, int(pr), int(pb),
                                                     a.ctypes.data_as(C.c_void_p), int(a.size)), "set_exchange_list")


def plan_exchanges(blocks: list, placement: dict, rank: int, nranks: int, dt: float, moist_end: int = 1,
                   overlap: bool | None = None, positional: bool = False) -> tuple[np.ndarray, list[str]]:
    """Dry run of the exchange planner for one rank, on the host (no GPU): the RCCL messages
    this rank posts over model init and one step on each time-level parity, and the plan key of
    every exchange call in issue order (mpas_dyc_plan_exchanges).  Messages are a structured array
    with fields point, direction (_lib.SEND / _lib.RECV), block, peer_rank, peer_block, count."""
    lib = _lib.load()
    cases = [b.case for b in blocks]
    dims = _make_dims(cases, [b.solve for b in blocks], moist_end)
    cfg = _lib.make_config(cases[0]["config"])
    h = C.c_void_p()
    rc = lib.mpas_dyc_create_blocks(len(cases), dims, C.byref(cfg), _lib.HOST_ONLY, C.byref(h))
    if rc != 0 or not h.value:
        raise DycoreError(f"mpas_dyc_create_blocks(HOST_ONLY) failed ({rc})")

    def check(r, what):
        if r != 0:
            msg = lib.mpas_dyc_last_error(h)
            raise DycoreError(f"{what} failed ({r}): {msg.decode() if msg else ''}")
    try:
        _install_lists(lib, h, blocks, placement, check, positional_rank=rank if positional else None)
        check(lib.mpas_dyc_set_overlap(h, -1 if overlap is None else int(bool(overlap))), "set_overlap")
        nm, kl = C.c_int64(), C.c_int64()
        lib.mpas_dyc_plan_exchanges(h, int(nranks), int(rank), float(dt), None, 0, C.byref(nm), None, 0,
                                    C.byref(kl))
        msgs = (_lib.PlanMsg * max(1, nm.value))()
        keys = C.create_string_buffer(kl.value)
        check(lib.mpas_dyc_plan_exchanges(h, int(nranks), int(rank), float(dt), msgs, nm.value, C.byref(nm), keys,
                                          kl.value, C.byref(kl)), "plan_exchanges")
        dt_msg = np.dtype([("point", "<i4"), ("direction", "<i4"), ("block", "<i4"), ("peer_rank", "<i4"),
                           ("peer_block", "<i4"), ("count", "<i8")], align=True)
        assert dt_msg.itemsize == C.sizeof(_lib.PlanMsg)
        arr = np.frombuffer(bytes(msgs), dtype=dt_msg)[:nm.value].copy()
        return arr, keys.value.decode().splitlines()
    finally:
        lib.mpas_dyc_destroy(h)


class Dycore:
    """The blocks of this process on one GPU (MPAS domain%blocklist).

    ``Dycore(case)`` is one block owning every element (the single-GPU path);
    ``Dycore.from_blocks(...)`` takes the blocks of a decomposition
    (``mpas_dycore.decomp``) and installs their exchange lists."""

    def __init__(self, case: dict | None = None, device: int = 0, solve: tuple | None = None, moist_end: int = 1,
                 _blocks: list | None = None, model_init: str = "host"):
        self.lib = _lib.load()
        cases = [case] if _blocks is None else [b.case for b in _blocks]
        solves = [solve] if _blocks is None else [b.solve for b in _blocks]
        self.cases = cases
        self.case = cases[0]
        self.K = self.case["nVertLevels"]
        self.ns = self.case["num_scalars"]
        self.nblocks = len(cases)
        self.nb = [{"cell": c["nCells"], "edge": c["nEdges"], "vertex": c["nVertices"]} for c in cases]
        self.n = self.nb[0]
        dims = _make_dims(cases, solves, moist_end)
        cfg = _lib.make_config(self.case["config"])
        h = C.c_void_p()
        rc = self.lib.mpas_dyc_create_blocks(len(cases), dims, C.byref(cfg), int(device), C.byref(h))
        if rc != 0 or not h.value:
            raise DycoreError(f"mpas_dyc_create_blocks failed ({rc})")
        self.h = h
        if model_init not in ("host", "device", "device_cr"):
            raise ValueError("model_init: 'host' (the case's precomputed arrays), 'device' (mpas_dyc_model_init with "
                             "the C library's x**0.25 / sin from the host) or 'device_cr' (correctly rounded on the device)")
        for ib, c in enumerate(cases):
            self._upload_case(c, ib, device_init=model_init != "host", host_libm=model_init == "device")
        if model_init != "host":
            cfg = self.case["config"]
            self._check(self.lib.mpas_dyc_model_init(self.h, int(bool(cfg.get("config_h_ScaleWithMesh", True))),
                                                     float(cfg["config_zd"]), float(cfg["config_xnutr"])),
                        "model_init")
            if all(n in c for c in cases for n in RECONSTRUCT_IN):
                self._check(self.lib.mpas_dyc_init_reconstruct(self.h), "init_reconstruct")

    @classmethod
    def from_blocks(cls, blocks: list, device: int = 0, moist_end: int = 1, placement: dict | None = None,
                    rank: int = 0, nranks: int = 1, comm_id: bytes | None = None, rccl_local: bool = False,
                    positional: bool = False, p2p: bool | None = None, host_group=None):
        """Blocks of this process (``decomp.decompose(..., parts=...)``) on one GPU.

        ``placement`` maps every block (part) id to (rank, local block index); by
        default all blocks live in this process, in the given order.  With
        ``nranks`` > 1, ``comm_id`` is the RCCL unique id created on rank 0.  ``p2p``: one-sided
        transfer between the ranks of the node (mpas_dyc_set_p2p; None = MPAS_DYCORE_P2P).
        ``host_group``: a torch.distributed process group (gloo) of the ranks instead of ``comm_id``: no
        RCCL communicator, the set-up all-gathers go through the group (mpas_dyc_comm_init_host) and
        every halo message through the one-sided transfer."""
        if placement is None:
            placement = {b.part: (0, i) for i, b in enumerate(blocks)}
        self = cls(device=device, moist_end=moist_end, _blocks=blocks)
        if comm_id is not None:
            idb = C.create_string_buffer(bytes(comm_id), len(comm_id))
            self._check(self.lib.mpas_dyc_comm_init(self.h, idb, len(comm_id), int(nranks), int(rank)), "comm_init")
        elif host_group is not None:
            self._host_allgather = _host_allgather_fn(host_group, int(nranks))  # kept alive with the context
            self._check(self.lib.mpas_dyc_comm_init_host(self.h, int(nranks), int(rank), self._host_allgather, None),
                        "comm_init_host")
        if rccl_local:
            self._check(self.lib.mpas_dyc_set_transport(self.h, 1), "set_transport")
        if p2p is not None:
            self._check(self.lib.mpas_dyc_set_p2p(self.h, int(bool(p2p))), "set_p2p")
        # positional: the lists with other ranks as mpas_dmpar keeps them for tasks of several blocks (with
        # rccl_local, this process's block pairs too) -- the Fortran drop-in's path
        _install_lists(self.lib, self.h, blocks, placement, self._check, positional_rank=rank if positional else None,
                       include_self=positional and rccl_local)
        return self

    def p2p_active(self) -> bool:
        """True while halo messages between ranks use the one-sided transfer (mpas_dyc_get_p2p)."""
        return bool(self.lib.mpas_dyc_get_p2p(self.h))

    def graph_active(self) -> bool:
        """True if the last step replayed its captured hipGraph (False: it ran eagerly)."""
        return bool(self.lib.mpas_dyc_graph_active(self.h))

    @staticmethod
    def comm_unique_id() -> bytes:
        lib = _lib.load()
        n = lib.mpas_dyc_comm_unique_id_bytes()
        buf = C.create_string_buffer(n)
        if lib.mpas_dyc_comm_unique_id(buf, n) != 0:
            raise DycoreError("mpas_dyc_comm_unique_id failed")
        return buf.raw

    def init_deriv_two(self, inputs, block: int = 0):
        """mpas_dyc_init_deriv_two: deriv_two's least-squares fits on the device into mesh.deriv_two,
        from the transcendental inputs init_atm.deriv_two_inputs(mesh) returns (xp, yp, sin_the,
        cos_the, each (nCells, maxEdges))."""
        nC, me = self.cases[block]["nCells"], self.cases[block]["maxEdges"]
        arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in inputs]
        if len(arrs) != 4 or any(a.shape != (nC, me) for a in arrs):
            raise ValueError(f"deriv_two inputs: four ({nC}, {me}) arrays")
        self._check(self.lib.mpas_dyc_init_deriv_two(self.h, block, *[a.ctypes.data_as(C.c_void_p) for a in arrs]),
                    "init_deriv_two")

    def init_zb(self, theta_adv_order: int = 3, block: int = 0):
        """mpas_dyc_init_zb: zb / zb3 on the device from the block's deriv_two and zgrid."""
        self._check(self.lib.mpas_dyc_init_zb(self.h, block, int(theta_adv_order)), "init_zb")

    # -------------------------------------------------------------- fields
    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.mpas_dyc_last_error(self.h)
            raise DycoreError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def set_raw(self, pool: str, name: str, fortran_image: np.ndarray, time_level: int = 1, block: int = 0):
        a = np.ascontiguousarray(fortran_image)
        self._check(self.lib.mpas_dyc_set_block_field(self.h, block, pool.encode(), name.encode(), time_level,
                                                      a.ctypes.data_as(C.c_void_p), a.nbytes),
                    f"set {pool}.{name}")

    def set(self, pool: str, name: str, arr, time_level: int = 1, block: int = 0):
        """Upload an element-major array (0-based indices for index fields)."""
        self.set_raw(pool, name, to_fortran({**self.cases[block], name: arr}, name), time_level, block)

    def get_raw(self, pool: str, name: str, time_level: int = 1, block: int = 0) -> np.ndarray:
        """Download a field's Fortran memory image (flat, garbage slot included): set_raw's inverse."""
        nb = self.lib.mpas_dyc_block_field_bytes(self.h, block, pool.encode(), name.encode())
        if nb <= 0:
            raise DycoreError(f"unknown field {pool}.{name}")
        buf = np.empty(nb // 8, dtype=np.float64)
        self._check(self.lib.mpas_dyc_get_block_field(self.h, block, pool.encode(), name.encode(), time_level,
                                                      buf.ctypes.data_as(C.c_void_p), buf.nbytes),
                    f"get {pool}.{name}")
        return buf

    def get(self, pool: str, name: str, time_level: int = 1, block: int = 0) -> np.ndarray:
        """Download a real field as element-major (n, inner) numpy (garbage slot dropped)."""
        nb = self.lib.mpas_dyc_block_field_bytes(self.h, block, pool.encode(), name.encode())
        if nb <= 0:
            raise DycoreError(f"unknown field {pool}.{name}")
        buf = np.empty(nb // 8, dtype=np.float64)
        self._check(self.lib.mpas_dyc_get_block_field(self.h, block, pool.encode(), name.encode(), time_level,
                                                      buf.ctypes.data_as(C.c_void_p), buf.nbytes),
                    f"get {pool}.{name}")
        loc = _loc_of(pool, name)
        if loc is None:
            return buf
        n1 = self.nb[block][loc] + 1
        if name in ("scalars", "scalars_tend"):
            return buf.reshape(n1, self.K, self.ns)[:-1]
        return buf.reshape(n1, buf.size // n1)[:-1]

    def set_overlap(self, on: bool | None = None):
        """Split-phase exchanges (interior elements overlap the halo traffic): True / False,
        or None for the library's automatic choice (on when exchanges go through RCCL)."""
        self._check(self.lib.mpas_dyc_set_overlap(self.h, -1 if on is None else (1 if on else 0)), "set_overlap")

    def halo_exchange(self, pool: str, name: str, time_level: int = 1, layers=(1, 2, 3)):
        """mpas_dmpar_exch_halo_field(field, haloLayers) over the blocks of this process (and peers)."""
        mask = sum(1 << (l - 1) for l in layers)
        self._check(self.lib.mpas_dyc_halo_exchange(self.h, pool.encode(), name.encode(), time_level, mask),
                    f"halo_exchange {pool}.{name}")

    def _upload_case(self, case: dict, block: int = 0, device_init: bool = False, host_libm: bool = True):
        """device_init: leave atm_mpas_init_block's precompute to the device (mpas_dyc_model_init) --
        upload its inputs (the init file's deriv_two, zb, zb3, meshDensity, areaCell, areaTriangle)
        instead of the case's precomputed arrays."""
        device_rec = device_init and all(n in case for n in RECONSTRUCT_IN)  # else the case's coefficients
        if device_init:
            for name in MODEL_INIT_IN + (RECONSTRUCT_IN if device_rec else ()):
                self.set_raw("mesh", name, to_fortran(case, name), block=block)
            # the C library's meshDensity**0.25 and damping-layer sin, as the compiled reference gets them
            # (init_atm.model_init_libm): the device's precompute then has the reference's bits
            if host_libm:
                from .init_atm import model_init_libm
                lm = model_init_libm(case, case["config"])
                for name, a in lm.items():
                    self.set_raw("mesh", name, to_fortran({**case, name: a}, name), block=block)
        for name in case:
            if name in _SKIP or (device_init and name in MODEL_INIT_OUT) or (device_rec and name == "coeffs_reconstruct"):
                continue
            if name in F.LOCATION or name in F.VERTICAL_1D:
                if name in F.VERTICAL_1D:
                    self.set_raw("mesh", name, np.asarray(case[name], dtype=np.float64), block=block)
                else:
                    self.set_raw("mesh", name, to_fortran(case, name), block=block)
            elif name in F.SCALARS_0D:
                self.set_raw("mesh", name, np.asarray([case[name]], dtype=np.float64), block=block)
        for name in STATE_INPUTS:
            self.set_raw("state", name, to_fortran(case, name), 1, block)
        for name in DIAG_INPUTS:
            self.set_raw("diag", name, to_fortran(case, name), block=block)

    # -------------------------------------------------------- operators
    def init_diagnostics(self, dt: float):
        """atm_init_coupled_diagnostics + atm_compute_solve_diagnostics (mpas_atm_core.F:387-404)."""
        self._check(self.lib.mpas_dyc_init_diagnostics(self.h, float(dt)), "init_diagnostics")

    def restart_diagnostics(self, dt: float):
        """Model init of a restart run (config_do_restart, mpas_atm_core.F:387-404): only
        atm_compute_solve_diagnostics, on a coupled state the host has set (mpas_dyc_solve_diagnostics)."""
        self._check(self.lib.mpas_dyc_solve_diagnostics(self.h, float(dt)), "solve_diagnostics")

    def atm_timestep(self, dt: float, itimestep: int = 1):
        """atm_timestep -> atm_srk3 (mpas_atm_time_integration.F:87-139); asynchronous."""
        self._check(self.lib.mpas_dyc_timestep(self.h, float(dt), int(itimestep)), "atm_timestep")

    def set_lbc(self, apply: bool, seconds_to_interval_end: float = 0.0):
        """config_apply_lbcs (mpas_dyc_set_lbc): regional boundary conditions on/off, and before every
        step the seconds from the step's start to the end of the current LBC interval.  The driving
        data go into pool "lbc" (lbc_u, lbc_ru, lbc_rho_zz, lbc_rtheta_m, lbc_scalars; time level 1 =
        tendency, 2 = interval-end state) and the masks into the mesh pool."""
        self._check(self.lib.mpas_dyc_set_lbc(self.h, 1 if apply else 0, float(seconds_to_interval_end)), "set_lbc")

    PHYSICS_TENDENCIES, PHYSICS_RQVDYNTEN, PHYSICS_MICROPHYSICS = 1, 2, 4

    def set_physics(self, tendencies: bool = True, rqvdynten: bool = False, microphysics: bool = False):
        """Physics coupling (the reference's DO_PHYSICS build): the host sets tend_physics.
        tend_ru_physics / tend_rtheta_physics / tend_rho_physics and tend.scalars_tend before each
        step (as physics_get_tend does, mpas_atm_time_integration.F:424-449).  ``microphysics``: the
        host runs the microphysics on time level 2 after each step and then calls finish_step(),
        which runs the rest of atm_srk3 (the regional specified-zone reset, summarize_timestep)."""
        flags = ((self.PHYSICS_TENDENCIES if tendencies else 0) | (self.PHYSICS_RQVDYNTEN if rqvdynten else 0)
                 | (self.PHYSICS_MICROPHYSICS if microphysics else 0))
        self._check(self.lib.mpas_dyc_set_physics(self.h, flags), "set_physics")

    def finish_step(self, dt: float):
        """The end of atm_srk3 after the host's microphysics (1672-1794); a no-op unless
        set_physics(microphysics=True).  Call before shift_time_levels."""
        self._check(self.lib.mpas_dyc_finish_step(self.h, float(dt)), "finish_step")

    def output_diagnostics(self, time_level: int = 1):
        """atm_compute_output_diagnostics (mpas_atm_core.F:753-800): diag theta, rho, pressure."""
        self._check(self.lib.mpas_dyc_output_diagnostics(self.h, int(time_level)), "output_diagnostics")

    def set_summary(self, global_minmax_vel: bool = True, detailed_minmax_vel: bool = False,
                    global_minmax_sca: bool = False):
        """The namelist switches of summarize_timestep (Registry.xml:339-349): which reductions
        every following step performs at its end (mpas_atm_time_integration.F:1794)."""
        flags = ((_lib.PRINT_GLOBAL_MINMAX_VEL if global_minmax_vel else 0)
                 | (_lib.PRINT_DETAILED_MINMAX_VEL if detailed_minmax_vel else 0)
                 | (_lib.PRINT_GLOBAL_MINMAX_SCA if global_minmax_sca else 0))
        self._check(self.lib.mpas_dyc_set_summary(self.h, flags), "set_summary")

    def summarize_timestep(self, log=None, block: int | None = None) -> dict:
        """summarize_timestep (mpas_atm_time_integration.F:6675-7018) of the last step: the global
        extrema over all blocks and ranks, and the reference's log lines (passed to ``log`` if given).
        ``block``: that block of this process only, reduced over ranks -- the reference writes one
        set of lines per block (6945-6983).
        In detailed mode a NaN in w or u raises DycoreError, as the reference aborts (6926-6940)."""
        s = _lib.Summary()
        mm = (C.c_double * (2 * self.ns))()
        if block is None:
            rc = self.lib.mpas_dyc_get_summary(self.h, C.byref(s), mm, 2 * self.ns)
        else:
            rc = self.lib.mpas_dyc_get_block_summary(self.h, int(block), C.byref(s), mm, 2 * self.ns)
        self._check(rc, "summarize_timestep")
        out = {"flags": s.flags, "w_min": s.w_min, "w_max": s.w_max, "u_min": s.u_min, "u_max": s.u_max,
               "nan_w": s.nan_w, "nan_u": s.nan_u, "scalars": [(mm[2 * i], mm[2 * i + 1]) for i in range(self.ns)]}
        for n in ("w_min_at", "w_max_at", "u_min_at", "u_max_at", "wsp_max_at"):
            e = getattr(s, n)
            out[n] = {"value": e.value, "k": e.k, "index": e.index, "lat": e.lat, "lon": e.lon}
        lines = []
        if s.flags & _lib.PRINT_DETAILED_MINMAX_VEL:
            lines.append("")
            for n, tag in (("w_min_at", "min w"), ("w_max_at", "max w"), ("u_min_at", "min u"),
                           ("u_max_at", "max u"), ("wsp_max_at", "max wsp")):
                e = out[n]
                lines.append(f" global {tag}: {e['value']} k={e['k']}, {e['lat']} lat, {e['lon']} lon")
        elif s.flags & _lib.PRINT_GLOBAL_MINMAX_VEL:
            lines += ["", f"global min, max w {s.w_min} {s.w_max}", f"global min, max u {s.u_min} {s.u_max}"]
        if s.flags & _lib.PRINT_GLOBAL_MINMAX_SCA:
            if not s.flags & (_lib.PRINT_GLOBAL_MINMAX_VEL | _lib.PRINT_DETAILED_MINMAX_VEL):
                lines.append("")
            lines += [f" global min, max scalar {i + 1} {a} {b}" for i, (a, b) in enumerate(out["scalars"])]
        out["log"] = lines
        if log is not None:
            for ln in lines:
                log(ln)
        if s.flags & _lib.PRINT_DETAILED_MINMAX_VEL and (s.nan_w or s.nan_u):
            raise DycoreError("NaN detected in '" + ("w" if s.nan_w else "u") + "' field.")
        return out

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

    def layout(self, block: int = 0) -> dict:
        """How the kernels see a block (mpas_dyc_block_layout): the maxEdges / maxEdges2 they index
        with, the kernel family and the column shape ("wavefront": nVertLevels <= 63, a column per
        wavefront or half of one; "wide": 64..127, a wavefront per column in the pair layout, a
        128-lane workgroup in the per-cell kernels; "wide256": 128..255, a 256-lane workgroup per
        column in every kernel; "wide512": 256..511, a 512-lane workgroup)."""
        out = (C.c_int32 * 4)()
        self._check(self.lib.mpas_dyc_block_layout(self.h, int(block), out), "block_layout")
        return {"maxEdges": out[0], "maxEdges2": out[1], "family": ("general", "batched", "pair")[out[2]],
                "column": ("wavefront", "wide", "wide256", "wide512")[out[3]]}

    def exchange_profile(self, dt: float, itimestep: int = 1) -> dict:
        """One eager atm_timestep with HIP events around every exchange's exposed part and every
        RCCL group (mpas_dyc_set_profile / mpas_dyc_get_profile); synchronous.  Shift the time
        levels afterwards as after any step."""
        self._check(self.lib.mpas_dyc_set_profile(self.h, 1), "set_profile")
        try:
            self.atm_timestep(dt, itimestep)
        finally:
            self._check(self.lib.mpas_dyc_set_profile(self.h, 0), "set_profile")
        out = (C.c_double * 5)()
        self._check(self.lib.mpas_dyc_get_profile(self.h, out, 5), "get_profile")
        return {"exchanges": int(out[0]), "ms_step_eager": out[1], "ms_exchange_exposed": out[2],
                "ms_compute": out[1] - out[2], "rccl_groups": int(out[3]), "ms_rccl_groups": out[4]}

    def last_exchange(self) -> str:
        """Plan key of the exchange whose RCCL group was enqueued last (thread-safe read)."""
        k = self.lib.mpas_dyc_last_exchange(self.h) if self.h else None
        return k.decode() if k else ""

    @staticmethod
    def rccl_version() -> int:
        return int(_lib.load().mpas_dyc_rccl_version())

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
for _n in ("theta_m", "rho_zz", "rho_p", "rtheta_p", "exner", "pressure_p", "pressure", "kdiff", "ke", "divergence", "rw",
           "wwAvg", "cqw", "h_divergence", "pv_cell", "rho_pp", "rtheta_pp", "rw_p", "exner_base", "pressure_base",
           "rtheta_base", "coftz", "cofwz", "cofwr", "cofwt", "a_tri", "alpha_tri", "gamma_tri", "rw_save",
           "tend_rtheta_adv", "rho_p_save", "rtheta_p_save", "rho_zz_old_split", "rtheta_pp_old", "wwAvg_split",
           "tend_rtheta_physics", "tend_rho_physics", "rqvdynten",
           "scalars_tend", "rthdynten", "rt_diabatic_tend", "theta_euler", "w_euler", "uReconstructX",
           "uReconstructY", "uReconstructZ", "uReconstructZonal", "uReconstructMeridional"):
    _LOCS[_n] = "cell"
for _n in ("ru", "ruAvg", "ru_p", "ru_save", "cqu", "rho_edge", "v", "pv_edge", "gradPVn", "gradPVt", "tend_ru_physics",
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
