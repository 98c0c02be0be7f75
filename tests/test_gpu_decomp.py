"""GPU: domain decomposition with halo exchange reproduces the single-block dycore bit for bit.

MPAS results do not depend on the decomposition: every stencil reads halo
values that the reference's mpas_dmpar_exch_halo_field calls have made exact.
The HIP path is therefore checked in three ways:
  * Owned values after N blocks + exchanges are **bitwise equal** to one block.
  * The exchange itself matches global values on every halo layer.
  * The RCCL transport (send/recv to self, one rank) gives the same bits as the
    in-process block-to-block copies.
Multi-process RCCL between GPUs is exercised by bench.py --gpus N.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DT = 2880.0
FIELDS = [("state", "u", "edge"), ("state", "theta_m", "cell"), ("state", "rho_zz", "cell"),
          ("state", "w", "cell"), ("state", "scalars", "cell")]


def _run(dy, nsteps):
    dy.init_diagnostics(DT)
    for it in range(nsteps):
        dy.atm_timestep(DT, it + 1)
        dy.shift_time_levels()
    dy.synchronize()


def _single(case, nsteps, graph=False):
    from mpas_dycore import Dycore
    dy = Dycore(case, device=0)
    dy.use_graph(graph)
    _run(dy, nsteps)
    out = {n: dy.get(p, n, 1) for p, n, _ in FIELDS}
    dy.close()
    return out


def _blocks(case, nblocks, nsteps, graph=False, rccl_local=False, overlap=True, positional=False, moist_end=1):
    from mpas_dycore import Dycore, decomp
    part = decomp.partition_sfc(case["nCells"], nblocks)
    blocks = decomp.decompose(case, part)
    comm_id = Dycore.comm_unique_id() if rccl_local else None
    dy = Dycore.from_blocks(blocks, device=0, comm_id=comm_id, nranks=1, rank=0, rccl_local=rccl_local,
                            positional=positional, moist_end=moist_end)
    dy.set_overlap(overlap)
    dy.use_graph(graph)
    _run(dy, nsteps)
    n_glob = {"cell": case["nCells"], "edge": case["nEdges"]}
    out = {}
    for p, n, loc in FIELDS:
        per = [dy.get(p, n, 1, block=i) for i in range(len(blocks))]
        out[n] = decomp.gather_owned(blocks, per, loc, n_glob[loc])
    dy.close()
    return out


@pytest.mark.parametrize("nblocks", [2, 5])
def test_halo_exchange_fills_every_layer(small_case, nblocks):
    from mpas_dycore import Dycore, decomp
    case = small_case
    blocks = decomp.decompose(case, decomp.partition_sfc(case["nCells"], nblocks))
    dy = Dycore.from_blocks(blocks, device=0)
    rng = np.random.default_rng(7)
    for pool, name, loc, tl in (("state", "u", "edge", 2), ("diag", "pv_edge", "edge", 0),
                                ("diag", "rho_pp", "cell", 0), ("state", "w", "cell", 1),
                                ("diag", "vorticity", "vertex", 0)):
        inner = dy.get(pool, name, max(tl, 1)).shape[1]
        n = {"cell": case["nCells"], "edge": case["nEdges"], "vertex": case["nVertices"]}[loc]
        g = rng.standard_normal((n, inner))
        for i, b in enumerate(blocks):
            a = np.full((b.glob[loc].size + 1, inner), np.nan)
            no = b.layer_end[loc][0]
            a[:no] = g[b.glob[loc][:no]]
            dy.set_raw(pool, name, a, max(tl, 1), block=i)
        dy.halo_exchange(pool, name, max(tl, 1))
        for i, b in enumerate(blocks):
            got = dy.get(pool, name, max(tl, 1), block=i)
            assert np.array_equal(got, g[b.glob[loc]]), f"{pool}.{name} block {i}"
    dy.close()


@pytest.mark.parametrize("nblocks", [3, 4])
def test_blocks_bitwise_equal_single_block(small_case, nblocks):
    ref = _single(small_case, 3)
    got = _blocks(small_case, nblocks, 3)
    for name in ref:
        assert np.array_equal(got[name], ref[name]), f"{name}: max diff {np.nanmax(np.abs(got[name] - ref[name]))}"


def test_blocks_moist_mono_transport_bitwise(moist_case):
    ref = _single(moist_case, 2)
    got = _blocks(moist_case, 3, 2, graph=True)
    for name in ref:
        assert np.array_equal(got[name], ref[name]), f"{name}: max diff {np.nanmax(np.abs(got[name] - ref[name]))}"


@pytest.mark.parametrize("graph", [False, True])
def test_split_phase_exchange_bitwise(small_case, graph):
    """Interior/boundary split around the tend_u / rho_pp / rtheta_pp exchanges (exchange
    stream overlapping the interior kernels) changes no bit."""
    ref = _single(small_case, 3)
    got = _blocks(small_case, 4, 3, graph=graph, overlap=True)
    seq = _blocks(small_case, 4, 3, graph=graph, overlap=False)
    for name in ref:
        assert np.array_equal(got[name], ref[name]), name
        assert np.array_equal(seq[name], ref[name]), name


def test_rccl_transport_matches_device_copies(small_case):
    a = _blocks(small_case, 2, 2, graph=False, rccl_local=False)
    b = _blocks(small_case, 2, 2, graph=True, rccl_local=True)
    for name in a:
        assert np.array_equal(a[name], b[name]), name


@pytest.mark.parametrize("which", ["small_case", "moist_case"])
def test_positional_lists_bitwise(which, request):
    """The lists of a task that holds several blocks, as mpas_dmpar keeps them and the Fortran drop-in
    hands them over (one buffer per task pair and halo layer, positions filled by all the task's
    blocks; mpas_dyc_set_exchange_positions): 4 blocks exchanging through RCCL by positions equal the
    block-pair lists and one block bit for bit, graph replay, split-phase exchanges."""
    case = request.getfixturevalue(which)
    me = case["num_scalars"]
    a = _blocks(case, 4, 3, graph=True, rccl_local=True, moist_end=me)
    b = _blocks(case, 4, 3, graph=True, rccl_local=True, positional=True, moist_end=me)
    for name in a:
        assert np.array_equal(a[name], b[name]), f"{name}: positional lists differ from block-pair lists"


@pytest.mark.parametrize("overlap", [True, False])
def test_fused_pack_bitwise(small_case, overlap):
    """The per-sub-step rtheta_pp / rho_pp exchange packed by the acoustic cell phase itself (the
    PackMap epilogue of k_acoustic_cells_r, no pack kernel) and unpacked by its consumer (the next
    edge phase or the stage's last damping read the receive buffer through an UnpackMap and write
    the halo columns back, no unpack kernel) gives the bits of the separate pack / unpack kernels
    (MPAS_DYCORE_FUSED_PACK=0) and of one block; 4 RCCL blocks, graph replay."""
    import os
    one = _single(small_case, 3)
    runs = []
    for fused in ("1", "0"):
        old = os.environ.get("MPAS_DYCORE_FUSED_PACK")
        os.environ["MPAS_DYCORE_FUSED_PACK"] = fused
        try:
            runs.append(_blocks(small_case, 4, 3, graph=True, rccl_local=True, overlap=overlap))
        finally:
            if old is None:
                os.environ.pop("MPAS_DYCORE_FUSED_PACK", None)
            else:
                os.environ["MPAS_DYCORE_FUSED_PACK"] = old
    for name in one:
        assert np.array_equal(runs[0][name], runs[1][name]), f"{name}: fused pack differs from the pack kernel"
        assert np.array_equal(runs[0][name], one[name]), f"{name}: fused-pack blocks differ from one block"


def test_fused_exchanges_keep_halo_fields(small_case):
    """The tend_u exchange (642), the exchange before the recovery (876-887) and the u exchange
    after it (988) packed by their producing kernels and unpacked by their consumers (XPack /
    XUnpack: dyn_tend's final tend_u kernel -> k_smlstep_pert_b; the stage's last cell phase and
    damping -> k_recover_cells1 / k_recover_edges; the recovery -> k_diag_vertices_p), and the
    exchange after the diagnostics (1234-1249, with 1282-1297 at a substep's end) packed by the w
    recovery and the diagnostics' edge kernel, leave every exchanged field, halo columns included,
    as the pack / unpack kernels do (MPAS_DYCORE_FUSED_PACK=0); 4 RCCL blocks, split-phase
    exchanges, graph replay."""
    import os
    from mpas_dycore import Dycore, decomp
    part = decomp.partition_sfc(small_case["nCells"], 4)
    blocks = decomp.decompose(small_case, part)
    names = [("diag", "rw_p"), ("diag", "ru_p"), ("diag", "rho_pp"), ("diag", "rtheta_pp"), ("tend", "u"),
             ("state", "u"), ("state", "w"), ("diag", "pv_edge"), ("diag", "rho_edge"), ("state", "theta_m"),
             ("diag", "pressure_p"), ("diag", "rtheta_p"), ("diag", "exner")]
    runs = []
    for fused in ("1", "0"):
        old = os.environ.get("MPAS_DYCORE_FUSED_PACK")
        os.environ["MPAS_DYCORE_FUSED_PACK"] = fused
        try:
            dy = Dycore.from_blocks(blocks, device=0, comm_id=Dycore.comm_unique_id(), nranks=1, rank=0,
                                    rccl_local=True)
        finally:
            if old is None:
                os.environ.pop("MPAS_DYCORE_FUSED_PACK", None)
            else:
                os.environ["MPAS_DYCORE_FUSED_PACK"] = old
        dy.set_overlap(True)
        dy.use_graph(True)
        _run(dy, 2)
        runs.append({(p, n, i): dy.get(p, n, 1, block=i) for p, n in names for i in range(len(blocks))})
        dy.close()
    for key in runs[1]:
        assert np.array_equal(runs[0][key], runs[1][key]), f"{key}: fused exchange differs from pack/unpack kernels"


@pytest.mark.parametrize("mode", ["pull", "buffers", "split"])
@pytest.mark.parametrize("which", ["small_case", "moist_case"])
def test_p2p_transport_bitwise(which, mode, request):
    """One-sided transfer (MPAS_DYCORE_P2P=1; halo.hip): 4 blocks of one rank whose messages all go
    through the one-sided protocol equal one block bit for bit, graph replay.  pull: blocking
    exchanges, the receiver copies the sender's owned columns from its fields (k_p2p_pull, the p2p
    default); buffers: blocking, send buffers pulled into receive buffers with the fused packs and
    unpacks (k_p2p_exchange, MPAS_DYCORE_P2P_PULL=0); split: split-phase exchanges (k_p2p_post at the
    exchange, k_p2p_get where the halo is read)."""
    import os
    case = request.getfixturevalue(which)
    one = _single(case, 3)
    env = {"MPAS_DYCORE_P2P": "1", "MPAS_DYCORE_P2P_PULL": "0" if mode == "buffers" else "1"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        got = _blocks(case, 4, 3, graph=True, rccl_local=True, overlap=mode == "split")
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for name in one:
        assert np.array_equal(got[name], one[name]), f"{name}: p2p blocks differ from one block"
