"""Several blocks per task with several tasks: the exchange lists as mpas_dmpar keeps them then.

With more than one block on a task, parinfo's xToSend / xToRecv lists name the peer *task* only
(endPointID) and place each element at a position of one buffer per task pair and halo layer, which
all blocks of the task fill together (mpas_dmpar.F:5448-5535).  The Fortran drop-in hands those lists
to the library unchanged (mpas_dyc_set_exchange_positions).  Checked here without a GPU, in host-only
contexts (mpas_dyc_plan_exchanges) over one model run's exchange calls:

  * the reference's own lists -- mpas_block_decomp.F / mpas_block_creator.F run by
    oracle/_ref/decomp_harness under mpirun, 4 blocks on 2 tasks -- installed as the drop-in installs
    them: every task's RCCL sends pair with its peer's receives, message by message and size by size;
  * the Python host's restatement of such lists (decomp.positional_lists) for 2 tasks x 2 blocks and
    4 tasks x 2 blocks at x1.163842: the same, and each message is the sum of its regions.
"""
import ctypes as C
import os

import numpy as np
import pytest

from mpas_dycore import _lib, decomp
from mpas_dycore.dycore import plan_exchanges
from mpas_dycore.preflight import check_plans

LOCS = {"cell": _lib.CELL, "edge": _lib.EDGE, "vertex": _lib.VERTEX}


@pytest.fixture(scope="module")
def mesh2562():
    from mpas_dycore.cases import jw_case
    return jw_case(2562, K=26, ns=1, cache=False)


def _plan_rank(case, blocks_res, task, blocks_of_task):
    """A host-only context of one task's blocks with the reference's lists installed as the drop-in
    installs them (copy lists block to block, the other tasks' lists by position)."""
    lib = _lib.load()
    dims = (_lib.Dims * len(blocks_of_task))()
    for d, gb in zip(dims, blocks_of_task):
        r = blocks_res[gb]
        d.nCells, d.nEdges, d.nVertices = (len(r[f"{loc}_index"]) for loc in ("cell", "edge", "vertex"))
        d.nCellsSolve, d.nEdgesSolve, d.nVerticesSolve = (int(r[f"{loc}_solve"][0]) for loc in ("cell", "edge", "vertex"))
        d.nVertLevels, d.maxEdges, d.maxEdges2, d.num_scalars = case["nVertLevels"], case["maxEdges"], case["maxEdges2"], 1
        d.moist_start, d.moist_end, d.index_qv = 1, 1, 1
    cfg = _lib.make_config(case["config"])
    h = C.c_void_p()
    assert lib.mpas_dyc_create_blocks(len(blocks_of_task), dims, C.byref(cfg), _lib.HOST_ONLY, C.byref(h)) == 0

    def i32(a):
        return np.ascontiguousarray(np.asarray(a, dtype=np.int32))
    try:
        for lb, gb in enumerate(blocks_of_task):
            r = blocks_res[gb]
            for loc, code in LOCS.items():
                for layer in (1, 2, 3):
                    for ep, src, dst in r.get(f"{loc}_copy_{layer}", []):
                        s, d = i32(src), i32(dst)
                        assert lib.mpas_dyc_set_exchange_list(h, lb, code, layer, _lib.SEND, task, ep, s.ctypes.data_as(C.c_void_p), s.size) == 0
                        assert lib.mpas_dyc_set_exchange_list(h, ep, code, layer, _lib.RECV, task, lb, d.ctypes.data_as(C.c_void_p), d.size) == 0
                    for ep, src, dst in r.get(f"{loc}_send_{layer}", []):
                        s, p = i32(src), i32(dst)
                        assert lib.mpas_dyc_set_exchange_positions(h, lb, code, layer, _lib.SEND, ep, s.ctypes.data_as(C.c_void_p), p.ctypes.data_as(C.c_void_p), s.size) == 0
                    for ep, src, dst in r.get(f"{loc}_recv_{layer}", []):
                        p, d = i32(src), i32(dst)
                        assert lib.mpas_dyc_set_exchange_positions(h, lb, code, layer, _lib.RECV, ep, d.ctypes.data_as(C.c_void_p), p.ctypes.data_as(C.c_void_p), d.size) == 0
        nm, kl = C.c_int64(), C.c_int64()
        ntask = 2
        rc = lib.mpas_dyc_plan_exchanges(h, ntask, task, float(case["dt"]), None, 0, C.byref(nm), None, 0, C.byref(kl))
        assert nm.value > 0, (rc, lib.mpas_dyc_last_error(h))
        msgs = (_lib.PlanMsg * max(1, nm.value))()
        keys = C.create_string_buffer(kl.value)
        assert lib.mpas_dyc_plan_exchanges(h, ntask, task, float(case["dt"]), msgs, nm.value, C.byref(nm), keys, kl.value,
                                           C.byref(kl)) == 0
        dt_msg = np.dtype([("point", "<i4"), ("direction", "<i4"), ("block", "<i4"), ("peer_rank", "<i4"),
                           ("peer_block", "<i4"), ("count", "<i8")], align=True)
        return np.frombuffer(bytes(msgs), dtype=dt_msg)[:nm.value].copy(), keys.value.decode().splitlines()
    finally:
        lib.mpas_dyc_destroy(h)


@pytest.mark.skipif(not os.access("/opt/conda/bin/mpirun", os.X_OK), reason="no mpirun")
def test_reference_lists_four_blocks_two_tasks(mesh2562):
    from oracle import ref_runner
    if not ref_runner.available(ref_runner.DECOMP_HARNESS):
        pytest.skip("oracle/_ref/decomp_harness not built")
    part = decomp.partition_sfc(mesh2562["nCells"], 4)
    res = ref_runner.run_reference_decomp(mesh2562, part, nprocs=2)
    # mpas_get_owning_proc with 4 blocks on 2 tasks: blocks 0, 1 on task 0, blocks 2, 3 on task 1
    plans = [_plan_rank(mesh2562, res, t, [2 * t, 2 * t + 1]) for t in range(2)]
    got = check_plans(plans)
    assert got["plan_keys"] > 40 and got["messages"] > 0
    # one message per peer task and exchange, filled by both blocks (block -1); the copy lists between
    # the blocks of a task stay device copies, no message
    for t, (msgs, _) in enumerate(plans):
        assert (msgs["peer_rank"] == 1 - t).all()
        assert (msgs["block"] == -1).all() and (msgs["peer_block"] == -1).all()
    # the step-start exchange of theta_m etc. moves 5 fields x K levels over the buffer's slots: its
    # cell message from task 0 to task 1 is 5 K times the largest position of the two layers' lists
    K = mesh2562["nVertLevels"]
    msgs, keys = plans[0]
    i = next(j for j, k in enumerate(keys) if "state.theta_m" in k and "diag.exner" in k and "diag.pv_edge" not in k)
    m = msgs[(msgs["point"] == i) & (msgs["direction"] == _lib.SEND)]
    slots = sum(max(int(d.max()) for b in (0, 1) for ep, s, d in res[b][f"cell_send_{layer}"] if ep == 1)
                for layer in (1, 2))
    assert len(m) == 1 and m["count"][0] == 5 * K * slots


@pytest.mark.parametrize("ntask,nper,ncells", [(2, 2, 2562), (4, 2, 163842)])
def test_python_positional_lists_pair_up(ntask, nper, ncells, mesh2562):
    from mpas_dycore.cases import jw_case
    case = mesh2562 if ncells == 2562 else jw_case(163842, K=56, ns=1, order=3)
    cell_part = decomp.partition_sfc(case["nCells"], ntask * nper)
    plans = []
    for r in range(ntask):
        blocks, placement = decomp.rank_blocks(case, ntask, r, nper, cell_part=cell_part)
        plans.append(plan_exchanges(blocks, placement, r, ntask, float(case["dt"]), positional=True))
    got = check_plans(plans)
    assert got["messages"] > 0
    # with block-pair lists the same run posts one message per peer rank too (merged), of the sum of
    # its block pairs; positional buffers hold every element once per (peer task, layer), so they are
    # no larger
    plain = []
    for r in range(ntask):
        blocks, placement = decomp.rank_blocks(case, ntask, r, nper, cell_part=cell_part)
        plain.append(plan_exchanges(blocks, placement, r, ntask, float(case["dt"])))
    for (mp, kp), (mb, kb) in zip(plans, plain):
        assert kp == kb
        for d in (_lib.SEND, _lib.RECV):
            a, b = mp[mp["direction"] == d], mb[mb["direction"] == d]
            assert np.array_equal(a[["point", "peer_rank"]], b[["point", "peer_rank"]])
            assert (a["count"] <= b["count"]).all()
