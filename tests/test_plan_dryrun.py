"""The multi-process RCCL path, checked on the host before any GPU runs it.

Every rank of an N-GPU run (bench.py --gpus N: one block per rank, SFC partition) builds its
exchange plans with the library's own planner in a host-only context (MPAS_DYC_HOST_ONLY,
mpas_dyc_plan_exchanges) over what a run issues: the model-init exchanges and one atm_srk3 on
each time-level parity.  For N = 2, 4, 8 on the x1.163842 mesh this asserts what ncclGroupStart /
ncclGroupEnd needs across ranks (the reference's MPI_Isend/MPI_Irecv pairs, mpas_dmpar.F:5386-5552):

  * every rank issues the same exchange calls in the same order (same plan keys), so the
    captured graphs and warm_rccl (plans in key order) line up;
  * at every call, rank r's ncclSend list to rank p equals rank p's ncclRecv list from r:
    same messages (source block -> destination block), same order, same element counts;
  * the counts are the sizes of the exchange lists decomp.py built for that pair.
"""
import numpy as np
import pytest

from mpas_dycore import _lib, decomp
from mpas_dycore.dycore import plan_exchanges
from mpas_dycore.preflight import PlanMismatch, check_plans


@pytest.fixture(scope="module")
def case163842():
    from mpas_dycore.cases import jw_case
    return jw_case(163842, K=56, ns=1, order=3)


def _plans(case, nranks, overlap=None):
    cell_part = decomp.partition_sfc(case["nCells"], nranks)
    out = []
    for r in range(nranks):
        blocks, placement = decomp.rank_blocks(case, nranks, r, 1, cell_part=cell_part)
        out.append(plan_exchanges(blocks, placement, r, nranks, float(case["dt"]), overlap=overlap))
    return out


def _check_matching(plans, nranks):
    assert len(plans) == nranks
    got = check_plans(plans)
    assert got["plan_keys"] > 40
    return got["messages"]


def test_mismatch_is_reported(case163842):
    """A rank whose receive list differs is caught before any GPU call, naming the exchange."""
    plans = _plans(case163842, 2)
    msgs = plans[1][0].copy()
    j = np.flatnonzero(msgs["direction"] == _lib.RECV)[3]
    msgs["count"][j] += 1
    with pytest.raises(PlanMismatch) as e:
        check_plans([plans[0], (msgs, plans[1][1])])
    assert e.value.key == plans[0][1][e.value.point]


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_rank_plans_match_x1_163842(case163842, nranks):
    plans = _plans(case163842, nranks)
    nmsg = _check_matching(plans, nranks)
    assert nmsg > 0
    # a rank never messages itself with one block per rank
    for r in range(nranks):
        assert not np.any(plans[r][0]["peer_rank"] == r)


def test_message_sizes_are_the_exchange_lists(case163842):
    """The step-start exchange (theta_m, scalars, pressure_p, rtheta_p, exner over all layers,
    mpas_atm_time_integration.F:329-338 + 513) of rank 0 sends, per peer, 5 cell fields of K
    levels over every cell this rank lists for that peer."""
    nranks = 4
    case = case163842
    cell_part = decomp.partition_sfc(case["nCells"], nranks)
    blocks, placement = decomp.rank_blocks(case, nranks, 0, 1, cell_part=cell_part)
    msgs, keys = plan_exchanges(blocks, placement, 0, nranks, float(case["dt"]))
    i = next(j for j, k in enumerate(keys) if "state.theta_m" in k and "diag.exner" in k and "diag.pv_edge" not in k)
    K = case["nVertLevels"]
    send = decomp.messages(blocks[0], "send", layers=(1, 2), locs=("cell",))
    got = msgs[(msgs["point"] == i) & (msgs["direction"] == _lib.SEND)]
    assert sorted(got["peer_rank"].tolist()) == sorted(placement[p][0] for p in send)
    for part, idx in send.items():
        pr, pb = placement[part]
        m = got[(got["peer_rank"] == pr) & (got["peer_block"] == pb)]
        assert len(m) == 1 and m["count"][0] == 5 * K * idx.size


def test_plans_match_without_split_phase(case163842):
    plans = _plans(case163842, 2, overlap=False)
    assert _check_matching(plans, 2) > 0


def test_host_only_context_refuses_device_calls(case163842):
    import ctypes as C
    lib = _lib.load()
    c = case163842
    from mpas_dycore.dycore import _make_dims
    dims = _make_dims([c], [None], 1)
    cfg = _lib.make_config(c["config"])
    h = C.c_void_p()
    assert lib.mpas_dyc_create_blocks(1, dims, C.byref(cfg), _lib.HOST_ONLY, C.byref(h)) == 0
    try:
        assert lib.mpas_dyc_timestep(h, 1.0, 1) == -3
        assert lib.mpas_dyc_init_diagnostics(h, 1.0) == -3
        buf = np.zeros(8)
        assert lib.mpas_dyc_set_field(h, b"mesh", b"cf1", 1, buf.ctypes.data_as(C.c_void_p), 8) == -3
        # the device model-init entry points: ESTATE without a device, EINVAL for bad arguments
        assert lib.mpas_dyc_model_init(h, 1, 22000.0, 0.2) == -3
        x = buf.ctypes.data_as(C.c_void_p)
        assert lib.mpas_dyc_init_deriv_two(h, 0, x, x, x, x) == -3
        assert lib.mpas_dyc_init_deriv_two(h, 0, None, x, x, x) == -1
        assert lib.mpas_dyc_init_zb(h, 0, 3) == -3
        assert lib.mpas_dyc_init_zb(h, 0, 5) == -1
        assert lib.mpas_dyc_init_reconstruct(h) == -3
        assert lib.mpas_dyc_init_reconstruct(None) == -1
    finally:
        lib.mpas_dyc_destroy(h)
