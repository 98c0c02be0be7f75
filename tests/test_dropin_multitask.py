"""CPU: the Fortran drop-in's multi-task path, executed.

The drop-in (mpas-model_amd/fortran/atm_time_integration_mi355x.F90) builds its domain context on
the first atm_srk3 (create_domain_context): every block of domain%blocklist, the RCCL id broadcast
from task 0 over dminfo%comm (mpas_dmpar_bcast_ints), and set_block_lists, which hands parinfo's
xToCopy / xToSend / xToRecv lists to the library -- sorted by buffer position with one block per task
(block-pair lists), as they are with several blocks per task (positional lists).  On MI355X this
code runs first in every multi-GPU deployment of the drop-in.

Here it runs without a GPU: oracle/_ref/dropin_plan_harness is decomp_harness.F90 built with
-DDROPIN_PLAN against the drop-in module and libmpas_dycore.so.  Under mpirun -np P it runs the
reference's own decomposition (mpas_block_decomp.F, mpas_block_creator.F's halo builder), gives each
task's blocks their parinfo lists and pool dimensions as mpas_block_creator.F:1000-1147 does, and calls
the drop-in's atm_dycore_plan_exchanges: create_domain_context on host-only contexts (no uploads, no
model init), then mpas_dyc_plan_exchanges over one model run's exchange calls.  Checked:
  * every task received task 0's id words;
  * every task's RCCL sends pair with its peers' receives, in order and size (preflight.check_plans);
  * each task's plan equals, message by message and key by key, the plan the Python host builds
    for the same partition from mpas_dycore.decomp (block-pair lists for one block per task,
    decomp.positional_lists for two).
"""
import os

import numpy as np
import pytest

from mpas_dycore import decomp
from mpas_dycore.dycore import plan_exchanges
from mpas_dycore.preflight import check_plans
from oracle import ref_runner

pytestmark = [
    pytest.mark.skipif(not ref_runner.available(ref_runner.DROPIN_PLAN_HARNESS),
                       reason="make -C oracle dropin_plan not run"),
    pytest.mark.skipif(not os.access(ref_runner.MPIRUN, os.X_OK), reason="no mpirun"),
]

DT_MSG = np.dtype([("point", "<i4"), ("direction", "<i4"), ("block", "<i4"), ("peer_rank", "<i4"),
                   ("peer_block", "<i4"), ("count", "<i8")], align=True)


@pytest.fixture(scope="module")
def mesh2562():
    from mpas_dycore.cases import jw_case
    return jw_case(2562, K=26, ns=1, cache=False)


def _plan_namelist(case, moist_end=1):
    c = case["config"]
    return dict(nVertLevels=case["nVertLevels"], maxEdges2=case["maxEdges2"], num_scalars=case["num_scalars"],
                moist_end=moist_end, dt=float(case["dt"]),
                config_time_integration_order=c["config_time_integration_order"],
                config_number_of_sub_steps=c["config_number_of_sub_steps"],
                config_dynamics_split_steps=c["config_dynamics_split_steps"],
                config_split_dynamics_transport=c["config_split_dynamics_transport"],
                config_scalar_advection=c["config_scalar_advection"], config_monotonic=c["config_monotonic"],
                config_positive_definite=c["config_positive_definite"])


def _as_plan(entry):
    _, msgs, keys = entry
    return np.array(msgs, dtype=[(n, DT_MSG.fields[n][0]) for n in DT_MSG.names]).astype(DT_MSG), keys


@pytest.fixture(scope="module")
def moist2562():
    from mpas_dycore.cases import jw_case
    return jw_case(2562, K=26, ns=6, moist=True, order=3, cache=False)


@pytest.mark.parametrize("ntask,nper,moist", [(2, 1, False), (4, 1, False), (2, 2, False), (4, 2, True)])
def test_dropin_multitask_plans(mesh2562, moist2562, ntask, nper, moist):
    """moist: num_scalars = 6, monotone split transport at order 3 (BASELINE configs[3]'s options)"""
    case = moist2562 if moist else mesh2562
    cell_part = decomp.partition_sfc(case["nCells"], ntask * nper)
    res = ref_runner.run_dropin_plan(case, cell_part, ntask, _plan_namelist(case))
    plans = res["plans"]
    assert sorted(plans) == list(range(ntask))
    # the id broadcast: every task holds task 0's words
    ids = {plans[t][0] for t in plans}
    assert len(ids) == 1 and ids.pop() != 0
    got = [_as_plan(plans[t]) for t in range(ntask)]
    summary = check_plans(got)
    assert summary["messages"] > 0 and summary["plan_keys"] > 40
    # the Python host's plan of the same partition, as Dycore.from_blocks installs it
    for t in range(ntask):
        if nper == 1:
            placement = {p: (p, 0) for p in range(ntask)}
            blocks = decomp.decompose(case, cell_part, parts=[t], placement=placement)
            want = plan_exchanges(blocks, placement, t, ntask, float(case["dt"]))
        else:
            blocks, placement = decomp.rank_blocks(case, ntask, t, nper, cell_part=cell_part)
            # mpas_block_decomp deals blocks to tasks in contiguous runs: the drop-in's local block order
            assert [b.part for b in blocks] == list(range(t * nper, (t + 1) * nper))
            want = plan_exchanges(blocks, placement, t, ntask, float(case["dt"]), positional=True)
        msgs, keys = got[t]
        assert keys == want[1], f"task {t}: plan keys differ"
        assert len(msgs) == len(want[0]), f"task {t}: {len(msgs)} messages, the host plans {len(want[0])}"
        for n in DT_MSG.names:
            assert np.array_equal(msgs[n], want[0][n]), f"task {t}: message field {n} differs"
        if nper > 1:  # positional: one message per peer task, filled by all blocks of the task
            assert (msgs["block"] == -1).all()
