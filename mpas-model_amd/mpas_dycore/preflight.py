"""Checks a multi-rank run makes on the host before any rank touches its GPU.

Every rank plans its RCCL messages with the library's own planner in a host-only context
(mpas_dyc_plan_exchanges: the model-init exchanges and one atm_srk3 on each time-level parity).
ncclGroupStart / ncclGroupEnd pair rank r's k-th ncclSend to rank p with rank p's k-th ncclRecv
from r, as the reference's MPI_Isend / MPI_Irecv pairs do (mpas_dmpar.F:5386-5552); a mismatch
would hang both ranks inside the captured step.  `check_plans` proves the plans of all ranks pair
up: same exchange calls in the same order, and at every call equal message lists both ways.
"""
from __future__ import annotations

import numpy as np

from . import _lib


class PlanMismatch(RuntimeError):
    def __init__(self, msg: str, point: int = -1, key: str = ""):
        super().__init__(msg)
        self.point, self.key = point, key


def check_plans(plans: list) -> dict:
    """plans[r] = (messages, keys) of rank r (dycore.plan_exchanges).  Returns {"plan_keys": calls
    per run, "messages": RCCL messages over all ranks}; raises PlanMismatch at the first call whose
    sends and receives do not pair."""
    nranks = len(plans)
    keys0 = plans[0][1]
    for r in range(nranks):
        if plans[r][1] != keys0:
            i = next((j for j, (a, b) in enumerate(zip(plans[r][1], keys0)) if a != b),
                     min(len(plans[r][1]), len(keys0)))
            raise PlanMismatch(f"rank {r} issues a different exchange sequence from rank 0 at call {i}", i,
                               keys0[i] if i < len(keys0) else "")
    nmsg = 0
    for r in range(nranks):
        sends = plans[r][0][plans[r][0]["direction"] == _lib.SEND]
        for p in range(nranks):
            recvs = plans[p][0][plans[p][0]["direction"] == _lib.RECV]
            for i in range(len(keys0)):
                s = sends[(sends["point"] == i) & (sends["peer_rank"] == p)]
                v = recvs[(recvs["point"] == i) & (recvs["peer_rank"] == r)]
                ok = (len(s) == len(v) and np.array_equal(s["count"], v["count"])
                      and np.array_equal(s["peer_block"], v["block"]) and np.array_equal(s["block"], v["peer_block"]))
                if not ok:
                    raise PlanMismatch(f"call {i}: rank {r} posts {len(s)} sends {list(s['count'])} to rank {p}, "
                                       f"which posts {len(v)} receives {list(v['count'])}", i, keys0[i])
                nmsg += len(s)
    return {"plan_keys": len(keys0), "messages": nmsg}
