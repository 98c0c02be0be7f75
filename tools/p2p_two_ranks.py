#!/usr/bin/env python3
"""Two ranks on ONE GPU, each stepping its block of a 2-way split, exchanging every halo through the
library's one-sided transfer with the host's all-gather (gloo, mpas_dyc_comm_init_host) -- no RCCL:
the multi-process path of the transfer end to end (the set-up records of real peers, IPC mappings of
the peer's fields and flag arena, ready / consumed across processes, pull exchanges).  Rank 0 then
steps the whole mesh as one block and compares every rank's owned values with it, bit for bit.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \\
        tools/p2p_two_ranks.py [--ncells 2562] [--levels 26] [--steps 3] [--moist] [--pull 0|1]

Prints one JSON line (rank 0) and exits non-zero on a difference.  Timing only in the sense of a
smoke test: the two ranks share one GPU.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpas-model_amd"))

FIELDS = [("state", "u", "edge"), ("state", "theta_m", "cell"), ("state", "rho_zz", "cell"),
          ("state", "w", "cell"), ("state", "scalars", "cell")]


def run(dy, dt, steps, graph=True):
    dy.init_diagnostics(dt)
    dy.use_graph(graph)
    for it in range(steps):
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
    dy.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ncells", type=int, default=2562)
    ap.add_argument("--levels", type=int, default=26)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--moist", action="store_true")
    ap.add_argument("--graph", type=int, default=1, help="0: launch the kernels one by one (no hipGraph)")
    ap.add_argument("--pull", type=int, default=1, help="0: send / receive buffers (MPAS_DYCORE_P2P_PULL=0)")
    a = ap.parse_args()
    os.environ["MPAS_DYCORE_P2P_PULL"] = str(a.pull)
    import numpy as np
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from mpas_dycore import Dycore, decomp
    from mpas_dycore.cases import jw_case
    case = jw_case(a.ncells, K=a.levels, ns=3 if a.moist else 1, moist=a.moist, order=3, cache=False)
    dt = float(case["dt"])
    part = decomp.partition_sfc(case["nCells"], world)
    placement = {p: (p, 0) for p in range(world)}
    blocks = decomp.decompose(case, part, parts=[rank], placement=placement)
    dy = Dycore.from_blocks(blocks, device=0, placement=placement, rank=rank, nranks=world,
                            host_group=dist.group.WORLD)
    run(dy, dt, a.steps, bool(a.graph))
    active = dy.p2p_active()
    mine = {n: dy.get(p, n, 1) for p, n, _ in FIELDS}
    dy.close()
    allv = [None] * world
    dist.all_gather_object(allv, mine)
    ok = True
    out = {"ranks": world, "ncells": case["nCells"], "levels": case["nVertLevels"], "steps": a.steps,
           "moist": a.moist, "pull": a.pull, "p2p_active": active}
    if rank == 0:
        one = Dycore(case, device=0)
        run(one, dt, a.steps)
        ref = {n: one.get(p, n, 1) for p, n, _ in FIELDS}
        one.close()
        allb = decomp.decompose(case, part, placement=placement)
        n_glob = {"cell": case["nCells"], "edge": case["nEdges"]}
        diffs, where = {}, {}
        for p, n, loc in FIELDS:
            got = decomp.gather_owned(allb, [allv[r][n] for r in range(world)], loc, n_glob[loc])
            same = bool(np.array_equal(got, ref[n]))
            diffs[n] = 0.0 if same else float(np.nanmax(np.abs(got - ref[n])))
            if not same:  # where it differs: which side holds non-finite values, how many columns
                bad = np.atleast_2d(got != ref[n])
                where[n] = {"nonfinite_split": int((~np.isfinite(got)).sum()),
                            "nonfinite_one": int((~np.isfinite(ref[n])).sum()),
                            "columns": int(bad.any(axis=tuple(range(1, bad.ndim))).sum()) if bad.ndim > 1 else int(bad.sum())}
            ok = ok and same
        out.update(bitwise=ok, max_abs_diff=diffs)
        if where:
            out["where"] = where
        print(json.dumps(out), flush=True)
    flag = [ok and active]
    dist.broadcast_object_list(flag, src=0)
    dist.destroy_process_group()
    return 0 if flag[0] else 1


if __name__ == "__main__":
    sys.exit(main())
