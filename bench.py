#!/usr/bin/env python3
"""Benchmark: MPAS-Atmosphere dycore cell-updates/s on MI355X (BASELINE.json metric).

One "step" = one full atm_timestep / atm_srk3 (dt) of the split-explicit dycore
(3 dynamics substeps x RK3 x acoustic substeps + split scalar transport with the
monotone limiter) on a synthetic x1.163842 JW baroclinic-wave state, 56 levels,
fp64.  value = nCells * nVertLevels / t_dt (cell-updates per second of the whole mesh;
N GPUs split the mesh into N blocks with halos -- strong scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Also reported:
  roofline      acoustic sub-step (atm_advance_acoustic_step + atm_divergence_damping_3d),
                algorithmic bytes B_ac / measured time (HIP events on the
                dycore's stream) vs the 8 TB/s HBM peak
  cpu_baseline  the reference Fortran dycore (oracle/_ref, compiled from /root/reference)
                on the host cores, bounded sample
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpas-model_amd"))
sys.path.insert(0, ROOT)

METRIC = "dycore cell-updates/sec (nCells×nVertLevels/step) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured copy


def _dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def cpu_baseline(case, dt, nthreads, steps, moist_end=1):
    """Reference dycore (compiled Fortran) timed on host cores -- the cpu_baseline leg only."""
    from oracle import ref_runner
    if not ref_runner.available():
        return None
    _, times = ref_runner.run_reference(case, nsteps=steps, dt=dt, dump_steps=[], nthreads=nthreads, timeout=1200,
                                        moist_end=moist_end)
    use = times[1:] if len(times) > 1 else times  # first step pays allocation / first-touch
    t = sum(use) / len(use)
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    value = case["nCells"] * case["nVertLevels"] / t
    # the whole host as context: the pool's rules give one GPU's job 16 host threads (OMP_NUM_THREADS on
    # the box), so the reference is not run on every core of the shared host; at ideal (linear) OpenMP
    # scaling over `affinity` cores it could reach at most this
    whole = None
    if affinity and affinity > nthreads:
        whole = dict(value=value * affinity / nthreads, cores=affinity, kind="upper bound, linear scaling of the "
                     f"{nthreads}-thread measurement (not run: the box's CPU share is {nthreads} threads)")
    return dict(value=value, unit="cell-updates/s", cores=nthreads, whole_host=whole,
                kind="reference", cpu_model=_cpu_model(), host_nproc=os.cpu_count(), affinity=affinity,
                omp_num_threads=os.environ.get("OMP_NUM_THREADS"),
                cores_note="threads = the host-CPU share the GPU pool gives one GPU (OMP_NUM_THREADS on the box); "
                           "host_nproc counts the whole machine, shared by its 8 GPUs",
                sample=f"unmodified reference atm_srk3 (amdflang -O2, OpenMP {nthreads} threads) on the same "
                       f"{case['nCells']}-cell x {case['nVertLevels']} JW case: {steps} dt steps, mean of the "
                       f"{len(use)} timed steps 2..{steps} ({t:.2f} s/step)")


class Watchdog:
    """Bounds every phase of a multi-rank run: a phase that does not finish in time (ncclCommInitRank,
    a halo exchange's RCCL group, a captured step) makes this rank print one JSON line naming the
    phase and the library's last enqueued exchange (mpas_dyc_last_exchange) and exit with status 3
    (os._exit from this thread: the main thread may be blocked inside RCCL; nothing is re-executed)."""

    def __init__(self, rank: int, enabled: bool):
        import threading
        self.rank, self.enabled = rank, enabled
        self.name, self.deadline, self.t0 = None, None, time.time()
        self.dy = None
        self.lock = threading.Lock()
        if enabled:
            threading.Thread(target=self._run, daemon=True).start()

    def phase(self, name: str, seconds: float):
        with self.lock:
            self.name, self.deadline, self.t0 = name, time.time() + seconds, time.time()

    def done(self):
        with self.lock:
            self.name, self.deadline = None, None

    def _run(self):
        while True:
            time.sleep(1.0)
            with self.lock:
                expired = self.deadline is not None and time.time() > self.deadline
                name, t0 = self.name, self.t0
            if expired:
                last = ""
                try:
                    last = self.dy.last_exchange() if self.dy is not None else ""
                except Exception:
                    pass
                msg = {"metric": METRIC, "value": None, "error": f"rank {self.rank}: phase '{name}' did not finish "
                       f"within {time.time() - t0:.0f} s", "rank": self.rank, "phase": name, "last_exchange": last}
                print(json.dumps(msg), flush=True)
                print(json.dumps(msg), file=sys.stderr, flush=True)
                os._exit(3)


def agree_on_failure(dist, world, err):
    """Every rank's warm-up outcome over the host group (gloo): the first failing rank's message on
    every rank, or None when all succeeded -- the ranks then drop the one-sided transfer together."""
    errs = [None] * world
    dist.all_gather_object(errs, err or "")
    bad = [e for e in errs if e]
    return bad[0] if bad else None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def small_mesh_line(args, torch, device, ncells=10242, steps=20, warmup=3):
    from mpas_dycore import Dycore
    from mpas_dycore.cases import jw_case
    ns = 6 if args.moist else 1
    case = jw_case(ncells, K=args.levels, ns=ns, moist=args.moist, order=args.order)
    dt = case["dt"]
    dy = Dycore(case, device=device, moist_end=ns if args.moist else 1)
    dy.init_diagnostics(dt)
    if not args.no_graph:
        dy.use_graph(True)
    for i in range(warmup):
        dy.atm_timestep(dt, i + 1)
        dy.shift_time_levels()
    dy.synchronize()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(steps):
        dy.atm_timestep(dt, warmup + i + 1)
        dy.shift_time_levels()
    dy.synchronize()
    torch.cuda.synchronize(device)
    ms = (time.perf_counter() - t0) / steps * 1e3
    nss = case["config"]["config_number_of_sub_steps"]
    dts = dt / case["config"]["config_dynamics_split_steps"] / nss
    _, ms_k = dy.time_acoustic_step(dts, small_step=2, reps=args.acoustic_reps)
    b_ac = dy.acoustic_bytes()
    dy.close()
    achieved = b_ac / (sum(ms_k) / 1e3) / 1e9
    return {"workload": f"x1.{ncells} {'moist (num_scalars=6)' if args.moist else 'dry'} dycore, "
                        f"{case['nVertLevels']} levels, dt={dt:g}s, 1 GPU (BASELINE.json configs[1])",
            "value": case["nCells"] * case["nVertLevels"] / (ms / 1e3), "unit": "cell-updates/s",
            "ms_per_step": ms, "steps": steps, "warmup": warmup,
            "acoustic_roofline": {"achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": achieved / HBM_PEAK_GBS, "ms_per_substep": sum(ms_k)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--ncells", type=int, default=163842)
    ap.add_argument("--levels", type=int, default=56)
    ap.add_argument("--num-scalars", type=int, default=None)
    ap.add_argument("--varres", type=int, default=0, metavar="NCELLS",
                    help="BASELINE.json configs[4]: variable-resolution SCVT (20x refinement) with NCELLS cells, "
                         "e.g. 835586")
    ap.add_argument("--init", default=None, metavar="FILE",
                    help="start from an MPAS init file (x1.N.init.nc, netCDF CDF-1/2/5) instead of the synthetic "
                         "JW case; needs --dt and --len-disp (namelist config_dt / config_len_disp)")
    ap.add_argument("--dt", type=float, default=None)
    ap.add_argument("--len-disp", type=float, default=None)
    ap.add_argument("--max-edges", default=None, metavar="ME[,ME2]",
                    help="declare the mesh with maxEdges ME and maxEdges2 ME2 (default 2 ME), as MPAS mesh files "
                         "do (10,20): the unused slots are padding the kernels never read")
    ap.add_argument("--moist", action="store_true",
                    help="BASELINE.json configs[3]: moist JW (qv) + tracer blobs, num_scalars=6, monotone transport")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=4, help="reference steps; the first is untimed")
    ap.add_argument("--order", type=int, default=3, choices=(2, 3),
                    help="config_time_integration_order of the synthetic cases (SURVEY.md §8d: 3)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: OMP_NUM_THREADS (the box's share), else 16")
    ap.add_argument("--acoustic-reps", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=1, help="blocks per GPU (MPAS blocks with halos)")
    ap.add_argument("--rccl-local", action="store_true", help="route in-process block exchanges through RCCL")
    ap.add_argument("--same-device", action="store_true",
                    help="test: every rank on GPU 0, no RCCL (the host's all-gather over gloo, one-sided "
                         "transfer between the processes) -- exercises the multi-rank path on a one-GPU box")
    ap.add_argument("--transport", choices=("rccl", "p2p"), default="p2p",
                    help="halo messages between ranks: RCCL send/recv groups, or the one-sided intra-node "
                         "transfer (mpas_dyc_set_p2p: pulled over xGMI by the receiving rank's kernel)")
    ap.add_argument("--no-configs1", action="store_true",
                    help="skip the secondary x1.10242 (BASELINE.json configs[1]) measurement")
    ap.add_argument("--preflight-only", action="store_true",
                    help="multi-rank: check on the host that every rank's RCCL plans pair up, print the result "
                         "and exit before touching a GPU")
    ap.add_argument("--phase-timeout", type=float, default=600.0,
                    help="multi-rank watchdog: seconds any one phase (RCCL init, model init, first step with its "
                         "capture, warmup, profile) may take; the timed loop gets this plus 10 s per step")
    args = ap.parse_args()

    world, rank, local = _dist()
    import torch
    dist = None
    if world > 1:
        # gloo for the host-side rendezvous, barriers and the max-over-ranks timing; the halo
        # exchanges of the dycore itself run over the library's own RCCL communicator
        import torch.distributed as dist
        dist.init_process_group("gloo")
    device = 0 if args.same_device else local

    from mpas_dycore import Dycore, decomp
    from mpas_dycore.cases import jw_case

    # rank 0 builds (and caches) the synthetic case before any rank touches the GPU
    if args.num_scalars is None:
        args.num_scalars = 6 if args.moist else 1
    def make_case():
        c = _make_case()
        if args.max_edges:
            from mpas_dycore.mesh import pad_max_edges
            me = [int(x) for x in str(args.max_edges).split(",")]
            c = pad_max_edges(c, me[0], me[1] if len(me) > 1 else 2 * me[0])
        return c

    def _make_case():
        if args.init:
            from mpas_dycore.mpas_files import read_init
            if args.dt is None or args.len_disp is None:
                raise SystemExit("--init needs --dt and --len-disp")
            return read_init(args.init, config=dict(config_dt=args.dt, config_len_disp=args.len_disp,
                                                    config_time_integration_order=args.order))
        if args.varres:
            from mpas_dycore.cases import varres_case
            return varres_case(args.varres, ratio=20.0, K=args.levels, ns=args.num_scalars, moist=args.moist,
                               order=args.order)
        return jw_case(args.ncells, K=args.levels, ns=args.num_scalars, moist=args.moist, order=args.order)

    t_build = time.time()
    if rank == 0:
        case = make_case()
    if dist:
        dist.barrier()
    if rank != 0:
        case = make_case()
    dt = case["dt"]
    t_build = time.time() - t_build

    # WSM6-like species set: every scalar is a moist species (moist_start..moist_end, qtot)
    moist_end = case["num_scalars"] if (args.moist or args.init) else 1
    nparts = world * args.blocks
    wd = Watchdog(rank, world > 1)
    preflight = None
    if nparts > 1:
        blocks, placement = decomp.rank_blocks(case, world, rank, args.blocks)
        if world > 1 or args.preflight_only:
            # every rank's RCCL plans, checked against each other on the host before any GPU call
            from mpas_dycore.dycore import plan_exchanges
            from mpas_dycore.preflight import PlanMismatch, check_plans
            wd.phase("preflight", args.phase_timeout)
            mine = plan_exchanges(blocks, placement, rank, world, float(dt), moist_end=moist_end)
            allp = [None] * world
            if dist:
                dist.all_gather_object(allp, mine)
            else:
                allp = [mine]
            try:
                preflight = dict(check_plans(allp), ok=True)
            except PlanMismatch as e:
                preflight = {"ok": False, "error": str(e), "point": e.point, "key": e.key}
            wd.done()
            if not preflight["ok"] or args.preflight_only:
                if rank == 0:
                    print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world, "preflight": preflight,
                                      "rccl_version": Dycore.rccl_version()}), flush=True)
                if dist:
                    dist.destroy_process_group()
                raise SystemExit(0 if preflight["ok"] else 2)
        # --rccl-local: blocks of this process also exchange through RCCL (send to self), to
        # measure the cost of the RCCL path on one GPU
        if args.same_device and (args.transport != "p2p" or args.rccl_local):
            raise SystemExit("--same-device needs --transport p2p and no --rccl-local")
        torch.cuda.set_device(device)

        def build(transport):
            comm_id = None
            if not args.same_device and (world > 1 or args.rccl_local):
                obj = [Dycore.comm_unique_id() if rank == 0 else None]
                if dist:
                    dist.broadcast_object_list(obj, src=0)
                comm_id = obj[0]
            wd.phase("rccl_init (ncclCommInitRank) and upload", args.phase_timeout)
            return Dycore.from_blocks(blocks, device=device, placement=placement, rank=rank, nranks=world,
                                      comm_id=comm_id, moist_end=moist_end, rccl_local=args.rccl_local,
                                      p2p=transport == "p2p",
                                      host_group=dist.group.WORLD if (args.same_device and dist) else None)
        dy = build(args.transport)
        owned = sum(b.solve[0] for b in blocks)
        halo = sum(b.case["nCells"] - b.solve[0] for b in blocks)
    else:
        dy = Dycore(case, device=device, moist_end=moist_end)
        owned, halo = case["nCells"], 0

    def step(i):
        dy.atm_timestep(dt, i)
        dy.shift_time_levels()

    def warm_up():
        wd.dy = dy
        wd.phase("model init (init_diagnostics)", args.phase_timeout)
        dy.init_diagnostics(dt)
        dy.synchronize()
        if not args.no_graph:
            dy.use_graph(True)
        for i in range(args.warmup):
            wd.phase(f"warmup step {i + 1}" + (" (exchange plans, RCCL warm-up, hipGraph capture)" if i == 0 else ""),
                     args.phase_timeout)
            step(i + 1)
            dy.synchronize()

    # the one-sided transfer's first run between separate GPUs may be the driver's: if any rank's
    # warm-up fails with it (a wait that timed out, a refused mapping at run time), every rank drops
    # it together and runs again over RCCL, and the line says so (config.transport_fallback)
    fallback = None
    if nparts > 1 and world > 1 and args.transport == "p2p" and not args.same_device:
        err = ""
        try:
            warm_up()
        except Exception as e:  # noqa: BLE001 -- any failure: decided collectively below
            err = f"rank {rank}: {str(e)[:300]}"
        first = agree_on_failure(dist, world, err)
        if first:
            fallback = {"from": "p2p", "to": "rccl", "error": first}
            wd.done()
            try:
                dy.close()
            except Exception:  # noqa: BLE001
                pass
            dy = build("rccl")
            warm_up()
    else:
        warm_up()
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    wd.phase("timed loop", args.phase_timeout + 10.0 * args.steps)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i + 1)
    dy.synchronize()
    torch.cuda.synchronize(device)
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    wd.done()
    elapsed = t1 - t0
    graph = dy.graph_active()
    layout = dy.layout()
    transport = ("one-sided over xGMI (IPC)" if dy.p2p_active() else "RCCL send/recv groups") if nparts > 1 else None
    ranks = None
    if nparts > 1:
        # one more step, eager, with HIP events around every exchange's exposed part (outside the
        # timed region): where this rank's time goes
        wd.phase("exchange profile step", args.phase_timeout)
        prof = dict(dy.exchange_profile(dt, args.warmup + args.steps + 1), rank=rank, owned_cells=int(owned),
                    halo_cells=int(halo))
        dy.shift_time_levels()
        wd.done()
        ranks = [None] * world
        if dist:
            dist.all_gather_object(ranks, prof)
        else:
            ranks = [prof]
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # every rank replays its captured step, or none does (the library refuses a per-rank
        # eager fallback with more than one rank; this checks the outcome)
        g = torch.tensor([int(graph), -int(graph)], dtype=torch.int64)
        dist.all_reduce(g, op=dist.ReduceOp.MAX)
        if int(g[0]) != -int(g[1]):
            raise SystemExit("hipGraph replay differs between ranks")
    ms_per_step = elapsed / args.steps * 1e3
    # strong scaling: the whole x1.N mesh is advanced once per step, whatever the rank count
    value = case["nCells"] * case["nVertLevels"] / (ms_per_step / 1e3)

    # ---- roofline of the acoustic sub-step (graded kernel), measured with HIP events
    nss = case["config"]["config_number_of_sub_steps"]
    dts = dt / case["config"]["config_dynamics_split_steps"] / nss
    ms_sub, ms_k = dy.time_acoustic_step(dts, small_step=2, reps=args.acoustic_reps)
    b_ac = dy.acoustic_bytes()
    t_kern = sum(ms_k) / 1e3
    achieved = b_ac / t_kern / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "acoustic_traffic.json")
    if os.path.isfile(tf) and nparts == 1:  # the PMC figures are for the whole mesh as one block
        try:
            with open(tf) as f:
                tj = json.load(f)
            if tj.get("ncells") == case["nCells"] and tj.get("levels") == case["nVertLevels"]:
                traffic = tj.get("bytes_per_substep")
        except Exception:
            traffic = None

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "cell-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": (f"MPAS init file {args.init}" if args.init else
                 "synthetic (icosahedral SCVT mesh + Jablonowski-Williamson baroclinic wave, built on the box)"),
        "config": {
            "workload": (f"MPAS init file {os.path.basename(args.init)}: {case['nCells']} cells, "
                         f"{case['nVertLevels']} levels, {case['num_scalars']} scalars, dt={dt:g}s "
                         f"(one full atm_srk3 per step)" if args.init else
                         f"variable-resolution SCVT, {case['nCells']} cells (20x refinement, "
                         f"{case['dcEdge'].min() / 1e3:.1f}-{case['dcEdge'].max() / 1e3:.0f} km, maxEdges="
                         f"{case['maxEdges']}, {int((case['nEdgesOnCell'] == 5).sum())} pentagons / "
                         f"{int((case['nEdgesOnCell'] == 7).sum())} heptagons), {case['nVertLevels']} levels, "
                         f"dt={dt:g}s (BASELINE.json configs[4]; one full atm_srk3 per step)" if args.varres else
                         f"x1.{case['nCells']} moist dycore + scalar transport (num_scalars={case['num_scalars']}, "
                         f"monotone), {case['nVertLevels']} levels, dt={dt:g}s (BASELINE.json configs[3]; one full "
                         f"atm_srk3 per step)" if args.moist else
                         f"x1.{case['nCells']} dry dycore, {case['nVertLevels']} levels, dt={dt:g}s "
                         f"(BASELINE.json configs[2] mesh; one full atm_srk3 per step)"),
            "nCells": case["nCells"], "nVertLevels": case["nVertLevels"], "num_scalars": case["num_scalars"],
            "dt": dt, "time_integration_order": case["config"]["config_time_integration_order"],
            "split_steps": case["config"]["config_dynamics_split_steps"], "acoustic_substeps": nss,
            "parallelism": (f"domain decomposition: {nparts} SFC blocks with 2-layer halos, "
                            f"{args.blocks} per GPU, halo exchange {transport}" if nparts > 1 else "single block"),
            "owned_cells_rank0": owned, "halo_cells_rank0": halo,
            "hip_graph": graph,
            "transport_fallback": fallback,
            "maxEdges_declared": [case["maxEdges"], case["maxEdges2"]],
            "kernel_layout": layout,
        },
        "roofline": {
            "kernel": "acoustic sub-step (k_acoustic_edges<damped> + k_acoustic_cells; per sub-step of an "
                      "--acoustic-reps loop as srk3 runs it, plus that loop's final k_divdamp)",
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "bytes_per_launch": b_ac, "ms_per_substep": sum(ms_k),
            "ms_kernels": {"edges": ms_k[0], "cells": ms_k[1], "final_divdamp_share": ms_k[2]},
        },
        "cpu_baseline": None,
    }
    if nparts > 1:
        out["ranks"] = ranks
        out["preflight"] = preflight
        out["rccl_version"] = Dycore.rccl_version()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            # the box's CPU share for one GPU (OMP_NUM_THREADS there), not the machine's nproc
            nthreads = min(args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(case, dt, nthreads, args.cpu_steps, moist_end)
        except Exception as e:  # the measured GPU number stands on its own
            out["cpu_baseline"] = {"error": str(e)[:200]}
    out["build_s"] = round(t_build, 1)
    dy.close()
    # BASELINE.json configs[1] (x1.10242 x 56 on one MI355X) alongside the headline mesh: the same
    # measurement on the small mesh (launch-bound), reported under "configs1"
    if world == 1 and not (args.init or args.varres or args.no_configs1) and args.ncells != 10242:
        out["configs1"] = small_mesh_line(args, torch, device)
    if dist:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
