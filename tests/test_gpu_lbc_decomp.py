"""GPU: a regional run (config_apply_lbcs) decomposed into blocks reproduces the one-block run bit for bit.

The reference cannot be the oracle here: its boundary getters (mpas_atm_boundaries.F:268, 337) are
handed `domain % blocklist`, the first block of a task, by every caller in atm_srk3, so several
blocks per task are not a configuration it runs -- one block per MPI task is, and that is what the
blocks of this test stand for.  The limited-area case is test_gpu_lbc's (cases.regional_lbc) with
the boundary zone confined to rows 1..7 (interior_deg = 150: no cell lies beyond row 7 on
x1.2562), and nearestRelaxationCell recomputed as mpas_atm_setup_bdy_masks does (:466-518: the
nearest mask-5 cell among the neighbours, for row 7 through a row-6 neighbour), so every index it
holds lies within two cells and therefore inside each block's halo.  8 SFC blocks, 4 of which own
boundary-zone cells; the lbc pool of each block is the global driving data at its local elements.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = [("state", "u", "edge"), ("state", "theta_m", "cell"), ("state", "rho_zz", "cell"),
          ("state", "w", "cell"), ("state", "scalars", "cell")]
NSTEPS = 3


def _reference_nearest(case):
    """nearestRelaxationCell as mpas_atm_setup_bdy_masks computes it (0-based, -1 = none)."""
    mask = np.asarray(case["bdyMaskCell"])
    coc, noc = np.asarray(case["cellsOnCell"]), np.asarray(case["nEdgesOnCell"])
    xyz = np.stack([np.asarray(case["xCell"]), np.asarray(case["yCell"]), np.asarray(case["zCell"])], 1)
    near = np.full(case["nCells"], -1, dtype=np.int64)
    for c in np.flatnonzero(mask == 6):
        best = 1.0e36
        for i in coc[c, :noc[c]]:
            if mask[i] == 5:
                d = ((xyz[i] - xyz[c]) ** 2).sum()
                if d < best:
                    best, near[c] = d, i
    for c in np.flatnonzero(mask == 7):
        best = 1.0e36
        for i in coc[c, :noc[c]]:
            if mask[i] != 6:
                continue
            for ii in coc[i, :noc[i]]:
                if mask[ii] == 5:
                    d = ((xyz[ii] - xyz[c]) ** 2).sum()
                    if d < best:
                        best, near[c] = d, ii
    return near


def _case(moist, K=26):
    from mpas_dycore.cases import jw_case, regional_lbc
    case = jw_case(2562, K=K, ns=6 if moist else 1, moist=moist, cache=False)
    case, lbc = regional_lbc(case, interior_deg=150.0)
    assert (np.asarray(case["bdyMaskCell"]) == 7).sum() > 0
    case["nearestRelaxationCell"] = _reference_nearest(case)
    return case, lbc


def _run(dy, case, lbc, set_lbc_pool):
    dt = float(case["dt"])
    set_lbc_pool(dy)
    dy.init_diagnostics(dt)
    for it in range(NSTEPS):
        dy.set_lbc(True, lbc["interval_end"] - it * dt)
        dy.atm_timestep(dt, it + 1)
        dy.shift_time_levels()
    dy.synchronize()


@pytest.mark.parametrize("moist,rccl,K", [(False, False, 26), (True, False, 26), (True, True, 26), (True, True, 80)])
def test_regional_blocks_bitwise_equal_single_block(moist, rccl, K):
    """rccl: the blocks exchange through RCCL (send to self) with split-phase exchanges and graph
    replay, as ranks of a multi-GPU run do.  K = 80: the wide build (one column per wavefront in the
    pair-layout kernels)."""
    from mpas_dycore import Dycore, decomp
    from oracle import ref_runner
    case, lbc = _case(moist, K)
    me = 6 if moist else 1
    images = ref_runner.lbc_images(case, lbc)  # element-major, garbage row last

    one = Dycore(case, device=0, moist_end=me)

    def pool_one(dy):
        for (name, tl), img in images.items():
            dy.set_raw("lbc", name, img, tl)
    _run(one, case, lbc, pool_one)
    ref = {n: one.get(p, n, 1) for p, n, _ in FIELDS}
    one.close()

    blocks = decomp.decompose(case, decomp.partition_sfc(case["nCells"], 8))
    comm_id = Dycore.comm_unique_id() if rccl else None
    dy = Dycore.from_blocks(blocks, device=0, moist_end=me, comm_id=comm_id, nranks=1, rank=0, rccl_local=rccl)
    dy.use_graph(rccl)

    def pool_blocks(d):
        for i, b in enumerate(blocks):
            for (name, tl), img in images.items():
                loc = "edge" if name in ("lbc_u", "lbc_ru") else "cell"
                local = np.zeros((b.glob[loc].size + 1,) + img.shape[1:])
                local[:-1] = img[:-1][b.glob[loc]]
                d.set_raw("lbc", name, local, tl, block=i)
    _run(dy, case, lbc, pool_blocks)
    n_glob = {"cell": case["nCells"], "edge": case["nEdges"]}
    for p, n, loc in FIELDS:
        per = [dy.get(p, n, 1, block=i) for i in range(len(blocks))]
        got = decomp.gather_owned(blocks, per, loc, n_glob[loc])
        assert np.array_equal(got, ref[n]), f"{n}: max diff {np.nanmax(np.abs(got - ref[n]))}"
    dy.close()
