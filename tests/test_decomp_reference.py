"""decomp.py's blocks and exchange lists driven through the REFERENCE dycore's own halo exchanges.

The harness's multi-block mode (oracle/harness/mpas_ref_harness.F90, nblocks > 1) builds one MPAS
block per decomp.py block in one process -- its pools from the block's local arrays, and
parinfo % cellsToCopy / edgesToCopy / verticesToCopy from the block's send and receive lists --
links the blocks' fields and exchange lists as mpas_block_creator leaves them
(mpas_pool_link_pools, mpas_pool_link_parinfo), runs the model-init exchanges of
mpas_atm_core.F:143-186, and steps the unmodified atm_srk3, whose every
mpas_dmpar_exch_halo_field then copies between the blocks through those lists
(mpas_dmpar.F:5480-5502).  If a list missed an element the reference reads, or listed one in a
different order on the two sides, the blocks would drift from the one-block run; they must agree
to the bit, owned elements and halo layer 1.

Limits of the reference itself, which is why this runs dry and with the largest block first:
  * atm_srk3 sizes its module scratch (qtot, tend_*_physics) from the first block of the list
    (mpas_atm_time_integration.F:268-279), so a larger later block would write past it;
  * qtot is one module array for all blocks: atm_compute_moist_coefficients fills it block by
    block, so every block but the last reads the last block's qtot -- with moisture the blocks
    of one process drift (zero for a dry run);
  * the monotone limiter exchanges scale_arr through a temporary field with no next block
    (4084-4098), which copies nothing between blocks of one process.
The GPU product has none of these (tests/test_gpu_decomp.py: moist monotone blocks bitwise).
"""
import numpy as np
import pytest

from conftest import rel_linf

NSTEPS = 3
FIELDS = [("state.u.tl1", "edge"), ("state.theta_m.tl1", "cell"), ("state.rho_zz.tl1", "cell"),
          ("state.w.tl1", "cell"), ("diag.pv_edge", "edge"), ("diag.rho_edge", "edge"), ("diag.exner", "cell"),
          ("diag.ru", "edge"), ("diag.rw", "cell"), ("diag.vorticity", "vertex"), ("diag.uReconstructZonal", "cell")]
_N = {"cell": "nCells", "edge": "nEdges", "vertex": "nVertices"}


@pytest.fixture(scope="module")
def dry2562():
    from mpas_dycore.cases import jw_case
    return jw_case(2562, K=26, ns=1, cache=False)


@pytest.fixture(scope="module")
def one_block(dry2562):
    from oracle import ref_runner
    if not ref_runner.available():
        pytest.skip("oracle/_ref not built")
    c = dry2562
    res, _ = ref_runner.run_reference(c, nsteps=NSTEPS, dt=c["dt"], dump_steps=[0, NSTEPS], nthreads=4)
    return res


@pytest.mark.parametrize("nblocks", [2, 4])
def test_reference_dycore_on_decomp_blocks_is_bitwise_one_block(dry2562, one_block, nblocks):
    from mpas_dycore import decomp
    from oracle import ref_runner
    c = dry2562
    blocks = decomp.decompose(c, decomp.partition_sfc(c["nCells"], nblocks))
    blocks.sort(key=lambda b: (-b.case["nCells"], -b.case["nEdges"]))  # the largest first (see above)
    assert all(b.case["nEdges"] <= blocks[0].case["nEdges"] for b in blocks)
    multi, _ = ref_runner.run_reference_blocks(c, blocks, nsteps=NSTEPS, dt=c["dt"], dump_steps=[0, NSTEPS],
                                               nthreads=4)
    for step in (0, NSTEPS):
        for key, loc in FIELDS:
            ref = one_block[step][key].reshape((c[_N[loc]], -1))
            for m, b in zip(multi[step], blocks):
                a = m[key].reshape((b.case[_N[loc]], -1))
                # owned + halo layer 1 (mpas_reconstruct fills owned cells only)
                n1 = b.layer_end[loc][0 if "Reconstruct" in key else 1]
                got, want = a[:n1], ref[b.glob[loc][:n1]]
                assert np.array_equal(got, want), (
                    f"step {step}, {key}, block {b.part}: rel Linf {rel_linf(got, want):.3e}")
