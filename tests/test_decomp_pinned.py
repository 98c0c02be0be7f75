"""CPU: mpas_dycore.decomp pinned to the reference's own decomposition code.

oracle/_ref/decomp_harness runs the unmodified framework/mpas_block_decomp.F (cells per block from a
graph.info.part.N file) and mpas_block_creator.F's halo builder (setup_blocks_and_0halo_cells ..
build_edge_halos, the calls of mpas_bootstrapping.F:171-269) on the case's mesh and partition.  For
every block and location (cells, edges, vertices) decomp.py must give, bit for bit:
  * the local element order -- owned elements, then each halo layer -- as global indices
    (indexToCellID / indexToEdgeID / indexToVertexID of the block);
  * the end of the owned range and of every halo layer (the nCellsSolve / nEdgesSolve /
    nVerticesSolve fields, mpas_block_creator.F:470-716, 734-938);
  * the exchange lists:
    - one task, several blocks: copyList node (endPointID = receiving block, srcList here, destList
      there) == decomp's send list of this block and receive list of that block, in order;
    - one block per task (mpirun): sendList / recvList nodes, whose other list holds buffer
      positions; sorted by position they are decomp's send / receive lists (the message order the
      drop-in hands to the library, atm_time_integration_mi355x.F90 set_block_lists).
"""
import os

import numpy as np
import pytest

from oracle import ref_runner

pytestmark = pytest.mark.skipif(not ref_runner.available(ref_runner.DECOMP_HARNESS),
                                reason="make -C oracle decomp not run")

LOCS = ("cell", "edge", "vertex")


@pytest.fixture(scope="module")
def mesh2562():
    from mpas_dycore.cases import jw_case
    return jw_case(2562, K=4, ns=1, cache=False)


@pytest.fixture(scope="module")
def varres():
    from mpas_dycore.cases import varres_case
    return varres_case(2562, ratio=4.0, K=4, ns=1, cache=False)


def _lists(block, kind, loc, layer):
    out = {}
    for (l, y, peer, idx) in (block.send if kind == "send" else block.recv):
        if l == loc and y == layer:
            out[peer] = np.asarray(idx, dtype=np.int64)
    return out


def _check(case, part, nprocs):
    from mpas_dycore import decomp
    ref = ref_runner.run_reference_decomp(case, part, nprocs=nprocs)
    nb = int(np.max(part)) + 1
    placement = {p: (0 if nprocs == 1 else p, p if nprocs == 1 else 0) for p in range(nb)}
    blocks = decomp.decompose(case, part, placement=placement)
    by_part = {b.part: b for b in blocks}
    assert sorted(ref) == sorted(by_part)
    nlists = 0
    for bid, r in ref.items():
        b = by_part[bid]
        for loc in LOCS:
            assert np.array_equal(np.asarray(b.glob[loc]), r[f"{loc}_index"]), f"block {bid} {loc}: local order"
            assert list(b.layer_end[loc]) == r[f"{loc}_solve"].tolist(), f"block {bid} {loc}: halo layer ends"
            for layer in range(1, len(b.layer_end[loc])):
                send, recv = _lists(b, "send", loc, layer), _lists(b, "recv", loc, layer)
                if nprocs == 1:
                    # copyList: this block's owned srcList -> halo destList of block endPointID
                    for ep, src, dst in r[f"{loc}_copy_{layer}"]:
                        assert np.array_equal(send[ep], src - 1), f"{loc} layer {layer}: {bid}->{ep} send list"
                        assert np.array_equal(_lists(by_part[ep], "recv", loc, layer)[bid], dst - 1), (
                            f"{loc} layer {layer}: {bid}->{ep} receive list")
                        nlists += 1
                    assert len(r[f"{loc}_copy_{layer}"]) == len(send)
                else:
                    for ep, src, pos in r[f"{loc}_send_{layer}"]:
                        assert np.array_equal(send[ep], src[np.argsort(pos, kind="stable")] - 1), (
                            f"{loc} layer {layer}: {bid}->{ep} send list (buffer order)")
                        nlists += 1
                    for ep, pos, dst in r[f"{loc}_recv_{layer}"]:
                        assert np.array_equal(recv[ep], dst[np.argsort(pos, kind="stable")] - 1), (
                            f"{loc} layer {layer}: {ep}->{bid} receive list (buffer order)")
                    assert len(r[f"{loc}_send_{layer}"]) == len(send)
                    assert len(r[f"{loc}_recv_{layer}"]) == len(recv)
    assert nlists > 0


@pytest.mark.parametrize("nblocks", [2, 4, 8])
def test_decomp_equals_reference_blocks_one_task(mesh2562, nblocks):
    from mpas_dycore import decomp
    _check(mesh2562, decomp.partition_sfc(mesh2562["nCells"], nblocks), 1)


def test_decomp_equals_reference_scattered_partition(mesh2562):
    """A partition with interleaved, non-contiguous blocks (as METIS files can have)."""
    rng = np.random.default_rng(7)
    part = (np.arange(mesh2562["nCells"]) * 5 // mesh2562["nCells"]).astype(np.int32)
    flip = rng.choice(mesh2562["nCells"], 200, replace=False)
    part[flip] = rng.integers(0, 5, size=200)
    _check(mesh2562, part, 1)


def test_decomp_equals_reference_varres(varres):
    from mpas_dycore import decomp
    _check(varres, decomp.partition_sfc(varres["nCells"], 4), 1)


@pytest.mark.skipif(not os.access(ref_runner.MPIRUN, os.X_OK), reason="no mpirun")
@pytest.mark.parametrize("nprocs", [2, 4])
def test_decomp_equals_reference_one_block_per_task(mesh2562, nprocs):
    from mpas_dycore import decomp
    _check(mesh2562, decomp.partition_sfc(mesh2562["nCells"], nprocs), nprocs)
