"""Domain decomposition (CPU): block construction and exchange lists as MPAS builds them.

Checks the rules of mpas_block_creator.F / mpas_block_decomp.F restated in
mpas_dycore/decomp.py:
  * ownership partitions every cell, edge and vertex;
  * halo layers are the cellsOnCell rings;
  * the edge and vertex owner is the owner of the first valid cell;
  * local connectivity maps back to the global mesh;
  * the exchange lists make every halo exact.
The last check is run in one process and across two gloo ranks, using the
same message plan as the device exchange.
"""
import os

import numpy as np
import pytest

from mpas_dycore import decomp

NPARTS = [2, 3, 7]


@pytest.fixture(scope="module")
def blocks_by_n(small_case):
    return {n: decomp.decompose(small_case, decomp.partition_sfc(small_case["nCells"], n)) for n in NPARTS}


@pytest.mark.parametrize("n", NPARTS)
def test_ownership_partitions_every_element(small_case, blocks_by_n, n):
    blocks = blocks_by_n[n]
    for loc, key in (("cell", "nCells"), ("edge", "nEdges"), ("vertex", "nVertices")):
        owned = np.concatenate([b.glob[loc][:b.layer_end[loc][0]] for b in blocks])
        assert np.array_equal(np.sort(owned), np.arange(small_case[key])), loc


@pytest.mark.parametrize("n", NPARTS)
def test_halo_layers_and_owner_rules(small_case, blocks_by_n, n):
    c = small_case
    part = decomp.partition_sfc(c["nCells"], n)
    coc, noc = c["cellsOnCell"], c["nEdgesOnCell"]
    for b in blocks_by_n[n]:
        cells = b.glob["cell"]
        s0, e0 = b.layer_range("cell", 0)
        assert np.all(part[cells[s0:e0]] == b.part)
        prev = set(cells[s0:e0].tolist())
        for layer in (1, 2):
            s, e = b.layer_range("cell", layer)
            ring = set()
            for ci in cells[(0 if layer == 1 else b.layer_range("cell", layer - 1)[0]):
                            b.layer_range("cell", layer - 1)[1]]:
                ring.update(coc[ci, :noc[ci]].tolist())
            assert set(cells[s:e].tolist()) == ring - prev, f"cell layer {layer}"
            prev |= ring
        # owned edges: first cell of cellsOnEdge owned (mpas_block_decomp_partitioned_edge_list)
        own_e = b.glob["edge"][:b.layer_end["edge"][0]]
        assert np.all(part[c["cellsOnEdge"][own_e, 0]] == b.part)
        own_v = b.glob["vertex"][:b.layer_end["vertex"][0]]
        assert np.all(part[c["cellsOnVertex"][own_v, 0]] == b.part)
        # every edge of every block cell is in the block
        allc = cells
        eoc = c["edgesOnCell"][allc]
        need = np.unique(eoc[np.arange(eoc.shape[1])[None, :] < noc[allc][:, None]])
        assert set(need.tolist()) <= set(b.glob["edge"].tolist())


@pytest.mark.parametrize("n", NPARTS)
def test_local_connectivity_maps_to_global(small_case, blocks_by_n, n):
    c = small_case
    for b in blocks_by_n[n]:
        lc = b.case
        for name, loc, tgt in (("cellsOnCell", "cell", "cell"), ("edgesOnCell", "cell", "edge"),
                               ("verticesOnCell", "cell", "vertex"), ("cellsOnEdge", "edge", "cell"),
                               ("edgesOnEdge", "edge", "edge"), ("advCellsForEdge", "edge", "cell"),
                               ("cellsOnVertex", "vertex", "cell"), ("edgesOnVertex", "vertex", "edge")):
            loc_idx = lc[name]
            glob_idx = c[name][b.glob[loc]]
            inside = loc_idx >= 0
            assert np.array_equal(b.glob[tgt][loc_idx[inside]], glob_idx[inside]), name
            # owned cells/edges have their whole stencil inside the block
            n_own = b.layer_end[loc][0]
            if name in ("cellsOnCell", "edgesOnCell", "verticesOnCell"):
                cnt = c["nEdgesOnCell"][b.glob[loc][:n_own]]
                m = np.arange(loc_idx.shape[1])[None, :] < cnt[:, None]
                assert np.all(loc_idx[:n_own][m] >= 0), name
            if name == "advCellsForEdge":
                cnt = c["nAdvCellsForEdge"][b.glob[loc][:n_own]]
                m = np.arange(loc_idx.shape[1])[None, :] < cnt[:, None]
                assert np.all(loc_idx[:n_own][m] >= 0), name
        assert lc["nCells"] == b.glob["cell"].size and b.solve[0] == b.layer_end["cell"][0]


def _exchange_in_process(blocks, loc, g, layers=(1, 2, 3)):
    arrs = []
    for b in blocks:
        a = np.full((b.glob[loc].size,) + g.shape[1:], np.nan)
        no = b.layer_end[loc][0]
        a[:no] = g[b.glob[loc][:no]]
        arrs.append(a)
    msgs = {}
    for b, a in zip(blocks, arrs):
        for peer, idx in decomp.messages(b, "send", layers, (loc,)).items():
            msgs[(b.part, peer)] = a[idx].copy()
    for b, a in zip(blocks, arrs):
        for peer, idx in decomp.messages(b, "recv", layers, (loc,)).items():
            a[idx] = msgs.pop((peer, b.part))
    assert not msgs, "unmatched messages"
    return arrs


@pytest.mark.parametrize("n", NPARTS)
@pytest.mark.parametrize("loc,key", [("cell", "nCells"), ("edge", "nEdges"), ("vertex", "nVertices")])
def test_exchange_lists_make_halos_exact(small_case, blocks_by_n, n, loc, key):
    g = np.random.default_rng(3).standard_normal((small_case[key], 5))
    blocks = blocks_by_n[n]
    for b, a in zip(blocks, _exchange_in_process(blocks, loc, g)):
        assert np.array_equal(a, g[b.glob[loc]])
    # layer 1 only: outer layers keep their stale (NaN) values
    arrs = _exchange_in_process(blocks, loc, g, layers=(1,))
    for b, a in zip(blocks, arrs):
        s, e = b.layer_range(loc, 1)
        assert np.array_equal(a[:e], g[b.glob[loc][:e]])
        assert np.all(np.isnan(a[e:]))


def test_exchange_lists_on_variable_resolution_mesh():
    """Irregular halos (5/6/7-gons) still give exact halos on every layer."""
    from mpas_dycore.mesh import build_varres_mesh
    m = build_varres_mesh(2562, ratio=4.0, lloyd_iters=30)
    blocks = decomp.decompose(m, decomp.partition_sfc(m["nCells"], 6))
    for loc, key in (("cell", "nCells"), ("edge", "nEdges"), ("vertex", "nVertices")):
        g = np.random.default_rng(5).standard_normal((m[key], 2))
        for b, a in zip(blocks, _exchange_in_process(blocks, loc, g)):
            assert np.array_equal(a, g[b.glob[loc]])


def test_partition_file_round_trip(tmp_path, small_case):
    part = decomp.partition_sfc(small_case["nCells"], 4)
    p = tmp_path / "graph.info.part.4"
    np.savetxt(p, part, fmt="%d")
    assert np.array_equal(decomp.read_partition_file(str(p), small_case["nCells"]), part)


def _gloo_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from mpas_dycore.mesh import build_mesh
        from mpas_dycore.init_atm import build_case
        case = build_case(build_mesh(2, lloyd_iters=5), K=4, ns=1)
        (b,), placement = decomp.rank_blocks(case, world, rank, 1)
        assert placement == {p: (p, 0) for p in range(world)}
        # what I send to each rank is exactly what that rank expects to receive
        mine = {(b.part, peer): [(l, lay, int(i.size)) for (l, lay, q, i) in b.send if q == peer]
                for peer in range(world) if peer != rank}
        theirs = {(peer, b.part): [(l, lay, int(i.size)) for (l, lay, q, i) in b.recv if q == peer]
                  for peer in range(world) if peer != rank}
        everyone = [None] * world
        dist.all_gather_object(everyone, (mine, theirs))
        ok = all(everyone[dst][1][(src, dst)] == lists for src in range(world)
                 for (s_, dst), lists in everyone[src][0].items())
        for loc, key in (("cell", "nCells"), ("edge", "nEdges"), ("vertex", "nVertices")):
            g = np.random.default_rng(11).standard_normal((case[key], 3))
            a = np.full((b.glob[loc].size, 3), np.nan)
            no = b.layer_end[loc][0]
            a[:no] = g[b.glob[loc][:no]]
            sends = decomp.messages(b, "send", locs=(loc,))
            recvs = decomp.messages(b, "recv", locs=(loc,))
            reqs = [dist.isend(torch.from_numpy(np.ascontiguousarray(a[idx])), dst=peer)
                    for peer, idx in sends.items()]
            for peer, idx in recvs.items():
                buf = torch.empty((idx.size, 3), dtype=torch.float64)
                dist.recv(buf, src=peer)
                a[idx] = buf.numpy()
            for r in reqs:
                r.wait()
            ok &= bool(np.array_equal(a, g[b.glob[loc]]))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, ok))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_across_gloo_ranks(world):
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}, res


def _reference_edge_order(case, part, p, on_cell, owner_of):
    """Loop-by-loop restatement of mpas_block_decomp_all_edges_in_block +
    mpas_block_decomp_partitioned_edge_list + build_edge_halos for one block."""
    noc = case["nEdgesOnCell"]
    coc = case["cellsOnCell"]
    owned = [c for c in range(case["nCells"]) if part[c] == p]
    cells = list(owned)
    layers = []
    seen = set(cells)
    for _ in range(2):
        ring = sorted({int(n) for c in (layers[-1] if layers else owned) for n in coc[c, :noc[c]]} - seen)
        seen |= set(ring)
        layers.append(ring)
    def all_in(cs):
        out, h = [], set()
        for c in cs:
            for j in range(noc[c]):
                e = int(case[on_cell][c, j])
                if e not in h:
                    h.add(e)
                    out.append(e)
        return out
    e0 = all_in(owned)
    lst = [None] * len(e0)
    last, ghost = 0, len(e0)
    for e in e0:
        if owner_of[e] == p:
            lst[last] = e
            last += 1
        else:
            ghost -= 1
            lst[ghost] = e
    have = set(lst)
    for h in range(2):
        cs = owned + sum(layers[:h + 1], [])
        for e in all_in(cs):
            if e not in have:
                have.add(e)
                lst.append(e)
    return cells + layers[0] + layers[1], lst


def test_local_order_matches_reference_block_creator(small_case):
    part = decomp.partition_sfc(small_case["nCells"], 3)
    owners = decomp.element_owners(small_case, part)
    for b in decomp.decompose(small_case, part):
        cells, edges = _reference_edge_order(small_case, part, b.part, "edgesOnCell", owners["edge"])
        assert b.glob["cell"].tolist() == cells
        assert b.glob["edge"].tolist() == edges
        _, verts = _reference_edge_order(small_case, part, b.part, "verticesOnCell", owners["vertex"])
        assert b.glob["vertex"].tolist() == verts
