"""Horizontal domain decomposition: blocks with halos and their exchange lists.

Restates how MPAS builds a block from a cell partition
(framework/mpas_bootstrapping.F:238-268, mpas_block_creator.F,
mpas_block_decomp.F) so one rank's dycore sees exactly what the reference's
would.

* **Cells.** A block owns the cells its partition assigns it (nCellsSolve).
  It then adds ``nHalos`` = config_num_halos = 2 layers (Registry.xml:242).
  Layer ``l`` is the set of cellsOnCell neighbours of layers < l that are not
  yet in the block (mpas_block_creator_build_cell_halos, :470-716).
* **Edges and vertices.** A block owns an edge when the first valid
  cellsOnEdge entry is an owned cell (mpas_block_decomp_partitioned_edge_list,
  mpas_block_decomp.F:301-356). Vertices use cellsOnVertex the same way
  (mpas_bootstrapping.F:253).
  * Halo layer 1 holds the remaining edges of the owned cells.
  * Layer ``l`` > 1 holds the edges of the cell-halo layer ``l-1`` not yet in
    the block (build_edge_halos, :734-938).
  * Edge and vertex fields therefore have nHalos+1 = 3 exchange layers.
* **Local order** is the reference's (see ``_block_elements``): owned first,
  then each halo layer, so the local indices and exchange lists a rank sees are
  the ones MPAS would build from the same partition file.
* **Missing neighbours.** Connectivity is remapped to block-local indices, and
  neighbours outside the block become -1, which is the garbage slot n+1 at the
  C ABI (mpas_block_creator.F:1445).
* **Exchange lists** (mpas_dmpar_get_exch_list, mpas_dmpar.F:1483-2038). For
  every (block, location, halo layer), the halo elements are grouped by owning
  block, and both sides list them in the same order:
  * between blocks of different MPI tasks, in ascending global index (the
    message buffer order of sendList / recvList);
  * between blocks of one task, in the owner's local order (copyList,
    :1825-1875).
  ``tests/test_decomp_pinned.py`` checks local orders, halo layers and both list
  kinds against the reference's own mpas_block_decomp.F / mpas_block_creator.F.
* **Partition.** The default partition splits the cells into contiguous ranges
  of the space-filling-curve order of ``mesh.py``. A METIS
  ``graph.info.part.N`` file, as read by mpas_block_decomp.F, is accepted as
  well.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import fields as F

NHALOS = 2
LOCS = ("cell", "edge", "vertex")
LOC_CODE = {"cell": 0, "edge": 1, "vertex": 2}
NLAYERS = {"cell": NHALOS, "edge": NHALOS + 1, "vertex": NHALOS + 1}
_N = {"cell": "nCells", "edge": "nEdges", "vertex": "nVertices"}


def partition_sfc(nCells: int, nparts: int) -> np.ndarray:
    """Owner block of every cell: contiguous ranges of the (Hilbert-ordered) cell index."""
    if nparts < 1 or nparts > nCells:
        raise ValueError(f"cannot split {nCells} cells into {nparts} blocks")
    return (np.arange(nCells, dtype=np.int64) * nparts // nCells).astype(np.int32)


def read_partition_file(path: str, nCells: int) -> np.ndarray:
    """graph.info.part.N: one 0-based owning block per line (mpas_block_decomp.F:106-160)."""
    part = np.loadtxt(path, dtype=np.int64, ndmin=1)
    if part.size != nCells:
        raise ValueError(f"{path}: {part.size} entries for {nCells} cells")
    return part.astype(np.int32)


def _neighbours(idx2d: np.ndarray, counts: np.ndarray | None, rows: np.ndarray) -> np.ndarray:
    """Unique valid entries of idx2d[rows, :counts[rows]]."""
    if rows.size == 0:
        return rows
    sub = idx2d[rows]
    if counts is not None:
        mask = np.arange(sub.shape[1])[None, :] < counts[rows][:, None]
        vals = sub[mask]
    else:
        vals = sub.ravel()
    vals = vals[vals >= 0]
    return np.unique(vals)


def element_owners(case: dict, cell_part: np.ndarray) -> dict:
    """Owning block of every cell, edge and vertex (first valid cell of cellsOnEdge / cellsOnVertex)."""
    def first_valid(c2):
        c = c2[:, 0].copy()
        for j in range(1, c2.shape[1]):
            bad = c < 0
            c[bad] = c2[bad, j]
        if (c < 0).any():
            raise ValueError("element not adjacent to any valid cell")
        return c
    return {"cell": np.asarray(cell_part, dtype=np.int32),
            "edge": cell_part[first_valid(np.asarray(case["cellsOnEdge"]))],
            "vertex": cell_part[first_valid(np.asarray(case["cellsOnVertex"]))]}


@dataclass
class Block:
    """One block: its local case plus the local -> global maps and halo layer sizes."""
    part: int
    case: dict
    glob: dict                      # loc -> global index of every local element
    layer_end: dict                 # loc -> cumulative counts [owned, +layer1, ...] (MPAS n*Solve arrays)
    send: list = field(default_factory=list)   # (loc, layer, peer, local idx 0-based)
    recv: list = field(default_factory=list)

    @property
    def solve(self) -> tuple:
        return (self.layer_end["cell"][0], self.layer_end["edge"][0], self.layer_end["vertex"][0])

    def layer_range(self, loc: str, layer: int) -> tuple:
        """[start, end) of halo layer ``layer`` (0 = owned) of a location."""
        e = self.layer_end[loc]
        return (0 if layer == 0 else e[layer - 1], e[layer])


def _discovery_order(idx2d: np.ndarray, counts: np.ndarray, rows: np.ndarray) -> np.ndarray:
    """Unique valid entries of idx2d[rows, :counts[rows]] in first-encounter order
    (mpas_block_decomp_all_edges_in_block, mpas_block_decomp.F:369-420)."""
    sub = idx2d[rows]
    mask = np.arange(sub.shape[1])[None, :] < counts[rows][:, None]
    vals = sub[mask]
    vals = vals[vals >= 0]
    _, first = np.unique(vals, return_index=True)
    return vals[np.sort(first)]


def _block_elements(case: dict, owners: dict, p: int) -> tuple[dict, dict]:
    """Local element order of block p, as mpas_block_creator builds it:
    cells: owned in ascending global ID, then each halo layer quicksorted (:601);
    edges/vertices: owned in discovery order over the owned cells, then layer 1 in
    reverse discovery order (ghostEdgeStart counts down, mpas_block_decomp.F:339-341),
    then the new edges of each cell-halo layer in discovery order (:859-876)."""
    nEdgesOnCell = np.asarray(case["nEdgesOnCell"])
    cellsOnCell = np.asarray(case["cellsOnCell"])
    owned = np.flatnonzero(owners["cell"] == p)
    if owned.size == 0:
        raise ValueError(f"block {p} owns no cells")
    cell_layers = [owned]
    seen = np.zeros(case["nCells"], dtype=bool)
    seen[owned] = True
    for _ in range(NHALOS):
        nb = _neighbours(cellsOnCell, nEdgesOnCell, cell_layers[-1])
        new = nb[~seen[nb]]
        seen[new] = True
        cell_layers.append(new)
    cells = np.concatenate(cell_layers)
    groups = {"cell": cell_layers}
    for loc, on_cell in (("edge", "edgesOnCell"), ("vertex", "verticesOnCell")):
        arr = np.asarray(case[on_cell])
        n = case[_N[loc]]
        e0 = _discovery_order(arr, nEdgesOnCell, owned)
        mine = owners[loc][e0] == p
        lays = [e0[mine], e0[~mine][::-1]]
        in_blk = np.zeros(n, dtype=bool)
        in_blk[e0] = True
        ncl = owned.size
        for h in range(1, NHALOS + 1):
            ncl += cell_layers[h].size
            found = _discovery_order(arr, nEdgesOnCell, cells[:ncl])
            new = found[~in_blk[found]]
            in_blk[new] = True
            lays.append(new)
        groups[loc] = lays
    glob = {loc: np.concatenate(groups[loc]).astype(np.int64) for loc in LOCS}
    layer_end = {loc: [int(x) for x in np.cumsum([g.size for g in groups[loc]])] for loc in LOCS}
    return glob, layer_end


def _local_case(case: dict, glob: dict) -> dict:
    g2l = {}
    for loc in LOCS:
        m = np.full(case[_N[loc]], -1, dtype=np.int64)
        m[glob[loc]] = np.arange(glob[loc].size)
        g2l[loc] = m
    out = {}
    for k, v in case.items():
        loc = F.LOCATION.get(k)
        if loc is None or not isinstance(v, np.ndarray):
            out[k] = v
            continue
        sub = v[glob[loc]]
        if k in F.INDEX_TARGET:
            tgt = g2l[F.INDEX_TARGET[k]]
            sub = np.where(sub >= 0, tgt[np.maximum(sub, 0)], -1)
        out[k] = np.ascontiguousarray(sub)
    for loc in LOCS:
        out[_N[loc]] = int(glob[loc].size)
    return out


def decompose(case: dict, cell_part: np.ndarray, parts=None, placement: dict | None = None) -> list[Block]:
    """Build the blocks of ``parts`` (default: all) with their send and receive lists.

    ``placement`` maps every block to (rank, local block index), as Dycore.from_blocks takes it;
    it decides the list order between two blocks (same rank: the owner's local order, else
    ascending global index, see the module docstring).  Default: one block per rank.
    The element sets of every block are computed (cheap), so a rank can build
    only its own block(s) and still know what each neighbour expects from it."""
    nparts = int(cell_part.max()) + 1
    owners = element_owners(case, cell_part)
    elems = [_block_elements(case, owners, p) for p in range(nparts)]
    want = list(range(nparts)) if parts is None else list(parts)
    rank_of = {p: (placement[p][0] if placement is not None else p) for p in range(nparts)}
    blocks = [Block(part=p, case=_local_case(case, elems[p][0]), glob=elems[p][0], layer_end=elems[p][1])
              for p in want]
    g2own_cache = {}

    def g2own(q, loc):   # global index -> owned local index in block q
        if (q, loc) not in g2own_cache:
            glob_q, lend_q = elems[q]
            m = np.full(case[_N[loc]], -1, dtype=np.int64)
            m[glob_q[loc][:lend_q[loc][0]]] = np.arange(lend_q[loc][0])
            g2own_cache[(q, loc)] = m
        return g2own_cache[(q, loc)]

    def message_order(gids, src, dst, loc):   # order of the elements gids sent by block src to dst
        key = g2own(src, loc)[gids] if rank_of[src] == rank_of[dst] else gids
        return np.argsort(key, kind="stable")

    for b in blocks:
        for loc in LOCS:
            for layer in range(1, NLAYERS[loc] + 1):
                # receive: my layer-`layer` halo elements, grouped by owner
                s, e = b.layer_range(loc, layer)
                gl = b.glob[loc][s:e]
                own = owners[loc][gl]
                for q in np.unique(own):
                    sel = np.flatnonzero(own == q)
                    sel = sel[message_order(gl[sel], int(q), b.part, loc)]
                    b.recv.append((loc, layer, int(q), (s + sel).astype(np.int32)))
                # send: every other block's layer-`layer` halo elements that I own
                for p in range(nparts):
                    if p == b.part:
                        continue
                    glob_p, lend_p = elems[p]
                    gids = glob_p[loc][lend_p[loc][layer - 1]:lend_p[loc][layer]]
                    gids = gids[owners[loc][gids] == b.part]
                    if gids.size:
                        gids = gids[message_order(gids, b.part, p, loc)]
                        b.send.append((loc, layer, p, g2own(b.part, loc)[gids].astype(np.int32)))
    return blocks


def gather_owned(blocks: list[Block], arrays: list, loc: str, n_global: int) -> np.ndarray:
    """Scatter each block's owned rows of an element-major array into the global array."""
    out = None
    for b, a in zip(blocks, arrays):
        a = np.asarray(a)
        if out is None:
            out = np.full((n_global,) + a.shape[1:], np.nan, dtype=a.dtype)
        n_own = b.layer_end[loc][0]
        out[b.glob[loc][:n_own]] = a[:n_own]
    return out


def messages(block: Block, direction: str, layers=(1, 2, 3), locs=LOCS) -> dict:
    """Host restatement of one block's messages for an exchange: peer -> list of local index
    arrays in message order (layers ascending), as the device plan packs them."""
    lists = block.send if direction == "send" else block.recv
    out = {}
    for loc in locs:
        for layer in sorted(layers):
            for (l, lay, peer, idx) in lists:
                if l == loc and lay == layer:
                    out.setdefault(peer, []).append(idx)
    return {p: np.concatenate(v) for p, v in sorted(out.items())}


def rank_blocks(case: dict, nranks: int, rank: int, blocks_per_rank: int = 1, cell_part=None):
    """Blocks of one rank and the placement of every block: block p lives on rank
    p // blocks_per_rank as local block p % blocks_per_rank (config_number_of_blocks
    per MPI task, mpas_block_decomp.F:65-100)."""
    nparts = nranks * blocks_per_rank
    if cell_part is None:
        cell_part = partition_sfc(case["nCells"], nparts)
    mine = list(range(rank * blocks_per_rank, (rank + 1) * blocks_per_rank))
    placement = {p: (p // blocks_per_rank, p % blocks_per_rank) for p in range(nparts)}
    blocks = decompose(case, cell_part, parts=mine, placement=placement)
    return blocks, placement


def positional_lists(blocks: list[Block], placement: dict, rank: int, include_self: bool = False) -> list:
    """The exchange lists of this rank's blocks as mpas_dmpar holds them when tasks own several blocks
    (parinfo xToSend / xToRecv: endPointID = the task, the other list = buffer positions,
    mpas_dmpar.F:5448-5535): for each (peer rank, location, halo layer) one buffer whose slots are the
    distinct elements the two tasks exchange there, in ascending global index -- a set both sides
    know, so both number it alike without knowing the other side's blocks.  Returns, per block, a
    list of (direction "send" / "recv", loc, layer, peer_rank, local 0-based indices, 1-based
    positions) for mpas_dyc_set_exchange_positions.  include_self: also the lists between blocks of
    this rank (a one-process test of the positional path over RCCL)."""
    def peer_ok(pr):
        return pr != rank or include_self
    union = {}   # (dir, loc, layer, peer_rank) -> global ids of this rank's side
    per = []     # per block: {(dir, loc, layer, peer_rank): (local idx, gids)}
    for b in blocks:
        mine = {}
        for dname, lists in (("send", b.send), ("recv", b.recv)):
            for loc, layer, peer, idx in lists:
                pr = placement[peer][0]
                if not peer_ok(pr):
                    continue
                key = (dname, loc, layer, pr)
                idx = np.asarray(idx, dtype=np.int64)
                mine.setdefault(key, []).append(idx)
        out = {}
        for key, parts in mine.items():
            idx = np.concatenate(parts)
            gids = b.glob[key[1]][idx]
            gids, first = np.unique(gids, return_index=True)   # an element goes once per buffer
            out[key] = (idx[first], gids)
            union.setdefault(key, []).append(gids)
        per.append(out)
    union = {k: np.unique(np.concatenate(v)) for k, v in union.items()}
    res = []
    for out in per:
        lst = []
        for key in sorted(out):
            idx, gids = out[key]
            pos = np.searchsorted(union[key], gids) + 1
            lst.append((key[0], key[1], key[2], key[3], idx.astype(np.int32), pos.astype(np.int32)))
        res.append(lst)
    return res
