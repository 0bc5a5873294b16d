"""One-world view of a :class:`DistributedWorld`: the reference ``World`` API with GLOBAL cell indices.

The decomposed world keeps every rank's cells in rank-local rows (the hot path works on them
without any global bookkeeping). :class:`GlobalWorld` wraps it for code written against the
reference API (``python/magicsoup/world.py``): every method takes and returns global cell indices
with the reference's index semantics, and placement is uniform over the whole torus.

Index semantics (reference world.py):
- ``spawn_cells`` / ``add_cells`` / ``divide_cells`` append new cells at the END of the global
  index space (world.py:318, 374, 451); existing cells keep their index, also when a child is
  born on another rank.
- ``kill_cells`` removes indices, the cells after them shift down (world.py:506-510).
- ``move_cells`` / ``reposition_cells`` keep indices, also when a cell changes rank.

The numbering is a replicated table ``global index -> (rank, local row)`` kept identical on every
rank: each op updates it from data every rank already holds (the op's arguments) plus one small
``all_gather_object`` of what crossed a strip boundary (recorded by DistributedWorld in
``_xfer``, in record order). Every method is collective: all ranks call it with the same
arguments. Ops called directly on the wrapped world (rank-local indices) invalidate the table; the
next call here notices (per-rank counts differ) and renumbers rank by rank (:meth:`resync`).

Placement over the whole map (``spawn_cells``, ``add_cells``, ``reposition_cells``): the number of
cells landing on each rank is a multivariate-hypergeometric draw over the ranks' free pixel counts
(a shared stream, identical on every rank), each rank then places its share uniformly in its strip:
uniform over all free pixels of the torus, like world.py:307/363/603.

This view is for control-plane use (setup, analysis, occasional interventions). The steady-state
simulation loop belongs on the rank-local API (``bench.py``), which needs no collectives beyond the
physics' own.
"""

from __future__ import annotations

import random
from typing import Any

import numpy as np
import torch
import torch.distributed as dist

from magicsoup_amd.models.containers import Cell

from .dist_world import DistributedWorld

__all__ = ["GlobalWorld"]


class GlobalWorld:
    """Reference-``World``-shaped facade over a :class:`DistributedWorld` ``dw`` (see module doc).

    Attributes not defined here (``chemistry``, ``genetics``, ``kinetics``, ``map_size``,
    ``n_molecules``, ...) are forwarded to ``dw``.
    """

    def __init__(self, dw: DistributedWorld):
        self.__dict__["dw"] = dw
        self.resync()

    # ------------------------------------------------------------------ plumbing
    def __getattr__(self, name: str) -> Any:
        return getattr(self.__dict__["dw"], name)

    @property
    def _ws(self) -> int:
        return self.dw.world_size

    @property
    def _me(self) -> int:
        return self.dw.rank

    def _gather(self, obj) -> list:
        out = [None] * self._ws
        dist.all_gather_object(out, obj, group=self.dw.group)
        return out

    def _shared_seed(self) -> int:
        seed = [random.getrandbits(63) if self._me == 0 else 0]
        g = self.dw.group
        dist.broadcast_object_list(seed, src=dist.get_global_rank(g, 0) if g is not None else 0, group=g)
        return int(seed[0])

    def resync(self) -> None:
        """Collective: renumber the cells rank by rank (rank 0's cells first, in local order)."""
        counts = [int(c) for c in self._gather(int(self.dw.n_cells))]
        self.__dict__["_rank"] = np.repeat(np.arange(self._ws, dtype=np.int32), counts)
        self.__dict__["_local"] = np.concatenate([np.arange(c, dtype=np.int64) for c in counts] or [np.zeros(0, np.int64)])

    def _begin(self) -> None:
        """Every op starts here on every rank: settle queued genome ops (their exchanges are
        collective, so all ranks issue them at the same point) and verify the table."""
        dw = self.dw
        dw._reconcile()
        counts = self._gather(int(dw.n_cells))
        if list(np.bincount(self._rank, minlength=self._ws)) != counts:
            self.resync()
        dw.__dict__.pop("_xfer", None)

    def _global_idxs(self, cell_idxs, default_all: bool) -> np.ndarray:
        n = len(self._rank)
        if cell_idxs is None:
            return np.arange(n, dtype=np.int64) if default_all else np.zeros(0, np.int64)
        if isinstance(cell_idxs, torch.Tensor):
            cell_idxs = cell_idxs.flatten().tolist()
        g = np.unique(np.asarray(list(cell_idxs), dtype=np.int64))  # duplicates dropped (world.py:437, 518)
        if g.size and (g[0] < 0 or g[-1] >= n):
            raise IndexError(f"cell index out of range for {n} cells")
        return g

    def _mine(self, g: np.ndarray) -> np.ndarray:
        """Local rows (ascending) of the global indices ``g`` that live on this rank."""
        sel = self._rank[g] == self._me
        return np.sort(self._local[g[sel]])

    def _l2g(self, r: int) -> np.ndarray:
        """Global index of every local row of rank ``r``."""
        at = np.nonzero(self._rank == r)[0]
        out = np.empty(at.size, dtype=np.int64)
        out[self._local[at]] = at
        return out

    def _drop(self, gone_per_rank: list[np.ndarray], keep_global: np.ndarray | None = None) -> np.ndarray:
        """Remove local rows from the table (order-preserving compaction on every rank, as the
        rank-local kill / emigration does). ``keep_global`` marks global entries that survive even
        though their row is listed (cells that moved to another rank). Returns the old -> new
        global index map (-1 for removed entries)."""
        rank, local = self._rank, self._local.copy()
        alive = np.ones(rank.size, dtype=bool)
        for r, gone in enumerate(gone_per_rank):
            if gone.size == 0:
                continue
            at = np.nonzero(rank == r)[0]
            row_gone = np.zeros(at.size, dtype=bool)
            row_gone[gone] = True
            hit = at[row_gone[local[at]]]
            alive[hit] = False
            shift = np.cumsum(row_gone) - row_gone  # rows removed before each row
            local[at] = local[at] - shift[local[at]]
        if keep_global is not None:
            alive |= keep_global
        new_idx = np.full(rank.size, -1, dtype=np.int64)
        new_idx[alive] = np.arange(int(alive.sum()))
        self.__dict__["_rank"] = rank[alive]
        self.__dict__["_local"] = local[alive]
        return new_idx

    def _append(self, ranks, locals_) -> None:
        self.__dict__["_rank"] = np.concatenate([self._rank, np.asarray(ranks, dtype=np.int32)])
        self.__dict__["_local"] = np.concatenate([self._local, np.asarray(locals_, dtype=np.int64)])

    def _xfer(self) -> dict:
        """This rank's boundary transfers of the last op as plain lists (empty without strips)."""
        x = self.dw.__dict__.pop("_xfer", None)
        if x is None:
            return {"up": [], "dn": [], "in_up": 0, "in_dn": 0}
        up, dn, in_up, in_dn = x
        return {"up": up.tolist(), "dn": dn.tolist(), "in_up": int(in_up), "in_dn": int(in_dn)}

    def _arrival_sources(self, info: list[dict], r: int) -> list[tuple[int, int]]:
        """(sender rank, sender row) of every arrival on rank ``r`` in append order: first the
        records from the upper neighbour (its ``dn`` exports), then from the lower one."""
        ws = self._ws
        u, d = (r - 1) % ws, (r + 1) % ws
        src = [(u, row) for row in info[u]["dn"]]
        src += [(d, row) for row in info[d]["up"]]
        assert len(src) == info[r]["in_up"] + info[r]["in_dn"], "boundary transfer bookkeeping out of step"
        return src

    def _split_counts(self, k: int, extra_free: list[int] | None = None) -> tuple[np.random.Generator, np.ndarray, list[int]]:
        """Shared draw: how many of ``k`` new placements land on each rank (uniform over the free
        pixels of the torus). Returns (shared rng, permutation of the k items, counts)."""
        dw = self.dw
        free = [int(f) for f in self._gather(int(dw.H * dw.map_size - dw.n_cells))]
        if extra_free is not None:
            free = [a + b for a, b in zip(free, extra_free)]
        rng = np.random.default_rng(self._shared_seed())
        n = min(k, sum(free))
        order = rng.permutation(k)[:n]
        counts = rng.multivariate_hypergeometric(np.asarray(free, dtype=np.int64), n) if n else np.zeros(self._ws, np.int64)
        return rng, order, [int(c) for c in counts]

    # ------------------------------------------------------------------ global state views
    @property
    def n_cells(self) -> int:
        """Number of cells of the whole job (replicated; no communication)."""
        return int(self._rank.size)

    def _gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        parts = self._gather(t.detach().cpu())
        out = torch.zeros((self.n_cells,) + tuple(parts[0].shape[1:]), dtype=parts[0].dtype)
        for r, p in enumerate(parts):
            out[torch.from_numpy(self._l2g(r))] = p
        return out

    @property
    def cell_molecules(self) -> torch.Tensor:
        """Collective: (n_cells, n_molecules) in global index order (CPU tensor; a copy)."""
        self._begin()
        return self._gather_rows(self.dw.cell_molecules)

    @property
    def cell_positions(self) -> torch.Tensor:
        """Collective: global map coordinates (n_cells, 2) int32 (CPU tensor; a copy)."""
        self._begin()
        return self._gather_rows(self.dw.global_positions())

    @property
    def cell_lifetimes(self) -> torch.Tensor:
        self._begin()
        return self._gather_rows(self.dw.cell_lifetimes)

    @property
    def cell_divisions(self) -> torch.Tensor:
        self._begin()
        return self._gather_rows(self.dw.cell_divisions)

    def _gather_strings(self, vals: list[str]) -> list[str]:
        parts = self._gather(vals)
        out = [""] * self.n_cells
        for r, p in enumerate(parts):
            for g, v in zip(self._l2g(r).tolist(), p):
                out[g] = v
        return out

    @property
    def cell_genomes(self) -> list[str]:
        self._begin()
        return self._gather_strings(list(self.dw.cell_genomes))

    @property
    def cell_labels(self) -> list[str]:
        self._begin()
        return self._gather_strings(list(self.dw.cell_labels))

    @property
    def molecule_map(self) -> torch.Tensor:
        """Collective: the global (n_molecules, S, S) map (CPU copy)."""
        self._begin()
        return torch.cat(self._gather(self.dw.owned_molecule_map().cpu()), dim=1)

    @property
    def cell_map(self) -> torch.Tensor:
        self._begin()
        return torch.cat(self._gather(self.dw.owned_cell_map().cpu()), dim=0)

    def global_index_of_local(self, local_idxs=None) -> list[int]:
        """Global indices of this rank's local rows (all of them by default). Not collective."""
        g = self._l2g(self._me)
        return g.tolist() if local_idxs is None else g[np.asarray(list(local_idxs), dtype=np.int64)].tolist()

    def local_of_global(self, cell_idxs) -> list[int]:
        """Local rows of those global indices that live on this rank (ascending). Not collective."""
        return self._mine(self._global_idxs(cell_idxs, True)).tolist()

    # ------------------------------------------------------------------ queries
    def get_cell(self, by_idx: int | None = None, by_position: tuple[int, int] | None = None,
                 by_label: str | None = None) -> Cell:
        """Collective: a :class:`Cell` snapshot (genome, global position, label, lifetime,
        divisions, intracellular and pixel molecules) of the cell with global index ``by_idx``, at
        global pixel ``by_position`` or with label ``by_label``."""
        self._begin()
        dw = self.dw
        me = self._me
        row = -1
        if by_idx is not None:
            g = int(by_idx) % max(self.n_cells, 1)
            if self._rank[g] == me:
                row = int(self._local[g])
        elif by_position is not None:
            x, y = int(by_position[0]) % dw.map_size, int(by_position[1]) % dw.map_size
            if dw.row0 <= x < dw.row0 + dw.H:
                hit = torch.nonzero((dw.global_positions().cpu() == torch.tensor([x, y], dtype=torch.int32)).all(1))
                row = int(hit[0]) if hit.numel() else -1
        elif by_label is not None:
            labels = list(dw.cell_labels)
            row = labels.index(by_label) if by_label in labels else -1
        snap = None
        if row >= 0:
            pos = dw.global_positions()[row].tolist()
            lp = dw.cell_positions[row].long().tolist()
            snap = dict(
                idx=int(self._l2g(me)[row]), genome=dw.cell_genomes[row], label=dw.cell_labels[row],
                position=(int(pos[0]), int(pos[1])), life=int(dw.cell_lifetimes[row]), div=int(dw.cell_divisions[row]),
                mol=dw.cell_molecules[row].detach().cpu().clone(), ext=dw.molecule_map[:, lp[0], lp[1]].detach().cpu().clone(),
            )
        hits = [s for s in self._gather(snap) if s is not None]
        if not hits:
            raise ValueError(f"Cell not found (by_idx={by_idx}, by_position={by_position}, by_label={by_label})")
        s = min(hits, key=lambda h: h["idx"])
        return Cell(world=self.dw, genome=s["genome"], position=s["position"], idx=s["idx"], label=s["label"],
                    n_steps_alive=s["life"], n_divisions=s["div"], int_molecules=s["mol"], ext_molecules=s["ext"])

    def get_neighbors(self, cell_idxs: list[int], nghbr_idxs: list[int] | None = None) -> list[tuple[int, int]]:
        """Collective: unique global pairs ``(a, b)``, ``a < b``, of cells in each other's Moore
        neighbourhood on the global torus (reference world.py:247-285)."""
        pos = self.cell_positions.long()
        frm = self._global_idxs(cell_idxs, False)
        to = frm if nghbr_idxs is None else self._global_idxs(nghbr_idxs, False)
        if frm.size == 0 or to.size == 0:
            return []
        S = self.dw.map_size
        occ = {}
        for g in to.tolist():
            occ[(int(pos[g, 0]), int(pos[g, 1]))] = g
        pairs = set()
        for a in frm.tolist():
            x, y = int(pos[a, 0]), int(pos[a, 1])
            for dx in (-1, 0, 1):
                for dy in (-1, 0, 1):
                    if dx == 0 and dy == 0:
                        continue
                    b = occ.get(((x + dx) % S, (y + dy) % S))
                    if b is not None and b != a:
                        pairs.add((min(a, b), max(a, b)))
        return sorted(pairs)

    # ------------------------------------------------------------------ lifecycle
    def spawn_cells(self, genomes: list[str]) -> list[int]:
        """Collective (same ``genomes`` everywhere): new cells on uniformly random free pixels of
        the whole map; returns their global indices (appended at the end, in ``genomes`` order)."""
        self._begin()
        return self._place_new(list(genomes), lambda items: self.dw.spawn_cells(items))

    def add_cells(self, cells: list[Cell]) -> list[int]:
        """Collective (same ``cells`` everywhere): place :class:`Cell` objects on uniformly random
        free pixels of the whole map, keeping genome, label, molecules, lifetime, divisions
        (reference world.py:343-404); returns their global indices."""
        self._begin()
        snap = [_CellRecord.of(c) for c in cells]
        return self._place_new(snap, lambda items: self.dw.add_cells([c.cell(self.dw) for c in items]))

    def _place_new(self, items: list, place) -> list[int]:
        _, order, counts = self._split_counts(len(items))
        lo = [0]
        for c in counts:
            lo.append(lo[-1] + c)
        mine = order[lo[self._me] : lo[self._me + 1]]
        rows = place([items[int(i)] for i in mine]) if mine.size else []
        assert len(rows) == mine.size, "a rank placed fewer cells than its free pixel count allows"
        # global order of the new cells: the order of `items` (restricted to the placed ones)
        got = self._gather([int(r) for r in rows])
        owner = []
        for r in range(self._ws):
            for i, row in zip(order[lo[r] : lo[r + 1]].tolist(), got[r]):
                owner.append((i, r, row))
        owner.sort()
        n0 = self.n_cells
        self._append([o[1] for o in owner], [o[2] for o in owner])
        return list(range(n0, n0 + len(owner)))

    def kill_cells(self, cell_idxs: list[int] | None = None) -> None:
        """Collective: remove cells (molecules spill onto their pixels); later indices shift down."""
        self._begin()
        g = self._global_idxs(cell_idxs, True)
        if g.size == 0:
            return
        mine = self._mine(g)
        if mine.size:
            self.dw.kill_cells(mine.tolist())
        self._drop([np.sort(self._local[g[self._rank[g] == r]]) for r in range(self._ws)])

    def divide_cells(self, cell_idxs: list[int]) -> list[tuple[int, int]]:
        """Collective: divisions into a free Moore neighbour on the global torus (children born
        across a strip boundary included). Returns ``(parent, child)`` global index pairs; the
        children are appended at the end in the order of their parents."""
        self._begin()
        g = self._global_idxs(cell_idxs, False)
        dw = self.dw
        mine = self._mine(g)
        par, ch = dw.divide_cells_t(torch.tensor(mine.tolist(), dtype=torch.long, device=dw.device))
        x = self._xfer()
        x["pairs"] = list(zip(par.tolist(), ch.tolist()))
        x["n"] = int(dw.n_cells)
        info = self._gather(x)
        births = []  # (parent global, child rank, child row)
        for r in range(self._ws):
            l2g = self._l2g(r)
            births += [(int(l2g[p]), r, c) for p, c in info[r]["pairs"]]
            n_in = info[r]["in_up"] + info[r]["in_dn"]
            for i, (sr, srow) in enumerate(self._arrival_sources(info, r)):
                births.append((int(self._l2g(sr)[srow]), r, info[r]["n"] - n_in + i))
        births.sort()
        n0 = self.n_cells
        self._append([b[1] for b in births], [b[2] for b in births])
        return [(b[0], n0 + i) for i, b in enumerate(births)]

    def move_cells(self, cell_idxs: list[int] | None = None) -> None:
        """Collective: every listed cell moves to a random free pixel of its Moore neighbourhood
        (across strip boundaries included); global indices do not change."""
        self._begin()
        g = self._global_idxs(cell_idxs, True)
        dw = self.dw
        mine = self._mine(g)
        dw.move_cells(torch.tensor(mine.tolist(), dtype=torch.long, device=dw.device))
        x = self._xfer()
        x["n"] = int(dw.n_cells)
        info = self._gather(x)
        self._migrated(info)

    def _migrated(self, info: list[dict]) -> None:
        """Table update after cells left rows (``up``/``dn`` exports, removed there) and arrived at
        the end of their new rank: the same global index now points to the new (rank, row)."""
        ws = self._ws
        old_rank, old_local = self._rank.copy(), self._local.copy()
        # where every emigrant lands, keyed by its (sender rank, sender row)
        dest = {}
        for r in range(ws):
            n_in = info[r]["in_up"] + info[r]["in_dn"]
            for i, src in enumerate(self._arrival_sources(info, r)):
                dest[src] = (r, info[r]["n"] - n_in + i)
        moved = np.zeros(old_rank.size, dtype=bool)
        new_rank, new_local = old_rank.copy(), old_local.copy()
        gone = []
        for r in range(ws):
            rows = np.asarray(sorted(info[r]["up"] + info[r]["dn"]), dtype=np.int64)
            gone.append(rows)
            if rows.size:
                l2g = self._l2g(r)
                for row in rows.tolist():
                    gi = int(l2g[row])
                    moved[gi] = True
                    new_rank[gi], new_local[gi] = dest[(r, row)]
        # survivors shift down past the emigrants of their rank; the emigrants keep their entries
        self._drop(gone, keep_global=moved)
        self._rank[moved] = new_rank[moved]
        self._local[moved] = new_local[moved]

    def reposition_cells(self, cell_idxs: list[int] | None = None) -> None:
        """Collective: the listed cells leave their pixels and take uniformly random free pixels
        of the whole map (reference world.py:575-608); a cell may change rank, its index does not."""
        self._begin()
        g = self._global_idxs(cell_idxs, True)
        if g.size == 0:
            return
        dw = self.dw
        sel_counts = [int((self._rank[g] == r).sum()) for r in range(self._ws)]
        # the pixels of the repositioned cells count as free (the reference vacates them first)
        rng, order, counts = self._split_counts(int(g.size), extra_free=sel_counts)
        dest = np.empty(g.size, dtype=np.int32)
        lo = 0
        for r, c in enumerate(counts):
            dest[order[lo : lo + c]] = r
            lo += c
        src = self._rank[g]
        me = self._me
        stay = g[(src == me) & (dest == me)]
        leave = g[(src == me) & (dest != me)]
        if stay.size:
            dw.reposition_cells(np.sort(self._local[stay]).tolist())
        records = []
        if leave.size:
            rows = self._local[leave].tolist()
            genomes, labels = dw.cell_genomes, dw.cell_labels
            mol = dw.cell_molecules[torch.tensor(rows, device=dw.device)].detach().cpu()
            life = dw.cell_lifetimes[torch.tensor(rows, device=dw.device)].tolist()
            div = dw.cell_divisions[torch.tensor(rows, device=dw.device)].tolist()
            records = [(int(gi), _CellRecord(genomes[r], labels[r], mol[i], life[i], div[i]))
                       for i, (gi, r) in enumerate(zip(leave.tolist(), rows))]
            dw._remove(torch.tensor(sorted(rows), dtype=torch.long, device=dw.device))
        allrec = self._gather(records)
        arrivals = sorted((gi, rec) for rr in allrec for gi, rec in rr if dest[np.searchsorted(g, gi)] == me)
        placed = []
        if arrivals:
            placed = dw.add_cells([rec.cell(dw) for _, rec in arrivals])
            assert len(placed) == len(arrivals), "no free pixel left for an arriving cell"
        info = self._gather([(gi, row) for (gi, _), row in zip(arrivals, placed)])
        leavers = [np.sort(self._local[g[(src == r) & (dest != r)]]) for r in range(self._ws)]
        moved = np.zeros(self._rank.size, dtype=bool)
        moved[g[src != dest]] = True
        new_rank = self._rank.copy()
        new_local = self._local.copy()
        for r, lst in enumerate(info):
            for gi, row in lst:
                new_rank[gi], new_local[gi] = r, row
        self._drop(leavers, keep_global=moved)
        self._rank[moved] = new_rank[moved]
        self._local[moved] = new_local[moved]

    def update_cells(self, genome_idx_pairs: list[tuple[str, int]]) -> None:
        """Collective: replace genomes of cells given by global index; proteomes re-derived."""
        self._begin()
        mine = [(gen, int(self._local[i])) for gen, i in genome_idx_pairs if self._rank[i] == self._me]
        self.dw.update_cells(mine)

    # ------------------------------------------------------------------ physics / evolution
    def enzymatic_activity(self) -> None:
        self._begin()
        self.dw.enzymatic_activity()

    def diffuse_molecules(self) -> None:
        self._begin()
        self.dw.diffuse_molecules()

    def degrade_molecules(self) -> None:
        self._begin()
        self.dw.degrade_molecules()

    def increment_cell_lifetimes(self) -> None:
        self._begin()
        self.dw.increment_cell_lifetimes()

    def mutate_cells(self, cell_idxs: list[int] | None = None, p: float = 1e-6, p_indel: float = 0.4,
                     p_del: float = 0.66) -> None:
        """Collective: point mutations of the listed cells (all by default); mutations are
        per-cell, so every rank mutates its own share."""
        self._begin()
        if cell_idxs is None:
            self.dw.mutate_cells(None, p=p, p_indel=p_indel, p_del=p_del)
            self.dw._reconcile()
            return
        mine = self._mine(self._global_idxs(cell_idxs, False))
        if mine.size:
            self.dw.mutate_cells(mine.tolist(), p=p, p_indel=p_indel, p_del=p_del)

    def recombinate_cells(self, cell_idxs: list[int] | None = None, p: float = 1e-7) -> None:
        """Collective: recombination between neighbouring cells of the listed set (all by default),
        pairs across strip boundaries included."""
        self._begin()
        if cell_idxs is None:
            self.dw.recombinate_cells(None, p=p)
        else:
            self.dw.recombinate_cells(self._mine(self._global_idxs(cell_idxs, False)).tolist(), p=p)
        self.dw._reconcile()

    def __repr__(self) -> str:
        return f"GlobalWorld(n_cells:{self.n_cells},{self.dw!r})"


class _CellRecord:
    """A cell's transferable state (picklable, world-free)."""

    __slots__ = ("genome", "label", "mol", "life", "div")

    def __init__(self, genome: str, label: str, mol: torch.Tensor, life: int, div: int):
        self.genome, self.label, self.mol, self.life, self.div = genome, label, mol, int(life), int(div)

    @classmethod
    def of(cls, c: Cell) -> "_CellRecord":
        return cls(c.genome, c.label, torch.as_tensor(c.int_molecules).detach().cpu().clone(), c.n_steps_alive, c.n_divisions)

    def __lt__(self, other: "_CellRecord") -> bool:  # (sorting (index, record) tuples never ties)
        return False

    def cell(self, world) -> Cell:
        return Cell(world=world, genome=self.genome, label=self.label, n_steps_alive=self.life, n_divisions=self.div,
                    int_molecules=self.mol)
