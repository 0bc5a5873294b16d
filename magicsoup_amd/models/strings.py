"""Device-resident string columns: genomes and labels of all cells.

The reference keeps ``world.cell_genomes`` / ``world.cell_labels`` as Python ``list[str]``
(``world.py:192-194``) and copies every genome across the Rust FFI on each mutation step. Here the
strings live on the world's device: GPU genomes in a ragged byte pool (:class:`PoolArena`: per-cell
offsets and lengths, no padding, shared between a parent and its children), labels and CPU genomes
in a row arena (:class:`StringArena`: one row of ``width`` bytes per cell plus a length, what the
OpenMP host core works on). Translation, mutation, recombination, division and compaction kernels
work on them in place. ``StringColumn`` is the list-like view users see: indexing, iteration, comparison and
assignment materialise / upload only what is touched, and a full materialisation is cached until the
arena changes.
"""
from __future__ import annotations

from typing import Iterable, Iterator

import numpy as np
import torch

_MIN_WIDTH = 16


def _round_width(n: int) -> int:
    w = _MIN_WIDTH
    while w < n:
        w *= 2 if w < 4096 else 1.25
        w = int(w + 15) // 16 * 16
    return w


def pack_strings(strs: list[str], width: int | None = None) -> tuple[np.ndarray, np.ndarray]:
    """Pack strings into a zero-padded uint8 array (n, width) and int32 lengths: one join + encode
    of all strings and one native pass writing the rows (host core ``pack_rows``)."""
    strs = strs if isinstance(strs, list) else list(strs)
    lens = np.fromiter(map(len, strs), dtype=np.int32, count=len(strs))
    w = int(lens.max()) if len(strs) else 0
    width = max(width or 0, _round_width(max(w, 1)))
    joined = "".join(strs).encode("ascii")
    if len(joined) != int(lens.sum(dtype=np.int64)):
        raise ValueError("genomes and labels must be ASCII strings")
    from magicsoup_amd.ops import native

    return native.host().pack_rows(joined, lens, width), lens


class StringArena:
    """Rows of bytes with per-row lengths and a row capacity (amortised O(1) appends)."""

    def __init__(self, device, width: int = 64, capacity: int = 0):
        self.device = torch.device(device)
        self.width = _round_width(width)
        self.data = torch.zeros(capacity, self.width, dtype=torch.uint8, device=self.device)
        self.lens = torch.zeros(capacity, dtype=torch.int32, device=self.device)
        self.n = 0
        self.version = 0

    # ---------------------------------------------------------------- capacity
    @property
    def capacity(self) -> int:
        return int(self.data.size(0))

    def reserve(self, rows: int, width: int | None = None) -> None:
        width = self.width if width is None or _round_width(width) <= self.width else _round_width(width)
        if rows <= self.capacity and width == self.width:
            return
        cap = max(rows, int(self.capacity * 1.5) + 16) if rows > self.capacity else self.capacity
        data = torch.zeros(cap, width, dtype=torch.uint8, device=self.device)
        lens = torch.zeros(cap, dtype=torch.int32, device=self.device)
        if self.n:
            data[: self.n, : self.width] = self.data[: self.n]
            lens[: self.n] = self.lens[: self.n]
        _retire(self.data)
        _retire(self.lens)
        self.data, self.lens, self.width = data, lens, width
        self.version += 1

    # ---------------------------------------------------------------- bulk ops
    def append_packed(self, rows: torch.Tensor, lens: torch.Tensor) -> None:
        k = int(rows.size(0))
        if k == 0:
            return
        self.reserve(self.n + k, int(rows.size(1)))
        self.data[self.n : self.n + k, : rows.size(1)] = rows.to(self.device)
        if rows.size(1) < self.width:
            self.data[self.n : self.n + k, rows.size(1) :] = 0
        self.lens[self.n : self.n + k] = lens.to(self.device, torch.int32)
        self.n += k
        self.version += 1

    def append_strings(self, strs: list[str]) -> None:
        if not strs:
            return
        arr, lens = pack_strings(strs)
        self.append_packed(torch.from_numpy(arr), torch.from_numpy(lens))

    def append_rows_from(self, src_rows: torch.Tensor) -> None:
        """Append copies of existing rows (e.g. children inherit their parent's genome)."""
        k = int(src_rows.numel())
        if k == 0:
            return
        self.reserve(self.n + k)
        src_rows = src_rows.to(self.device, torch.long)
        self.data[self.n : self.n + k] = self.data[src_rows]
        self.lens[self.n : self.n + k] = self.lens[src_rows]
        self.n += k
        self.version += 1

    def set_rows(self, rows: torch.Tensor, packed: torch.Tensor, lens: torch.Tensor) -> None:
        if rows.numel() == 0:
            return
        self.reserve(self.n, int(packed.size(1)))
        rows = rows.to(self.device, torch.long)
        w = int(packed.size(1))
        self.data[rows, :w] = packed.to(self.device)
        if w < self.width:
            self.data[rows, w:] = 0
        self.lens[rows] = lens.to(self.device, torch.int32)
        self.version += 1

    def set_strings(self, rows: list[int], strs: list[str]) -> None:
        if not rows:
            return
        arr, lens = pack_strings(strs)
        self.set_rows(torch.tensor(rows, dtype=torch.long), torch.from_numpy(arr), torch.from_numpy(lens))

    def keep(self, keep_idx: torch.Tensor) -> None:
        """Order-preserving compaction to the rows ``keep_idx`` (ascending long indices)."""
        k = int(keep_idx.numel())
        self.data[:k] = self.data[keep_idx]
        self.lens[:k] = self.lens[keep_idx]
        self.n = k
        self.version += 1

    def clear(self) -> None:
        self.n = 0
        self.version += 1

    # ---------------------------------------------------------------- fused row movement (device)
    def compact_pairs(self, k: int) -> list[tuple[torch.Tensor, torch.Tensor]]:
        """(source, target) row tensors for an order-preserving compaction to ``k`` rows into the
        spare buffers (see :meth:`commit_compact`)."""
        sp = self.__dict__.get("_spare")
        cap = max(k, self.capacity)
        if sp is None or sp[0].size(0) < cap or sp[0].size(1) != self.width or sp[0].device != self.data.device:
            sp = (torch.empty(cap, self.width, dtype=torch.uint8, device=self.device),
                  torch.empty(cap, dtype=torch.int32, device=self.device))
            self.__dict__["_spare"] = sp
        # genome rows: only the used bytes move (bytes past a row's length are never read)
        return [(self.data[: self.n], sp[0][:k], self.lens), (self.lens[: self.n], sp[1][:k])]

    def commit_compact(self, k: int) -> None:
        sd, sl = self.__dict__.pop("_spare")
        self.__dict__["_spare"] = (self.data, self.lens)
        self.data, self.lens = sd, sl
        self.n = k
        self.version += 1

    def clone_pairs(self, k: int) -> list[tuple[torch.Tensor, torch.Tensor]]:
        """Append ``k`` rows and return in-place (source, target) row tensors covering old and new
        rows, for copying existing rows into the new ones."""
        self.reserve(self.n + k)
        self.n += k
        self.version += 1
        return [(self.data[: self.n], self.data[: self.n], self.lens), (self.lens[: self.n], self.lens[: self.n])]

    def view(self) -> tuple[torch.Tensor, torch.Tensor]:
        return self.data[: self.n], self.lens[: self.n]

    def rows_of(self, cells: torch.Tensor | None, width: int | None = None) -> torch.Tensor:
        """Rows of ``cells`` (all when None), cut or zero-padded to ``width`` (default: the row width)."""
        rows = self.data[: self.n] if cells is None else self.data[cells.to(self.device, torch.long)]
        w = self.width if width is None else int(width)
        if w <= rows.size(1):
            return rows[:, :w]
        return torch.nn.functional.pad(rows, (0, w - rows.size(1)))

    # ---------------------------------------------------------------- materialisation
    def packed(self, rows: Iterable[int] | None = None) -> tuple[np.ndarray, np.ndarray]:
        """The strings of all rows (or of ``rows``) back to back as host bytes (uint8) plus their
        lengths (int64): the rows, cut to the longest string, are copied to the host in one transfer
        and the host core concatenates their used bytes (checkpoint shards store this layout)."""
        if rows is None:
            data, lens = self.data[: self.n], self.lens[: self.n]
        else:
            idx = torch.as_tensor(list(rows), dtype=torch.long, device=self.device)
            data, lens = self.data[idx], self.lens[idx]
        ls = lens.cpu().numpy().astype(np.int64)
        lmax = int(ls.max()) if ls.size else 0
        if data.numel() == 0 or lmax == 0:
            return np.zeros(0, dtype=np.uint8), np.zeros(ls.size, dtype=np.int64)
        from magicsoup_amd.ops import native

        sub = data[:, :lmax].contiguous().cpu().numpy()
        raw = native.host().unpack_rows(sub, ls.astype(np.int32))
        return np.frombuffer(raw, dtype=np.uint8), ls

    def to_strings(self, rows: Iterable[int] | None = None) -> list[str]:
        """The strings of all rows (or of ``rows``): :meth:`packed`, decoded once; the strings are
        slices of that buffer."""
        buf, ls = self.packed(rows)
        return _split(buf, ls)


_POOL_MIN = 16 << 20  # bytes


def _split(buf: np.ndarray, lens: np.ndarray) -> list[str]:
    """Strings of the given lengths, back to back in ``buf`` (ASCII): one decode, then slices."""
    if buf.size == 0:
        return [""] * int(lens.size)
    raw = str(memoryview(buf), "ascii")
    ends = np.cumsum(lens, dtype=np.int64).tolist()
    starts = [0] + ends[:-1]
    return [raw[a:b] for a, b in zip(starts, ends)]


def _r16(n: int) -> int:
    return (int(n) + 15) // 16 * 16


def _retire(t: torch.Tensor | None) -> None:
    """A device tensor about to be dropped while work on the current stream may still read it (a
    copy out of it was just queued): its block returns to the caching allocator only after that
    work, even if the tensor was allocated on another stream."""
    if t is not None and t.is_cuda:
        t.record_stream(torch.cuda.current_stream(t.device))


class PoolArena:
    """GPU genomes of every length in one byte pool (``csrc/hip/pool.hip``).

    Cell i's genome is the ``lens[i]`` bytes at ``data[off[i]:]``. Storage is taken by an atomic bump
    of the device counter ``top`` (16-byte aligned) and never written again: mutated or recombined
    genomes get new space (the device pipeline's commit), a dividing cell's child shares its parent's
    bytes (only ``off`` / ``lens`` are cloned), a kill compacts ``off`` / ``lens`` only. Nothing is as
    wide as the longest genome: one 20 kbp genome costs 20 kB, and no event re-lays the population
    out (the reference keeps one Python string per cell, ``world.py:192-194``).

    ``width`` is not a row width but the genome length bound the device pipeline sizes its scratch
    for: a result longer than it is committed on the host at reconcile (which raises the bound, an
    O(1) change). ``top_ub`` is the host's upper bound of the device counter; :meth:`ensure` collects
    (:meth:`collect`: unreferenced space is dropped, shared genomes stay shared) or grows the pool
    before an allocation could overrun it. Callers collect only with no device work pending on the
    pool (the World reconciles its genome pipeline first)."""

    def __init__(self, device, width: int = 64, capacity: int = 0):
        self.device = torch.device(device)
        self.width = _round_width(width)
        self.lens = torch.zeros(capacity, dtype=torch.int32, device=self.device)
        self.off = torch.zeros(capacity, dtype=torch.int64, device=self.device)
        self.data = torch.empty(_POOL_MIN, dtype=torch.uint8, device=self.device)
        self.top = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.failed = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._top_ub = 0
        self.inc_total = 0  # every raise of top_ub so far (genome_pipeline's pool mirror bound)
        self.collects = 0  # pool replacements (collect / clear): a mirrored device top is void after one
        self.n = 0
        self.version = 0

    def __setstate__(self, state: dict) -> None:
        # (states saved before the bound tracking carry a plain ``top_ub``)
        if "top_ub" in state:
            state["_top_ub"] = state.pop("top_ub")
        state.setdefault("inc_total", 0)
        state.setdefault("collects", 0)
        self.__dict__.update(state)

    @property
    def top_ub(self) -> int:
        return self._top_ub

    @top_ub.setter
    def top_ub(self, v: int) -> None:
        if v > self._top_ub:
            self.inc_total += v - self._top_ub
        self._top_ub = v

    # ---------------------------------------------------------------- capacity
    @property
    def capacity(self) -> int:
        return int(self.lens.size(0))

    @property
    def pool_cap(self) -> int:
        return int(self.data.numel())

    def args(self):
        """The pool as the kernels take it (GenomePoolArgs)."""
        from magicsoup_amd.ops import native

        a = native.hip().GenomePoolArgs()
        a.pool, a.off, a.top = self.data.data_ptr(), self.off.data_ptr(), self.top.data_ptr()
        a.failed, a.cap = self.failed.data_ptr(), self.pool_cap
        return a

    def reserve(self, rows: int, width: int | None = None) -> None:
        """Room for ``rows`` cells; ``width`` raises the genome length bound (no data moves). The
        bound follows the longest genome closely (64-multiples), not in powers of two: the device
        pipeline's gates and scratch scale with it."""
        if width is not None and int(width) > self.width:
            self.width = (int(width) + 63) // 64 * 64
        if rows <= self.capacity:
            return
        cap = max(rows, int(self.capacity * 1.5) + 16)
        lens = torch.zeros(cap, dtype=torch.int32, device=self.device)
        off = torch.zeros(cap, dtype=torch.int64, device=self.device)
        if self.n:
            lens[: self.n] = self.lens[: self.n]
            off[: self.n] = self.off[: self.n]
        _retire(self.lens)
        _retire(self.off)
        self.lens, self.off = lens, off
        self.__dict__.pop("_spare", None)
        self.version += 1

    def ensure(self, need: int) -> None:
        """Room for ``need`` more bytes of allocations: first a re-read of the device counter (the host
        bound adds worst cases), then a collection / growth of the pool."""
        if self.top_ub + need <= self.pool_cap:
            return
        self.top_ub = int(self.top.item())
        if self.top_ub + need <= self.pool_cap:
            return
        self.collect(need)

    def collect(self, extra: int = 0) -> None:
        """Move the referenced genomes into a fresh pool (each distinct genome once, in offset order)
        with room for ``extra`` more bytes; unreferenced space is dropped. Two synchronisations (the top, the new total)."""
        from magicsoup_amd.ops import native
        from magicsoup_amd.ops.hip_ops import _stream

        n = self.n
        self.collects += 1
        if n == 0:
            self.data = torch.empty(max(_POOL_MIN, 2 * _r16(extra)), dtype=torch.uint8, device=self.device)
            self.top.zero_()
            self.top_ub = 0
            return
        # on the device (pool.hip pool_collect_plan / _move): per 16-byte granule below the top, the
        # size of the allocation starting there (the longest genome naming it, at least one granule,
        # as pool_alloc) and its owner cell, a scan of the sizes (the new offsets, in old-offset
        # order), then the owners copy and every cell takes its new offset
        m = native.hip()
        st = _stream()
        G = max(1, (int(self.top.item()) + 15) // 16)
        dev = self.device
        size_g = torch.empty(G, dtype=torch.int32, device=dev)
        owner_g = torch.empty(G, dtype=torch.int32, device=dev)
        new_g = torch.empty(G, dtype=torch.int32, device=dev)
        tile_sum = torch.empty((G + 1023) // 1024, dtype=torch.int64, device=dev)
        total_g = torch.empty(1, dtype=torch.int64, device=dev)
        m.pool_collect_plan(n, self.off.data_ptr(), self.lens.data_ptr(), G, size_g.data_ptr(), owner_g.data_ptr(),
                            new_g.data_ptr(), tile_sum.data_ptr(), total_g.data_ptr(), st)
        total = 16 * int(total_g.item())
        cap = max(_POOL_MIN, 2 * (total + _r16(extra)))
        new = torch.empty(cap, dtype=torch.uint8, device=dev)
        m.pool_collect_move(n, self.off.data_ptr(), self.data.data_ptr(), new.data_ptr(), size_g.data_ptr(),
                            owner_g.data_ptr(), new_g.data_ptr(), st)
        for t in (self.data, size_g, owner_g, new_g):
            _retire(t)
        self.data = new
        self.top.fill_(total)
        self.top_ub = total
        self.version += 1

    def _write(self, rows: torch.Tensor, lens: torch.Tensor, dst: torch.Tensor | None, n0: int) -> None:
        """Genome rows (k, L) -> new allocations of cells ``dst`` (or n0 + j)."""
        from magicsoup_amd.ops import native
        from magicsoup_amd.ops.hip_ops import _stream

        k, L = int(rows.size(0)), int(rows.size(1))
        if k == 0:
            return
        # the length bound tracks the longest genome, not the row stride (pack_strings pads rows to a
        # power of two): lengths still on the host are read for free, device ones would cost a sync
        bound = int(lens.max()) if not lens.is_cuda else L
        rows = rows.to(self.device, torch.uint8).contiguous()
        lens = lens.to(self.device, torch.int32).contiguous()
        self.reserve(self.capacity if dst is not None else n0 + k, max(bound, 1))
        need = k * _r16(L)
        self.ensure(need)
        dst = None if dst is None else dst.to(self.device, torch.int64).contiguous()
        native.hip().pool_write(k, L, rows.data_ptr(), lens.data_ptr(), 0 if dst is None else dst.data_ptr(), n0,
                                self.data.data_ptr(), self.off.data_ptr(), self.top.data_ptr(), self.pool_cap,
                                self.lens.data_ptr(), self.failed.data_ptr(), _stream())
        self.top_ub += need

    def check(self) -> None:
        """Raise if an allocation ever found the pool full (a sizing bug; one read of the flag)."""
        if int(self.failed.item()):
            raise RuntimeError("genome pool overflow: an allocation found the pool full")

    # ---------------------------------------------------------------- bulk ops (StringArena's interface)
    def append_packed(self, rows: torch.Tensor, lens: torch.Tensor) -> None:
        k = int(rows.size(0))
        if k == 0:
            return
        self.reserve(self.n + k, int(rows.size(1)))
        self._write(rows, lens, None, self.n)
        self.n += k
        self.version += 1

    def append_strings(self, strs: list[str]) -> None:
        if not strs:
            return
        arr, lens = pack_strings(strs)
        self.append_packed(torch.from_numpy(arr), torch.from_numpy(lens))

    def append_rows_from(self, src_rows: torch.Tensor) -> None:
        """Append cells sharing the genomes of ``src_rows`` (children inherit their parent's)."""
        k = int(src_rows.numel())
        if k == 0:
            return
        self.reserve(self.n + k)
        src_rows = src_rows.to(self.device, torch.long)
        self.off[self.n : self.n + k] = self.off[src_rows]
        self.lens[self.n : self.n + k] = self.lens[src_rows]
        self.n += k
        self.version += 1

    def set_rows(self, rows: torch.Tensor, packed: torch.Tensor, lens: torch.Tensor) -> None:
        if rows.numel() == 0:
            return
        self._write(packed, lens, rows.to(torch.int64), 0)
        self.version += 1

    def set_strings(self, rows: list[int], strs: list[str]) -> None:
        if not rows:
            return
        arr, lens = pack_strings(strs)
        self.set_rows(torch.tensor(rows, dtype=torch.long), torch.from_numpy(arr), torch.from_numpy(lens))

    def keep(self, keep_idx: torch.Tensor) -> None:
        k = int(keep_idx.numel())
        self.off[:k] = self.off[keep_idx]
        self.lens[:k] = self.lens[keep_idx]
        self.n = k
        self.version += 1

    def clear(self) -> None:
        self.n = 0
        self.top.zero_()
        self.collects += 1
        self.top_ub = 0
        self.version += 1

    # ---------------------------------------------------------------- fused row movement (device)
    def compact_pairs(self, k: int) -> list[tuple[torch.Tensor, torch.Tensor]]:
        """(source, target) per-cell tensors (offsets, lengths) of an order-preserving compaction to
        ``k`` cells into the spares (see :meth:`commit_compact`); no genome byte moves."""
        sp = self.__dict__.get("_spare")
        cap = max(k, self.capacity)
        if sp is None or sp[0].size(0) < cap or sp[0].device != self.off.device:
            sp = (torch.empty(cap, dtype=torch.int64, device=self.device),
                  torch.empty(cap, dtype=torch.int32, device=self.device))
            self.__dict__["_spare"] = sp
        return [(self.off[: self.n], sp[0][:k]), (self.lens[: self.n], sp[1][:k])]

    def commit_compact(self, k: int) -> None:
        so, sl = self.__dict__.pop("_spare")
        self.__dict__["_spare"] = (self.off, self.lens)
        self.off, self.lens = so, sl
        self.n = k
        self.version += 1

    def clone_pairs(self, k: int) -> list[tuple[torch.Tensor, torch.Tensor]]:
        """Append ``k`` cells; in-place (source, target) offset / length tensors over old and new
        cells for cloning existing cells' entries into the new ones (shared genomes)."""
        self.reserve(self.n + k)
        self.n += k
        self.version += 1
        return [(self.off[: self.n], self.off[: self.n]), (self.lens[: self.n], self.lens[: self.n])]

    def rows_of(self, cells: torch.Tensor | None, width: int | None = None) -> torch.Tensor:
        """Genomes of ``cells`` (all when None) as zero-padded uint8 rows (k, width) on the device
        (width: the longest of them, rounded up to 16, unless given)."""
        from magicsoup_amd.ops import native
        from magicsoup_amd.ops.hip_ops import _stream

        idx = None if cells is None else cells.to(self.device, torch.int64).contiguous()
        k = self.n if idx is None else int(idx.numel())
        if width is None:
            ls = self.lens[: self.n] if idx is None else self.lens[idx]
            width = _r16(int(ls.max().item())) if k else 16
        out = torch.empty(k, max(int(width), 1), dtype=torch.uint8, device=self.device)
        if k:
            native.hip().pool_read(k, 0 if idx is None else idx.data_ptr(), self.data.data_ptr(), self.off.data_ptr(),
                                   self.lens.data_ptr(), out.data_ptr(), int(out.size(1)), _stream())
        return out

    def view(self) -> tuple[torch.Tensor, torch.Tensor]:
        """(rows (n, width), lengths) -- padded copies of the genomes (the pool holds no rows)."""
        return self.rows_of(None), self.lens[: self.n]

    # ---------------------------------------------------------------- materialisation
    def packed(self, rows: Iterable[int] | None = None) -> tuple[np.ndarray, np.ndarray]:
        """The genomes of all cells (or of ``rows``) back to back as host bytes (uint8) plus their
        lengths (int64): gathered on the device at an exclusive prefix sum of the lengths, then one
        transfer of exactly their bytes (checkpoint shards store this layout)."""
        idx = None if rows is None else torch.as_tensor(list(rows), dtype=torch.long, device=self.device)
        lens = self.lens[: self.n] if idx is None else self.lens[idx]
        ls = lens.cpu().numpy().astype(np.int64)
        k = int(ls.size)
        if k == 0 or int(ls.max()) == 0:
            return np.zeros(0, dtype=np.uint8), ls
        from magicsoup_amd.ops import native
        from magicsoup_amd.ops.hip_ops import _stream

        ends_np = np.cumsum(ls, dtype=np.int64)
        total = int(ends_np[-1])
        dst_off = torch.from_numpy(ends_np - ls).to(self.device)
        out = torch.empty(max(total, 1), dtype=torch.uint8, device=self.device)
        native.hip().pool_read_packed(k, 0 if idx is None else idx.data_ptr(), self.data.data_ptr(),
                                      self.off.data_ptr(), self.lens.data_ptr(), dst_off.data_ptr(), out.data_ptr(),
                                      _stream())
        return out[:total].cpu().numpy(), ls

    def to_strings(self, rows: Iterable[int] | None = None) -> list[str]:
        """One :meth:`packed` transfer, one decode; the strings are slices of it."""
        buf, ls = self.packed(rows)
        return _split(buf, ls)


class StringColumn:
    """``list[str]``-like view of a :class:`StringArena` (``world.cell_genomes`` / ``cell_labels``)."""

    def __init__(self, arena: StringArena):
        self._arena = arena
        self._cache: list[str] | None = None
        self._cache_version = -1

    def _all(self) -> list[str]:
        a = self._arena
        if self._cache is None or self._cache_version != a.version:
            self._cache = a.to_strings()
            self._cache_version = a.version
        return self._cache

    def __len__(self) -> int:
        return self._arena.n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return self._all()[i]
        n = self._arena.n
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError("cell index out of range")
        if self._cache is not None and self._cache_version == self._arena.version:
            return self._cache[i]
        return self._arena.to_strings([i])[0]

    def __setitem__(self, i: int, value: str) -> None:
        n = self._arena.n
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError("cell index out of range")
        cached = self._cache is not None and self._cache_version == self._arena.version
        self._arena.set_strings([i], [value])
        if cached:
            self._cache[i] = value  # type: ignore[index]
            self._cache_version = self._arena.version

    def __iter__(self) -> Iterator[str]:
        return iter(self._all())

    def __contains__(self, item) -> bool:
        return item in self._all()

    def __eq__(self, other) -> bool:
        if isinstance(other, StringColumn):
            other = other._all()
        if isinstance(other, (list, tuple)):
            return self._all() == list(other)
        return NotImplemented

    def __repr__(self) -> str:
        return repr(self._all())

    def index(self, value: str, *args) -> int:
        return self._all().index(value, *args)

    def count(self, value: str) -> int:
        return self._all().count(value)

    def copy(self) -> list[str]:
        return list(self._all())

    def tolist(self) -> list[str]:
        return list(self._all())

    # list mutators kept for code written against the reference's plain lists
    def append(self, value: str) -> None:
        self._arena.append_strings([value])

    def extend(self, values: Iterable[str]) -> None:
        self._arena.append_strings(list(values))

    def pop(self, i: int = -1) -> str:
        n = self._arena.n
        if i < 0:
            i += n
        val = self[i]
        keep = torch.tensor([j for j in range(n) if j != i], dtype=torch.long, device=self._arena.device)
        self._arena.keep(keep)
        return val
