"""Device-resident string columns: genomes and labels of all cells.

The reference keeps ``world.cell_genomes`` / ``world.cell_labels`` as Python ``list[str]``
(``world.py:192-194``) and copies every genome across the Rust FFI on each mutation step. Here the
strings live in a byte arena on the world's device — one row of ``width`` bytes per cell plus a
length — so translation, mutation, recombination, division and compaction kernels work on them in
place. ``StringColumn`` is the list-like view users see: indexing, iteration, comparison and
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

    # ---------------------------------------------------------------- materialisation
    def to_strings(self, rows: Iterable[int] | None = None) -> list[str]:
        """The strings of all rows (or of ``rows``): the rows (cut to the longest string) are copied
        to the host in one transfer, the host core concatenates their used bytes, and that buffer is
        decoded once; the strings are slices of it."""
        if rows is None:
            data, lens = self.data[: self.n], self.lens[: self.n]
        else:
            idx = torch.as_tensor(list(rows), dtype=torch.long, device=self.device)
            data, lens = self.data[idx], self.lens[idx]
        if data.numel() == 0:
            return [""] * int(lens.numel())
        ls = lens.cpu()
        lmax = int(ls.max()) if ls.numel() else 0
        if lmax == 0:
            return [""] * int(ls.numel())
        from magicsoup_amd.ops import native

        # rows cut to the longest string, one transfer; the host core concatenates the used bytes
        sub = data[:, :lmax].contiguous().cpu().numpy()
        raw = native.host().unpack_rows(sub, ls.numpy().astype(np.int32, copy=False)).decode("ascii")
        ends = np.cumsum(ls.numpy(), dtype=np.int64).tolist()
        starts = [0] + ends[:-1]
        return [raw[a:b] for a, b in zip(starts, ends)]


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
