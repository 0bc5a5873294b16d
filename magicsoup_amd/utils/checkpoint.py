"""Checkpoint / resume.

* ``save_state`` / ``load_state`` keep the reference's on-disk format (``world.py:795-878``):
  ``cell_molecules.pt``, ``cell_map.pt``, ``molecule_map.pt``, ``cell_lifetimes.pt``,
  ``cell_positions.pt``, ``cell_divisions.pt`` (``torch.save`` of the tensors) and ``cells.fasta``
  with entries ``>{idx} {label}\\n{genome}``. States from either implementation load in the other.
  Tensors are written from host copies and loaded with ``weights_only=True``.
* ``rng_state.pt`` (new; the reference ignores unknown files and keeps no RNG state, SURVEY §2.8
  item 9) holds every random stream a step draws from: the device and host native streams
  (seed, calls drawn), torch's CPU / device generators, the placement helper's generator and
  Python's ``random``. ``load_state(restore_rng=True)`` restores it (opt-in: by default, like the
  reference, loading a state leaves every random stream alone, so replicate runs started from one
  checkpoint diverge), and then save -> load -> N steps equals N uninterrupted steps (``tests/test_world.py::test_save_load_state_resumes_rng_streams``).
* ``load_world_pickle`` restores :meth:`World.save` pickles -- this package's own and the
  reference's (``magicsoup.world.World`` with ``Conv2d`` diffusion kernels, ``world.py:161-204``) --
  through a restricted unpickler: only an explicit list of data classes (World, Chemistry,
  Molecule, Genetics, Kinetics and its map factories, the domain containers), torch's tensor /
  parameter rebuild functions, dtypes and storages and a few builtin containers can be named by
  the file, and only the rebuild functions and plain containers can be called by it; tensor storages are read with ``torch.load(weights_only=True)`` onto the
  requested device, like the reference's ``_CPU_Unpickler`` (``world.py:17-33``) but without
  executing anything else from the file. Reference pickles are converted to this package's layout
  (``reference_world_state`` / ``reference_kinetics_state``). No reference pickle ships with the
  reference repository, so that path is covered by a hand-built pickle of the same structure
  (parity unpinned, ``tests/test_world.py::test_from_file_reads_reference_layout_pickle``).
"""
from __future__ import annotations

import collections
import io
import pickle
import random
from pathlib import Path

import numpy as np
import torch

_FILES = ("cell_molecules", "cell_map", "molecule_map", "cell_lifetimes", "cell_positions", "cell_divisions")
RNG_FILE = "rng_state.pt"


def save_state(world, statedir: Path) -> None:
    statedir.mkdir(parents=True, exist_ok=True)
    for name in _FILES:
        t = getattr(world, name).detach().cpu()
        if name == "molecule_map":
            t = t.to(torch.float32)  # checkpoints always hold fp32 maps, whatever the storage dtype
        torch.save(t.clone(), statedir / f"{name}.pt")
    # genomes and labels go from the arenas to the file as packed bytes (host core fasta_write: no
    # Python string per cell); the text is the reference's, entries joined by "\n"
    g, gl = world._genomes.packed()
    lab, ll = world._labels.packed()
    _host().fasta_write(str(statedir / "cells.fasta"), 0, g, gl, lab, ll)
    torch.save(rng_state(world.device), statedir / RNG_FILE)


def _host():
    from magicsoup_amd.ops import native

    return native.host()


def read_fasta_packed(path: Path) -> tuple:
    """(genome bytes, genome lengths, label bytes, label lengths) of a ``cells.fasta`` -- the
    reference's parsing rules (``world.py:853-866``), in the host core."""
    return _host().fasta_parse(str(path))


def packed_rows(buf, lens, idx=None) -> tuple[torch.Tensor, torch.Tensor]:
    """Zero-padded uint8 rows (k, width) + int32 lengths of the strings ``idx`` (all when None) of
    a packed buffer: what the arenas' ``append_packed`` takes."""
    buf = np.asarray(buf, dtype=np.uint8)
    lens = np.asarray(lens, dtype=np.int64)
    if idx is not None:
        idx = np.asarray(idx, dtype=np.int64)
        starts = np.cumsum(lens) - lens
        sl = lens[idx]
        total = int(sl.sum())
        if total:
            # byte j of the selection: its string's start + its position within the string
            rep = np.repeat(starts[idx] - (np.cumsum(sl) - sl), sl)
            buf = buf[rep + np.arange(total, dtype=np.int64)]
        else:
            buf = np.zeros(0, dtype=np.uint8)
        lens = sl
    width = max(16, (int(lens.max()) + 15) // 16 * 16 if lens.size else 16)
    rows = _host().pack_rows(buf.tobytes(), lens.astype(np.int32), width)
    return torch.from_numpy(rows), torch.from_numpy(lens.astype(np.int32))


def rng_state(device) -> dict:
    """Every random stream a world op draws from, as plain ints / tensors (``weights_only``-safe)."""
    from magicsoup_amd.ops import native, world_ops

    st = {
        "host": list(native.host().get_rng_state()),
        "torch_cpu": torch.get_rng_state(),
        "placement_cpu": world_ops._gen_cpu.get_state(),
        "python": _py_state_to_list(random.getstate()),
    }
    dev = torch.device(device)
    if dev.type == "cuda":
        st["hip"] = list(native.hip().get_rng_state())
        st["torch_cuda"] = torch.cuda.get_rng_state(dev)
    return st


def set_rng_state(st: dict, device) -> None:
    """Restore :func:`rng_state` (entries for a device type this process does not use are skipped)."""
    from magicsoup_amd.ops import native, world_ops

    native.host().set_rng_state(*[int(x) for x in st["host"]])
    torch.set_rng_state(st["torch_cpu"])
    world_ops._gen_cpu.set_state(st["placement_cpu"])
    random.setstate(_py_state_from_list(st["python"]))
    dev = torch.device(device)
    if dev.type == "cuda" and "hip" in st:
        native.hip().set_rng_state(*[int(x) for x in st["hip"]])
        torch.cuda.set_rng_state(st["torch_cuda"], dev)


def _py_state_to_list(s) -> list:
    version, internal, gauss = s
    return [int(version), [int(x) for x in internal], gauss]


def _py_state_from_list(v) -> tuple:
    return (int(v[0]), tuple(int(x) for x in v[1]), v[2])


def _parse_fasta(text: str) -> tuple[list[str], list[str]]:
    genomes, labels = [], []
    for entry in (e.strip() for e in text.split(">")):
        if not entry:
            continue
        parts = entry.split("\n")
        names = parts[0].split()
        labels.append(names[1].strip() if len(names) > 1 else "")
        genomes.append(parts[1] if len(parts) > 1 else "")
    return genomes, labels


def load_state(world, statedir: Path, ignore_cell_params: bool = False, restore_rng: bool = False) -> None:
    if world.n_cells > 0:
        world.kill_cells()
    dev = torch.device(world.device)

    def ld(name):
        return torch.load(statedir / f"{name}.pt", map_location=dev, weights_only=True)

    g, gl, lab, ll = read_fasta_packed(statedir / "cells.fasta")
    n = int(gl.size)
    cell_map = ld("cell_map").bool()
    world.molecule_map = ld("molecule_map").to(torch.float32).contiguous()
    world.cell_map = cell_map
    world.n_cells = 0
    world._grow(n)
    world.cell_molecules[:] = ld("cell_molecules").float()
    world.cell_lifetimes[:] = ld("cell_lifetimes").int()
    world.cell_positions[:] = ld("cell_positions").int()
    world.cell_divisions[:] = ld("cell_divisions").int()
    world._genomes.clear()
    world._labels.clear()
    if n:
        world._genomes.append_packed(*packed_rows(g, gl))
        world._labels.append_packed(*packed_rows(lab, ll))
    if not ignore_cell_params and n > 0:
        world._update_params_rows(torch.arange(n, device=dev))
    rng_file = statedir / RNG_FILE
    if restore_rng and rng_file.exists():
        set_rng_state(torch.load(rng_file, map_location="cpu", weights_only=True), world.device)


# ---------------------------------------------------------------------------- decomposed worlds
# A DistributedWorld checkpoints as one shard per rank, written by every rank at the same time from
# its own device memory (no gather through one process, no CPU World, no re-translation): the
# strip's owned map rows, its cells' columns with global positions, genomes and labels as packed
# bytes straight from the arenas, and the rank's random streams. ``assemble_state`` turns the
# shards into the reference layout (the files ``save_state`` writes) -- by rank 0 right after the
# save, or offline later for worlds whose global map rank 0 should not hold. Loading takes the
# shards directly when the rank count matches, and otherwise each rank reads only its strip of the
# reference files (memory-mapped map rows, its cells from the FASTA).
SHARD_DIR = "shards"
SHARD_FILES = ("molecule_map", "cell_map", "cell_molecules", "cell_positions", "cell_lifetimes", "cell_divisions",
               "genomes", "genome_lens", "labels", "label_lens")


def shard_dir(statedir: Path, rank: int, world_size: int) -> Path:
    return Path(statedir) / SHARD_DIR / f"rank{rank:04d}_of{world_size:04d}"


def save_shard(world, statedir: Path) -> Path:
    """Write this rank's shard of a DistributedWorld (not collective; the caller synchronises)."""
    import json

    d = shard_dir(statedir, world.rank, world.world_size)
    d.mkdir(parents=True, exist_ok=True)
    world._reconcile()
    g, gl = world._genomes.packed()
    lab, ll = world._labels.packed()
    tensors = {
        "molecule_map": world.owned_molecule_map(),  # (the storage dtype: fp16 / bf16 maps stay small)
        "cell_map": world.owned_cell_map(),
        "cell_molecules": world.cell_molecules,
        "cell_positions": world.global_positions(),
        "cell_lifetimes": world.cell_lifetimes,
        "cell_divisions": world.cell_divisions,
        "genomes": torch.from_numpy(np.array(g, dtype=np.uint8)),
        "genome_lens": torch.from_numpy(gl),
        "labels": torch.from_numpy(np.array(lab, dtype=np.uint8)),
        "label_lens": torch.from_numpy(ll),
    }
    for name, t in tensors.items():
        torch.save(t.detach().cpu().contiguous().clone(), d / f"{name}.pt")
    torch.save(rng_state(world.device), d / RNG_FILE)
    meta = {"format": 1, "rank": world.rank, "world_size": world.world_size, "map_size": world.map_size,
            "H": world.H, "row0": world.row0, "n_cells": world.n_cells, "n_molecules": world.n_molecules,
            "map_dtype": str(world.__dict__.get("map_dtype", torch.float32)).replace("torch.", ""), "xcall": int(world.__dict__.get("_xcall", 0)),
            "xseed": int(world.__dict__.get("_xseed", 0)),
            # (the arenas' length bounds: the strip-boundary recombination sizes its exchange by them)
            "genome_width": int(world._genomes.width), "label_width": int(world._labels.width)}
    (d / "meta.json").write_text(json.dumps(meta))
    return d


def shard_metas(statedir: Path) -> list[dict]:
    """The metas of the shards under ``statedir`` (sorted by rank; empty without shards). Raises if
    the shards of more than one rank count are mixed or a rank is missing."""
    import json

    root = Path(statedir) / SHARD_DIR
    if not root.is_dir():
        return []
    metas = sorted((json.loads((p / "meta.json").read_text()) for p in root.iterdir() if (p / "meta.json").exists()),
                   key=lambda m: m["rank"])
    if not metas:
        return []
    n = metas[0]["world_size"]
    if [m["rank"] for m in metas] != list(range(n)) or any(m["world_size"] != n for m in metas):
        raise ValueError(f"{root}: incomplete or mixed shards ({[(m['rank'], m['world_size']) for m in metas]})")
    return metas


def _ld(path: Path, device="cpu", mmap: bool = False) -> torch.Tensor:
    return torch.load(path, map_location=device, weights_only=True, mmap=mmap)


def assemble_state(statedir: Path) -> None:
    """Write the reference layout (``cell_*.pt``, ``molecule_map.pt``, ``cells.fasta``,
    ``rng_state.pt`` of rank 0) into ``statedir`` from its shards: maps stacked by rows, cells
    numbered rank by rank (the global index space of ``DistributedWorld``). The result is byte-equal
    to what a gathered single-process save of the same world writes."""
    statedir = Path(statedir)
    metas = shard_metas(statedir)
    if not metas:
        raise FileNotFoundError(f"{statedir}: no shards")
    dirs = [shard_dir(statedir, m["rank"], m["world_size"]) for m in metas]
    mm = torch.cat([_ld(d / "molecule_map.pt", mmap=True).to(torch.float32) for d in dirs], dim=1)
    torch.save(mm, statedir / "molecule_map.pt")
    del mm
    for name, dt in (("cell_map", torch.bool), ("cell_molecules", torch.float32), ("cell_positions", torch.int32),
                     ("cell_lifetimes", torch.int32), ("cell_divisions", torch.int32)):
        t = torch.cat([_ld(d / f"{name}.pt", mmap=True) for d in dirs], dim=0).to(dt)
        torch.save(t, statedir / f"{name}.pt")
    idx0 = 0
    for r, d in enumerate(dirs):
        gl = _ld(d / "genome_lens.pt").numpy()
        _host().fasta_write(str(statedir / "cells.fasta"), idx0, _ld(d / "genomes.pt").numpy(), gl,
                            _ld(d / "labels.pt").numpy(), _ld(d / "label_lens.pt").numpy(), r > 0, idx0 > 0)
        idx0 += int(gl.size)
    import shutil

    shutil.copyfile(dirs[0] / RNG_FILE, statedir / RNG_FILE)


def load_strip(world, statedir: Path, ignore_cell_params: bool = False, restore_rng: bool = False) -> str:
    """Load this rank's part of a state into a DistributedWorld (collective only through the halo
    refresh at the end): its own shard when the state holds shards of the same rank count and map
    (then ``restore_rng`` restores the rank's random streams and the boundary-recombination counter,
    and a run continues as an uninterrupted one), otherwise its strip of the reference files.
    Returns ``"shard"`` or ``"reference"``."""
    statedir = Path(statedir)
    metas = shard_metas(statedir)
    lo, H, row0 = world._lo, world.H, world.row0
    if metas and metas[0]["world_size"] == world.world_size and metas[0]["map_size"] == world.map_size:
        d = shard_dir(statedir, world.rank, world.world_size)
        meta = metas[world.rank]
        if meta["row0"] != row0 or meta["H"] != H:
            raise ValueError(f"{d}: strip rows {meta['row0']}+{meta['H']} differ from this rank's {row0}+{H}")
        mm = _ld(d / "molecule_map.pt")
        gpos = _ld(d / "cell_positions.pt").long()
        cols = {k: _ld(d / f"{k}.pt") for k in ("cell_molecules", "cell_lifetimes", "cell_divisions")}
        g, gl = _ld(d / "genomes.pt").numpy(), _ld(d / "genome_lens.pt").numpy()
        lab, ll = _ld(d / "labels.pt").numpy(), _ld(d / "label_lens.pt").numpy()
        mine = None
        kind = "shard"
    else:
        # the reference files: map rows memory-mapped (only this strip's pages are read), the cell
        # table filtered by global row
        mm = _ld(statedir / "molecule_map.pt", mmap=True)[:, row0 : row0 + H]
        gpos_all = _ld(statedir / "cell_positions.pt").long()
        sel = torch.nonzero((gpos_all[:, 0] >= row0) & (gpos_all[:, 0] < row0 + H)).flatten()
        gpos = gpos_all[sel]
        cols = {k: _ld(statedir / f"{k}.pt", mmap=True)[sel] for k in ("cell_molecules", "cell_lifetimes",
                                                                       "cell_divisions")}
        g, gl, lab, ll = read_fasta_packed(statedir / "cells.fasta")
        if int(gl.size) != int(gpos_all.size(0)):
            raise ValueError(f"{statedir}: {gl.size} FASTA entries for {gpos_all.size(0)} positions")
        mine = sel.numpy()
        kind = "reference"
        meta = None
    k = int(gpos.size(0))
    genomes = packed_rows(g, gl, mine) if k else None
    labels = packed_rows(lab, ll, mine) if k else None
    lpos = gpos.clone()
    lpos[:, 0] += lo - row0
    world._adopt_strip(mm, genomes, labels, lpos.to(torch.int32), cols, params=not ignore_cell_params)
    if kind == "shard" and restore_rng:
        set_rng_state(_ld(shard_dir(statedir, world.rank, world.world_size) / RNG_FILE), world.device)
        # (the strip-boundary recombination streams: a seed shared by all ranks and a call counter)
        world.__dict__["_xcall"] = int(meta.get("xcall", 0))
        if "xseed" in meta:
            world.__dict__["_xseed"] = int(meta["xseed"])
    if meta is not None:
        for arena, key in ((world._genomes, "genome_width"), (world._labels, "label_width")):
            if key in meta and int(meta[key]) > arena.width:
                arena.reserve(arena.n, int(meta[key]))
    return kind


# ---------------------------------------------------------------------------- world pickles
class _RefModule:
    """Stand-in for a ``torch.nn.Module`` in a reference pickle (the reference keeps one
    ``Conv2d`` per molecule as its diffusion kernel, ``world.py:948-984``): only its state is kept,
    nothing of the module is constructed or run."""

    def __setstate__(self, state):
        self.__dict__["state"] = state

    def weight(self) -> torch.Tensor | None:
        params = self.__dict__.get("state", {}).get("_parameters") or {}
        return params.get("weight")


_TORCH_FUNCS = {
    ("torch._utils", "_rebuild_tensor"),
    ("torch._utils", "_rebuild_tensor_v2"),
    ("torch._utils", "_rebuild_parameter"),
    ("torch._utils", "_rebuild_parameter_with_state"),
    ("torch._utils", "_rebuild_device_tensor_from_numpy"),
}
_BUILTINS = {
    ("collections", "OrderedDict"): collections.OrderedDict,
    ("builtins", "set"): set,
    ("builtins", "frozenset"): frozenset,
    ("builtins", "slice"): slice,
    ("builtins", "complex"): complex,
    ("torch", "Size"): torch.Size,
    ("torch", "device"): torch.device,
}
# the data classes a world pickle holds (module-relative names; ``magicsoup.*`` reference paths are
# aliased onto these by the ``magicsoup`` package). Only these may be named by a file, and of them
# only the plain containers may be *called* (REDUCE): the others are rebuilt with ``cls.__new__`` and
# their state, never their constructor (a World / Kinetics constructor allocates device memory)
_DATA_CLASSES = {
    "models.containers": ("Molecule", "Chemistry", "CatalyticDomain", "TransporterDomain",
                          "RegulatoryDomain", "Protein"),
    "models.genetics": ("Genetics",),
    "models.kinetics": ("Kinetics", "_HillMapFact", "_LogNormWeightMapFact", "_SignMapFact",
                        "_VectorMapFact", "_ReactionMapFact", "_TransporterMapFact", "_RegulatoryMapFact"),
    "models.world": ("World",),
}
# reference module paths (python/magicsoup/*.py) -> ours
_REF_MODULES = {"containers": "models.containers", "genetics": "models.genetics",
                "kinetics": "models.kinetics", "world": "models.world"}


def _allowed_class(module: str, name: str):
    root, _, rest = module.partition(".")
    if root == "magicsoup":
        rest = _REF_MODULES.get(rest, rest)
    elif root != "magicsoup_amd":
        return None
    if name not in _DATA_CLASSES.get(rest, ()):
        return None
    import importlib

    return getattr(importlib.import_module(f"magicsoup_amd.{rest}"), name)


class _WorldUnpickler(pickle._Unpickler):  # the pure-Python unpickler: its opcode table is reachable
    """Restricted unpickler for world pickles (ours and the reference's): see the module docstring
    for what a file may name; anything else raises ``pickle.UnpicklingError``. Besides the name
    check (``find_class``), calling an object the file named -- REDUCE, INST, OBJ -- is refused for
    everything but torch's tensor rebuild functions, the storage loader and the builtin containers;
    NEWOBJ / NEWOBJ_EX (``cls.__new__`` only) are limited to those and this package's data
    classes."""

    dispatch = dict(pickle._Unpickler.dispatch)

    def __init__(self, fh, map_location):
        super().__init__(fh)
        self._loc = map_location
        self._callable: set[int] = set()

    def _ok_call(self, obj):
        self._callable.add(id(obj))
        return obj

    def find_class(self, module, name):
        if module == "torch.storage" and name == "_load_from_bytes":
            loc = self._loc
            return self._ok_call(lambda b: torch.load(io.BytesIO(b), map_location=loc, weights_only=True))
        if (module, name) in _TORCH_FUNCS:
            return self._ok_call(super().find_class(module, name))
        if (module, name) in _BUILTINS:
            return self._ok_call(_BUILTINS[(module, name)])
        if module == "torch" and isinstance(getattr(torch, name, None), torch.dtype):
            return getattr(torch, name)
        if module == "torch" and name.endswith("Storage") and name[:1].isupper():
            return super().find_class(module, name)
        if module.startswith("torch.nn.modules."):
            return _RefModule
        cls = _allowed_class(module, name)
        if cls is not None:
            if module.startswith("magicsoup.") or module == "magicsoup":
                import magicsoup  # noqa: F401 - installs the reference-path aliases
            if name in ("Molecule", "Chemistry"):
                return self._ok_call(cls)  # plain containers (Molecule: __getnewargs__ by name)
            return cls
        raise pickle.UnpicklingError(f"world pickles may not reference {module}.{name}")

    def _load_reduce(self):
        stack = self.stack
        args = stack.pop()
        func = stack[-1]
        if id(func) not in self._callable:
            raise pickle.UnpicklingError(f"world pickles may not call {func!r}")
        stack[-1] = func(*args)

    dispatch[pickle.REDUCE[0]] = _load_reduce

    def _instantiate(self, klass, args):
        # INST ('i') and OBJ ('o') call the class itself: the same rule as REDUCE
        if id(klass) not in self._callable:
            raise pickle.UnpicklingError(f"world pickles may not instantiate {klass!r}")
        super()._instantiate(klass, args)

    def _newobj_ok(self, cls) -> bool:
        # NEWOBJ / NEWOBJ_EX run only ``cls.__new__`` (no constructor): allowed for the callable
        # containers and this package's data classes, never for a torch storage class (whose
        # ``__new__`` allocates whatever size the file names)
        if not isinstance(cls, type) or (cls.__module__ or "").startswith("torch"):
            return False
        return id(cls) in self._callable or (cls.__module__ or "").startswith("magicsoup_amd.")

    def _load_newobj(self):
        args = self.stack.pop()
        cls = self.stack[-1]
        if not self._newobj_ok(cls):
            raise pickle.UnpicklingError(f"world pickles may not create {cls!r}")
        self.stack[-1] = cls.__new__(cls, *args)

    def _load_newobj_ex(self):
        kwargs = self.stack.pop()
        args = self.stack.pop()
        cls = self.stack[-1]
        if not self._newobj_ok(cls):
            raise pickle.UnpicklingError(f"world pickles may not create {cls!r}")
        self.stack[-1] = cls.__new__(cls, *args, **kwargs)

    dispatch[pickle.NEWOBJ[0]] = _load_newobj
    dispatch[pickle.NEWOBJ_EX[0]] = _load_newobj_ex


def load_world_pickle(path: Path, device: str | None = None):
    loc = device if device is not None else ("cuda" if torch.cuda.is_available() else "cpu")
    with open(path, "rb") as fh:
        world = _WorldUnpickler(fh, loc).load()
    if device is not None and str(world.device) != str(device):
        world.to(device)
    return world


def reference_world_state(st: dict) -> dict:
    """A reference ``World.__dict__`` (``world.py:161-204``: list genomes / labels, dense per-cell
    tensors, one ``Conv2d`` per molecule) in this package's pickled layout (World.__getstate__)."""
    from magicsoup_amd.models.world import _diffusion_weights

    st = dict(st)
    out = {k: st[k] for k in ("device", "batch_size", "map_size", "abs_temp", "chemistry", "genetics", "kinetics")}
    m = int(st.get("n_molecules", len(st["chemistry"].molecules)))
    out["n_molecules"] = m
    out["_int_mol_idxs"] = list(range(m))
    out["_ext_mol_idxs"] = list(range(m, 2 * m))
    out["_mol_degrads"] = [float(x) for x in st["_mol_degrads"]]
    out["_permeation"] = [float(x) for x in st["_permeation"]]
    diff = []
    for conv, mol in zip(st.get("_diffusion", []), st["chemistry"].molecules):
        w = conv.weight() if isinstance(conv, _RefModule) else None
        if w is not None and w.numel() == 9:
            w = w.detach().reshape(3, 3).float().cpu()
            diff.append((float(w[0, 0]), float(w[1, 1])))  # kernel [[a,a,a],[a,b,a],[a,a,a]]
        else:
            diff.append(_diffusion_weights(mol.diffusivity))
    out["_diffusion"] = diff
    n = int(st["n_cells"])
    out["n_cells"] = n
    out["map_dtype"] = torch.float32
    out["_cols"] = {
        "cell_molecules": st["cell_molecules"].detach().float().cpu(),
        "cell_positions": st["cell_positions"].detach().int().cpu(),
        "cell_lifetimes": st["cell_lifetimes"].detach().int().cpu(),
        "cell_divisions": st["cell_divisions"].detach().int().cpu(),
    }
    out["_genomes"] = list(st["cell_genomes"])
    out["_labels"] = list(st["cell_labels"])
    out["_molmap"] = st["molecule_map"].detach().float().cpu()
    out["_cell_map"] = st["cell_map"].detach().bool().cpu()
    out["_pending_scale"] = None
    out["_pending_corr"] = None
    return out


def reference_kinetics_state(st: dict) -> dict:
    """A reference ``Kinetics.__dict__`` (``kinetics.py:390-460``: dense parameter tensors as
    attributes) in this package's layout (dense row storage, one row per cell)."""
    from magicsoup_amd.models.kinetics import _PARAMS

    st = dict(st)
    store = {}
    for name in _PARAMS:
        t = st.pop(name)
        store[name] = t.detach().contiguous()
    n = int(store["N"].size(0))
    st["_store_d"] = store
    st["_slot"] = None
    st["_ncells"] = n
    st["_nrows"] = n
    st.setdefault("n_signals", int(st["mol_energies"].numel()))
    st["last_masks"] = []
    return st
