"""Dispatch of the kinetics hot paths to the native cores.

CPU tensors go to the OpenMP host module, HIP tensors to the gfx950 kernels (no fallback between
the two). Tensors cross into C++ as contiguous buffers; HIP launches run on the current stream.
"""
from __future__ import annotations

import torch

from magicsoup_amd.constants import GAS_CONSTANT
from magicsoup_amd.ops import native

_I32 = ("N", "Nf", "Nb", "A")
_F32 = ("Kmr", "Kmf", "Kmb", "Vmax", "Ke")


def _canonical_params(kin) -> dict[str, torch.Tensor]:
    """Parameter storage in kernel layout (contiguous int32 / float32). Rows are storage rows: on
    a GPU, cell i's parameters are at row ``kin._slot_tensor()[i]`` when that is not None."""
    return kin._kernel_params()


def _np(t: torch.Tensor):
    return t.detach().numpy()


def integrate(kin, X: torch.Tensor, trims, n_iters: int, reduce_mask=None, decisions=None) -> list[int]:
    """Fused integrate_signals on X (c, s) in place; returns the per-part iteration masks.
    ``reduce_mask`` (host path) maps a part's local iteration mask to the global one.
    ``decisions`` (host path, diagnostics): a uint8 numpy array (c, parts, 4, P) receiving every
    protein's damping decision per iteration (bit 0 low, bit 1 high)."""
    c = X.size(0)
    if c == 0:
        return []
    if X.is_cuda:
        from magicsoup_amd.ops import hip_ops

        p = kin._packed_params()
        if kin.__dict__["_ncells"] < c:
            raise ValueError(f"kinetics has {kin.__dict__['_ncells']} cells but X has {c}")
        return hip_ops.integrate(kin, X, p, list(trims), n_iters, slot=kin._slot_tensor())
    kin._materialize()
    p = _canonical_params(kin)
    if p["N"].size(0) < c:
        raise ValueError(f"kinetics has {p['N'].size(0)} cell rows but X has {c}")
    masks = native.host().integrate_signals(
        _np(X),
        *(_np(p[k]) for k in ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax", "Ke")),
        None,
        [float(t) for t in trims],
        int(n_iters),
        reduce_mask,
        decisions,
    )
    return list(masks)


def _lut_sources(kin):
    return (kin.vmax_map.weights, kin.km_map.weights, kin.sign_map.signs, kin.hill_map.numbers, kin.reaction_map.M,
            kin.transport_map.M, kin.effector_map.M, kin.mol_energies)


def build_luts(kin, device) -> dict[str, torch.Tensor]:
    """Token -> value LUTs in kernel layout, cached until a map tensor is replaced or modified in
    place (identity + version counter): the device genome pipeline builds parameters twice a step."""
    src = _lut_sources(kin)
    key = (str(device),) + tuple((id(t), t._version) for t in src)
    c = kin.__dict__.get("_lut_cache")
    if c is not None and c[0] == key:
        return c[1]
    luts = _luts(kin, device)
    # vector maps may be narrower than the token alphabet if a user swapped them (tests do)
    n_vec = min(luts["react"].size(0), luts["trnsp"].size(0), luts["eff"].size(0))
    for k in ("react", "trnsp", "eff"):
        luts[k] = luts[k][:n_vec].contiguous()
    kin.__dict__["_lut_cache"] = (key, luts, src)  # src keeps the ids alive
    return luts


def _luts(kin, device) -> dict[str, torch.Tensor]:
    return {
        "vmax": kin.vmax_map.weights.to(device=device, dtype=torch.float32).contiguous(),
        "km": kin.km_map.weights.to(device=device, dtype=torch.float32).contiguous(),
        "signs": kin.sign_map.signs.to(device=device, dtype=torch.int32).contiguous(),
        "hills": kin.hill_map.numbers.to(device=device, dtype=torch.int32).contiguous(),
        "react": kin.reaction_map.M.to(device=device, dtype=torch.int32).contiguous(),
        "trnsp": kin.transport_map.M.to(device=device, dtype=torch.int32).contiguous(),
        "eff": kin.effector_map.M.to(device=device, dtype=torch.int32).contiguous(),
        "energies": kin.mol_energies.to(device=device, dtype=torch.float32).contiguous(),
    }


def build_params(kin, rows: torch.Tensor | None, tokens: torch.Tensor, nprot: torch.Tensor | None = None,
                 roff: torch.Tensor | None = None) -> None:
    """Write parameter rows ``rows`` from dense tokens (n, P, D, 5). With ``nprot`` (GPU), rows
    whose proteome is empty are unset (all zero) in the same launch. ``roff`` (GPU record storage,
    Kinetics._alloc_cells): the first record of each item instead of rows; only its ``nprot``
    proteins are written."""
    p = _canonical_params(kin)
    dev = p["Kmr"].device
    if dev.type != "cuda":
        kin._materialize()  # (host builds write the full parameter set)
        p = _canonical_params(kin)
    n = int(tokens.size(0)) if roff is not None else int(rows.numel())
    if n == 0:
        return
    tokens = tokens.to(device=dev, dtype=torch.int32).contiguous()
    luts = build_luts(kin, dev)
    if dev.type == "cuda":
        from magicsoup_amd.ops import hip_ops

        np_ = None if nprot is None else nprot.to(device=dev, dtype=torch.int32).contiguous()
        rows = None if rows is None else rows.to(device=dev, dtype=torch.int32).contiguous()
        hip_ops.build_params(kin, tokens, rows, luts, p, float(kin.abs_temp), GAS_CONSTANT, nprot=np_, roff=roff)
        return
    rows = rows.to(device=dev, dtype=torch.int32).contiguous()
    if nprot is not None:
        nprot = nprot.cpu()
        empty = nprot == 0
        if bool(empty.any()):
            kin.unset_cell_params(rows.cpu()[empty].long())
        full = ~empty
        if not bool(full.any()):
            return
        rows, tokens = rows[full], tokens[full]
    native.host().build_params(
        _np(tokens),
        _np(rows),
        _np(luts["vmax"]),
        _np(luts["km"]),
        _np(luts["signs"]),
        _np(luts["hills"]),
        _np(luts["react"]),
        _np(luts["trnsp"]),
        _np(luts["eff"]),
        _np(luts["energies"]),
        float(kin.abs_temp),
        float(GAS_CONSTANT),
        *(_np(p[k]) for k in ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax", "Ke")),
    )
