"""Loader for the native modules.

``host()`` returns the OpenMP host core, ``hip()`` the gfx950 device core. Both are built in-tree on
first use if missing (see :mod:`magicsoup_amd.ops.build`). A missing or broken device module on a
machine with a GPU is a hard error: there is no silent fallback from a CUDA/HIP tensor to a CPU or
eager-PyTorch implementation.
"""
from __future__ import annotations

import atexit
import importlib
import importlib.util
import os
import sys
import threading

_lock = threading.Lock()
_mods: dict[str, object] = {}


def _load(name: str, builder) -> object:
    with _lock:
        if name in _mods:
            return _mods[name]
        override = os.environ.get("MS_HOST_SO") if name == "_host" else None
        if override:
            # an instrumented build of the host core (scripts/sanitize_host.sh: ASan + UBSan)
            spec = importlib.util.spec_from_file_location(f"magicsoup_amd.{name}", override)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules[f"magicsoup_amd.{name}"] = mod
            _mods[name] = mod
            return mod
        try:
            mod = importlib.import_module(f"magicsoup_amd.{name}")
        except ImportError:
            if os.environ.get("MS_NO_AUTOBUILD"):
                raise
            builder()
            mod = importlib.import_module(f"magicsoup_amd.{name}")
        _mods[name] = mod
        return mod


def _release_static(mod) -> None:
    """Free the extension's process-wide HIP buffers before the C exit handlers run (a profiler's
    interception layer finalises there; the HIP runtime's own teardown of leftover allocations
    after that point ended profiled runs in SIGSEGV)."""
    try:
        mod.release_static()
    except Exception:  # noqa: BLE001 - exit path: a dead device must not turn into a traceback
        pass


def host():
    """The OpenMP host module ``magicsoup_amd._host`` (built on demand)."""
    from magicsoup_amd.ops import build

    return _load("_host", build.build_host)


def hip():
    """The gfx950 device module ``magicsoup_amd._hip`` (built on demand; raises if unavailable)."""
    from magicsoup_amd.ops import build

    fresh = "_hip" not in _mods
    try:
        mod = _load("_hip", build.build_hip)
    except Exception as err:  # pragma: no cover - exercised on GPU boxes only
        raise RuntimeError(
            "magicsoup_amd: the gfx950 HIP extension (_hip) could not be loaded; GPU execution"
            " requires it (no fallback). Build it with `python -m magicsoup_amd.ops.build`."
        ) from err
    if fresh and os.environ.get("MS_RELEASE_AT_EXIT", "1") == "1":
        atexit.register(_release_static, mod)
    if fresh and os.environ.get("MS_INTEGRATE_MODE"):
        # integrator launch-mode bits for whole-run A/B (kinetics.hip, set_integrate_mode)
        mod.set_integrate_mode(int(os.environ["MS_INTEGRATE_MODE"]))  # type: ignore[attr-defined]
    if fresh and os.environ.get("MS_SPL2_WAVES"):
        mod.set_spl2_waves(int(os.environ["MS_SPL2_WAVES"]))  # type: ignore[attr-defined]
    if fresh and os.environ.get("MS_RESCUE_MODE"):
        # 0: the separate launches behind the speculative integrator (A/B of the rescue launch)
        mod.set_rescue_mode(int(os.environ["MS_RESCUE_MODE"]))  # type: ignore[attr-defined]
    if fresh and os.environ.get("MS_PLACE_MODE"):
        # 1: per-round placement launches, 2: the single launch as a cooperative launch (world.hip)
        mod.set_place_mode(int(os.environ["MS_PLACE_MODE"]))  # type: ignore[attr-defined]
    if fresh and os.environ.get("MS_PLACE_TAIL"):
        # 0: the all-grid placement rounds (two grid barriers per round) for A/B
        mod.set_place_tail(int(os.environ["MS_PLACE_TAIL"]))  # type: ignore[attr-defined]
    if fresh and os.environ.get("MS_COOP_BLOCKS"):
        mod.set_coop_blocks(int(os.environ["MS_COOP_BLOCKS"]))  # type: ignore[attr-defined]
    if fresh and os.environ.get("MS_STENCIL_BLOCKS"):
        # blocks of the diffusion stencil launch (maps.hip; 0: one per tile)
        mod.set_stencil_blocks(int(os.environ["MS_STENCIL_BLOCKS"]))  # type: ignore[attr-defined]
    if fresh and os.environ.get("MS_EVENT_SPIN"):
        # 0: host event waits block at once (events.hip ev_sync)
        mod.set_event_spin(int(os.environ["MS_EVENT_SPIN"]))  # type: ignore[attr-defined]
    if fresh and os.environ.get("MS_REC_THIN"):
        # 0: the per-slot recombination draws + selection pass (world.hip rec_slots) for A/B
        mod.set_rec_thinning(int(os.environ["MS_REC_THIN"]))  # type: ignore[attr-defined]
    if fresh and os.environ.get("MS_SELECT_SINGLE"):
        # 0: the two-launch count + write selection (select.hip) for A/B
        mod.set_select_single_pass(int(os.environ["MS_SELECT_SINGLE"]), int(os.environ.get("MS_SELECT_ITEMS", "0")))  # type: ignore[attr-defined]
    if fresh and os.environ.get("MS_STENCIL_PF"):
        # rows in flight ahead of the stencil's current row (-1: auto, 0-3)
        mod.set_stencil_prefetch(int(os.environ["MS_STENCIL_PF"]))  # type: ignore[attr-defined]
    if fresh and os.environ.get("MS_STENCIL_BAND"):
        # rows per wave band of the vector stencils (0: auto)
        mod.set_stencil_band(int(os.environ["MS_STENCIL_BAND"]))  # type: ignore[attr-defined]
    return mod


def set_seed(seed: int) -> None:
    """Seed every native RNG stream (host and device) for reproducible runs."""
    host().set_seed(int(seed) & 0xFFFFFFFFFFFFFFFF)
    if "_hip" in _mods:
        _mods["_hip"].set_seed(int(seed) & 0xFFFFFFFFFFFFFFFF)  # type: ignore[attr-defined]
