"""Generate ``docs/reference.md`` (the API reference) from the package's docstrings.

The reference builds its API page with mkdocs + mkdocstrings (``mkdocs.yml:22-44``: public members
in source order, ``__init__`` merged into the class, members without a docstring hidden). Neither is
installed in this image, so this script does the same walk with :mod:`inspect` and writes plain
Markdown that any renderer (or ``mkdocs build`` with the ``mkdocs.yml`` at the repo root) shows.
``python docs/gen_api.py --check`` fails if the committed page is stale (``tests/test_docs.py``).

    python docs/gen_api.py            # rewrite docs/reference.md
    python docs/gen_api.py --check    # exit 1 if docs/reference.md differs
"""
from __future__ import annotations

import importlib
import inspect
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

OUT = os.path.join(ROOT, "docs", "reference.md")

# (section title, module, intro) -- the reference's page order (world, containers, factories,
# genetics, kinetics, mutations, util), then this package's additions
SECTIONS = [
    ("magicsoup_amd.models.world", "The simulation: cells on a toroidal map, molecules on per-species maps."),
    ("magicsoup_amd.models.containers", "Molecules, chemistries and the human-readable cell / protein / domain views."),
    ("magicsoup_amd.models.factories", "Genome factories: generate genomes that encode a given proteome."),
    ("magicsoup_amd.models.genetics", "Genome -> proteome translation tables."),
    ("magicsoup_amd.models.kinetics", "Proteome -> kinetic parameters, and the integrator behind enzymatic_activity."),
    ("magicsoup_amd.models.mutations", "Point mutations and recombinations of genome strings."),
    ("magicsoup_amd.utils.util", "Small helpers (random genomes, codons, distances)."),
    ("magicsoup_amd.parallel.dist_world", "One world domain-decomposed over the ranks of a node (RCCL over xGMI)."),
    ("magicsoup_amd.parallel.global_world", "The reference's global cell-index API over a decomposed world."),
    ("magicsoup_amd.parallel.ensemble", "Independent replicate worlds, one per GPU."),
    ("magicsoup_amd.utils.memory", "HBM sizing: bytes per pixel / cell and the largest config that fits a GPU."),
    ("magicsoup_amd.utils.checkpoint", "save_state / load_state file format and world pickles."),
    ("magicsoup_amd.utils.profiling", "Per-op timings and roctx ranges."),
]


def _line(obj) -> int:
    try:
        return inspect.getsourcelines(obj)[1]
    except (OSError, TypeError):
        return 1 << 30


def _doc(obj) -> str:
    d = inspect.getdoc(obj) or ""
    return d.strip()


def _sig(name: str, obj) -> str:
    try:
        sig = str(inspect.signature(obj))
    except (TypeError, ValueError):
        sig = "(...)"
    return f"{name}{sig}"


def _own(mod, obj) -> bool:
    return getattr(obj, "__module__", None) == mod.__name__


def _members(cls):
    out = []
    for name, raw in cls.__dict__.items():
        if name.startswith("_"):
            continue
        obj = raw
        kind = "method"
        if isinstance(raw, property):
            kind, obj = "property", raw.fget
        elif isinstance(raw, (classmethod, staticmethod)):
            kind, obj = ("classmethod" if isinstance(raw, classmethod) else "staticmethod"), raw.__func__
        elif not callable(raw):
            continue
        if not _doc(obj):
            continue  # (mkdocstrings: show_if_no_docstring false)
        out.append((_line(obj), name, kind, obj))
    return [m[1:] for m in sorted(out, key=lambda m: m[0])]


def _class_md(name: str, cls) -> list[str]:
    lines = [f"### `{name}`", ""]
    init = cls.__dict__.get("__init__")
    sig = _sig(name, init) if init is not None else _sig(name, cls)
    sig = sig.replace("(self, ", "(").replace("(self)", "()")
    lines += ["```python", f"class {sig}", "```", ""]
    doc = _doc(cls)
    if doc:
        lines += [doc, ""]
    for mname, kind, obj in _members(cls):
        if kind == "property":
            head = f"`{name}.{mname}` *(property)*"
        else:
            msig = _sig(mname, obj).replace("(self, ", "(").replace("(self)", "()").replace("(cls, ", "(")
            head = f"`{name}.{msig}`" + (f" *({kind})*" if kind != "method" else "")
        lines += [f"#### {head}", "", _doc(obj), ""]
    return lines


def _module_md(modname: str, intro: str) -> list[str]:
    mod = importlib.import_module(modname)
    lines = [f"## {modname}", "", intro, ""]
    items = []
    for name, obj in vars(mod).items():
        if name.startswith("_") or not _own(mod, obj):
            continue
        if inspect.isclass(obj) or inspect.isfunction(obj):
            if not _doc(obj):
                continue
            items.append((_line(obj), name, obj))
    for _, name, obj in sorted(items, key=lambda t: t[0]):
        if inspect.isclass(obj):
            lines += _class_md(name, obj)
        else:
            lines += [f"### `{_sig(name, obj)}`", "", _doc(obj), ""]
    return lines


def render() -> str:
    lines = [
        "# API reference",
        "",
        "Generated from the docstrings by `python docs/gen_api.py` (the reference renders the same",
        "page with mkdocstrings, `mkdocs.yml`). `import magicsoup_amd as ms` (or `import magicsoup as",
        "ms`, the reference's name) exposes the names of the first seven sections as `ms.*`.",
        "",
    ]
    for modname, intro in SECTIONS:
        lines += _module_md(modname, intro)
    return "\n".join(lines).rstrip() + "\n"


def main(argv: list[str]) -> int:
    text = render()
    if "--check" in argv:
        cur = open(OUT, encoding="utf-8").read() if os.path.exists(OUT) else ""
        if cur != text:
            print("docs/reference.md is stale: run python docs/gen_api.py", file=sys.stderr)
            return 1
        return 0
    with open(OUT, "w", encoding="utf-8") as fh:
        fh.write(text)
    print(f"wrote {OUT} ({text.count(chr(10))} lines)")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
