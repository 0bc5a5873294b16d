"""Reference-compatible import path: ``import magicsoup as ms`` resolves to :mod:`magicsoup_amd`.

Submodules of the reference layout (``magicsoup.world``, ``magicsoup.kinetics``,
``magicsoup.containers``, ``magicsoup.genetics``, ``magicsoup.factories``, ``magicsoup.mutations``,
``magicsoup.util``, ``magicsoup.constants``, ``magicsoup.examples.*``) are aliased to their
``magicsoup_amd`` implementations, so code written for the reference runs unchanged.
"""
import importlib
import sys

from magicsoup_amd import *  # noqa: F401,F403
from magicsoup_amd import set_seed, __version__  # noqa: F401

_ALIASES = {
    "_lib": "magicsoup_amd._lib",
    "constants": "magicsoup_amd.constants",
    "util": "magicsoup_amd.utils.util",
    "containers": "magicsoup_amd.models.containers",
    "genetics": "magicsoup_amd.models.genetics",
    "kinetics": "magicsoup_amd.models.kinetics",
    "world": "magicsoup_amd.models.world",
    "mutations": "magicsoup_amd.models.mutations",
    "factories": "magicsoup_amd.models.factories",
    "examples": "magicsoup_amd.examples",
    "examples.wood_ljungdahl": "magicsoup_amd.examples.wood_ljungdahl",
    "examples.co2_fixing": "magicsoup_amd.examples.co2_fixing",
    "examples.reverse_krebs": "magicsoup_amd.examples.reverse_krebs",
    "examples.n2_fixing": "magicsoup_amd.examples.n2_fixing",
}


def _install() -> None:
    import importlib.abc
    import importlib.util

    class _Finder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
        def find_spec(self, fullname, path, target=None):
            if fullname.startswith("magicsoup.") and fullname[len("magicsoup.") :] in _ALIASES:
                return importlib.util.spec_from_loader(fullname, self)
            return None

        def create_module(self, spec):
            return importlib.import_module(_ALIASES[spec.name[len("magicsoup.") :]])

        def exec_module(self, module):
            pass

    sys.meta_path.insert(0, _Finder())


_install()
