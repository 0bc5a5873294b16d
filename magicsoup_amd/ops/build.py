"""In-tree build of the native modules.

* ``magicsoup_amd/_host*.so`` — OpenMP host core (g++ -O3 -fopenmp): translation, mutations,
  geometry, CPU integrator, CPU diffusion.
* ``magicsoup_amd/_hip*.so`` — gfx950 device core (hipcc --offload-arch=gfx950): every HIP kernel
  and its launcher.

Both are plain pybind11 modules with a C ABI towards PyTorch (tensors cross as data pointers plus the
current HIP stream), so they do not depend on the torch C++ ABI and compile in seconds. Sources are
compiled to objects in parallel and relinked only when a source or header is newer than the module.

Usage: ``python -m magicsoup_amd.ops.build [--host-only|--hip-only] [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parents[1]
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "native"
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("MS_OFFLOAD_ARCH", "gfx950")


def _py_includes() -> list[str]:
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _newest(paths: list[Path]) -> float:
    return max((p.stat().st_mtime for p in paths), default=0.0)


def _run(cmd: list[str]) -> None:
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + res.stdout + res.stderr)
        raise RuntimeError(f"native build failed: {cmd[0]} {cmd[-1]}")


def _build(name: str, sources: list[Path], compiler: str, cflags: list[str], ldflags: list[str], force: bool, jobs: int) -> Path:
    out = PKG / f"{name}{EXT}"
    headers = list((CSRC / "include").glob("*.h")) + [p for s in sources for p in s.parent.glob("*.h")]
    if not force and out.exists() and out.stat().st_mtime >= _newest(sources + headers):
        return out
    objdir = BUILD / name
    objdir.mkdir(parents=True, exist_ok=True)
    objs = []
    cmds = []
    hdr_time = _newest(headers)
    for src in sources:
        obj = objdir / (src.stem + ".o")
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr_time):
            cmds.append([compiler, *cflags, "-c", str(src), "-o", str(obj)])
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, cmds))
    tmp = out.with_suffix(".tmp.so")
    _run([compiler, *ldflags, *map(str, objs), "-o", str(tmp)])
    os.replace(tmp, out)
    return out


def build_host(force: bool = False, jobs: int = 8) -> Path:
    srcs = sorted((CSRC / "host").glob("*.cpp"))
    cflags = ["-O3", "-std=c++17", "-fPIC", "-fopenmp", "-fvisibility=hidden", f"-I{CSRC / 'include'}", *_py_includes()]
    return _build("_host", srcs, "g++", cflags, ["-shared", "-fopenmp"], force, jobs)


def build_hip(force: bool = False, jobs: int = 8) -> Path:
    srcs = sorted((CSRC / "hip").glob("*.hip"))
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cflags = [
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-fvisibility=hidden",
        "-munsafe-fp-atomics",
        # no FMA contraction: device results match the OpenMP host core operation for operation
        "-ffp-contract=off",
        f"-I{CSRC / 'include'}",
        *_py_includes(),
    ]
    return _build("_hip", srcs, hipcc, cflags, ["-shared", f"--offload-arch={ARCH}"], force, jobs)


def build_all(force: bool = False, jobs: int = 8, host: bool = True, hip: bool = True) -> list[Path]:
    out = []
    if host:
        out.append(build_host(force, jobs))
    if hip:
        out.append(build_hip(force, jobs))
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--host-only", action="store_true")
    ap.add_argument("--hip-only", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    for p in build_all(a.force, a.j, host=not a.hip_only, hip=not a.host_only):
        print(p)


if __name__ == "__main__":
    main()
