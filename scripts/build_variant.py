"""Build a variant of the _hip module for in-process A/B (scripts/ab_so.py): the in-tree objects of
every HIP source except one, plus that source replaced by a variant file, linked into OUT.

usage: python scripts/build_variant.py <variant.hip> <replaced source name, e.g. kinetics.hip> <OUT.so>
VARIANT_CFLAGS: extra compiler flags for the variant source only."""
import os
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from magicsoup_amd.ops import build  # noqa: E402


def main():
    variant, name, out = Path(sys.argv[1]), sys.argv[2], Path(sys.argv[3])
    build.build_hip()
    hipdir = build.CSRC / "hip"
    objdir = build.BUILD / "_hip"
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cflags = [f"--offload-arch={build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
              "-munsafe-fp-atomics", "-ffp-contract=off", f"-I{build.CSRC / 'include'}", f"-I{hipdir}",
              *build._py_includes()]
    with tempfile.TemporaryDirectory() as td:
        src = Path(td) / name
        shutil.copy(variant, src)
        obj = Path(td) / "variant.o"
        extra = os.environ.get("VARIANT_CFLAGS", "").split()  # e.g. -ffp-contract=fast (later flags win)
        subprocess.run([hipcc, *cflags, *extra, "-c", str(src), "-o", str(obj)], check=True)
        objs = [str(objdir / (p.stem + ".o")) for p in sorted(hipdir.glob("*.hip")) if p.name != name]
        out.parent.mkdir(parents=True, exist_ok=True)
        subprocess.run([hipcc, "-shared", f"--offload-arch={build.ARCH}", *objs, str(obj), "-o", str(out)], check=True)
    print(out)


if __name__ == "__main__":
    main()
