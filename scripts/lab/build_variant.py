"""Build a variant of the _hip extension for an in-process A/B (scripts/lab/ab_so.py): the in-tree
objects of every source except those given, which are compiled from the given files.

    python scripts/lab/build_variant.py <out.so> <variant.hip> [...]   (each replaces its namesake)

MS_VARIANT_FLAGS: extra compiler flags for the variant sources (e.g. -DMS_INT_PROF)."""
import os
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from magicsoup_amd.ops import build  # noqa: E402


def main():
    out = Path(sys.argv[1])
    variants = {Path(p).stem.split(".")[0]: Path(p) for p in sys.argv[2:]}
    build.build_hip()
    objdir = build.BUILD / "_hip"
    out.parent.mkdir(parents=True, exist_ok=True)
    tmp = out.parent / "obj"
    tmp.mkdir(exist_ok=True)
    objs = []
    hipcc = "/opt/rocm/bin/hipcc"
    cflags = [f"--offload-arch={build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-munsafe-fp-atomics",
              "-ffp-contract=off", f"-I{build.CSRC / 'include'}", f"-I{build.CSRC / 'hip'}", *build._py_includes()]
    for src in sorted((build.CSRC / "hip").glob("*.hip")):
        if src.stem in variants:
            o = tmp / (src.stem + ".o")
            extra = os.environ.get("MS_VARIANT_FLAGS", "").split()
            subprocess.run([hipcc, *cflags, *extra, "-c", str(variants[src.stem]), "-o", str(o)], check=True)
            objs.append(o)
        else:
            objs.append(objdir / (src.stem + ".o"))
    subprocess.run([hipcc, "-shared", f"--offload-arch={build.ARCH}", *map(str, objs), "-o", str(out)], check=True)
    print(out)


if __name__ == "__main__":
    main()
