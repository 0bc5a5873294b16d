"""Where the device memory of a large world goes: build the bench's hbm-preset world (or a given
size), spawn the first batch, and list the largest live CUDA storages with the object attribute
that holds them.

    python scripts/lab/hbm_probe.py [map_size] [first_batch]
"""
import gc
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402


def owners(world) -> dict:
    """storage ptr -> attribute path, for the world, its kinetics, arenas and scratch."""
    out = {}

    def walk(obj, path, depth=0):
        if depth > 4:
            return
        if isinstance(obj, torch.Tensor):
            if obj.is_cuda:
                out.setdefault(obj.untyped_storage().data_ptr(), path)
            return
        if isinstance(obj, dict):
            for k, v in list(obj.items()):
                walk(v, f"{path}[{k!r}]", depth + 1)
        elif isinstance(obj, (list, tuple)):
            for i, v in enumerate(obj):
                walk(v, f"{path}[{i}]", depth + 1)
        elif hasattr(obj, "__dict__") and type(obj).__module__.startswith("magicsoup_amd"):
            for k, v in list(vars(obj).items()):
                walk(v, f"{path}.{k}", depth + 1)
        elif hasattr(obj, "__slots__"):
            for k in obj.__slots__:
                walk(getattr(obj, k, None), f"{path}.{k}", depth + 1)

    walk(world, "world")
    return out


def report(world, tag):
    torch.cuda.synchronize()
    own = owners(world)
    seen = {}
    for o in gc.get_objects():
        try:
            if isinstance(o, torch.Tensor) and o.is_cuda:
                st = o.untyped_storage()
                seen[st.data_ptr()] = st.nbytes()
        except Exception:  # noqa: BLE001
            pass
    top = sorted(seen.items(), key=lambda kv: -kv[1])[:25]
    print(json.dumps({"tag": tag, "allocated_gib": round(torch.cuda.memory_allocated() / 2**30, 2),
                      "live_tensor_gib": round(sum(seen.values()) / 2**30, 2),
                      "top": [(own.get(p, "?"), round(b / 2**30, 2)) for p, b in top]}), flush=True)


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 47872
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 500_000
    w = ms.World(chemistry=CHEMISTRY, map_size=size, device="cuda", seed=0, map_dtype=torch.float16)
    report(w, "empty")
    w.spawn_cells(bench.random_genomes(first, 500, "cuda"))
    w.synchronize()
    report(w, "first batch")
    print(json.dumps({"P": int(w.kinetics._P())}))
    w.kinetics._enter_slot_mode()
    w.synchronize()
    report(w, "slot mode")
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 7_000_000
    try:
        w.reserve_cells(n, 550)
        report(w, "reserved")
    except torch.OutOfMemoryError as e:
        print(json.dumps({"oom": str(e)[:300]}))
        report(w, "after oom")


if __name__ == "__main__":
    main()
