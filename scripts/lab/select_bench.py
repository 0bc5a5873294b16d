"""Device time of one order-preserving selection (select.hip): the single-pass form (select_lb.h)
against the count + write pair, per size; CUDA-event timing over back-to-back calls.

    python scripts/lab/select_bench.py [iters]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from magicsoup_amd.ops import native  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    m = native.hip()
    for n in (6250, 50_000, 200_000, 1_000_000):
        mask = (torch.rand(n, device="cuda") < 0.9).view(torch.uint8)
        sel = torch.empty(n, dtype=torch.int64, device="cuda")
        dc = torch.empty(2, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        args = (n, 0, mask.data_ptr(), sel.data_ptr(), 0, dc.data_ptr(), st)
        row = {"n": n}
        for single, items in ((0, 16), (1, 1), (1, 4), (1, 16)):
            m.set_select_single_pass(single, items)
            for _ in range(10):
                m.select_indices_async(*args)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(iters):
                m.select_indices_async(*args)
            b.record()
            b.synchronize()
            row[f"single{single}_items{items}_us"] = round(a.elapsed_time(b) * 1e3 / iters, 2)
        print(json.dumps(row), flush=True)
    m.set_select_single_pass(1, 4)


if __name__ == "__main__":
    main()
