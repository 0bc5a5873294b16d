"""When does a kernel launch block the host? A long device spin (torch.cuda._sleep) is queued,
then N small launches are issued; the host time of each launch call is recorded. Reports the
first launch that waited (> 50 us) and how long, for small-argument torch kernels and for the
framework's gather_rows kernel (1.4 KB of kernel arguments).

usage: python scripts/launch_block.py [n_launches]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from magicsoup_amd.ops import hip_ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
dev = "cuda"
x = torch.zeros(1024, device=dev)
src = torch.zeros(4096, 64, dtype=torch.uint8, device=dev)
dst = torch.zeros(4096, 64, dtype=torch.uint8, device=dev)
rows = torch.arange(4096, device=dev)


def spin_cycles(us):
    # calibrate: cycles per microsecond of torch.cuda._sleep
    return int(us * 2100)


def run(kind: str, spin_us: float):
    torch.cuda.synchronize()
    torch.cuda._sleep(spin_cycles(spin_us))
    ts = []
    for i in range(N):
        t0 = time.perf_counter()
        if kind == "add":
            x.add_(1.0)
        elif kind == "gather":
            hip_ops.gather_rows([(src, dst)] * 8, 4096, src_rows=rows)
        else:
            torch.cuda._sleep(10)
        ts.append((time.perf_counter() - t0) * 1e6)
    t_issue = sum(ts)
    torch.cuda.synchronize()
    blocked = [(i, round(t)) for i, t in enumerate(ts) if t > 50]
    print(f"{kind:7s} spin {spin_us:6.0f} us: issue total {t_issue:8.0f} us, median {sorted(ts)[N // 2]:.1f} us, "
          f"blocked {len(blocked)}: {blocked[:6]}")


t0 = time.perf_counter()
torch.cuda._sleep(spin_cycles(1000))
torch.cuda.synchronize()
print(f"calibration: 1000 us spin took {(time.perf_counter() - t0) * 1e6:.0f} us")
for kind in ("add", "gather", "sleep"):
    for spin in (2000, 10000):
        run(kind, spin)
