#!/bin/bash
# Which part of a run makes rocprofv3 (kernel trace) end in SIGSEGV at process exit? Each variant
# runs under its own time limit; the exit status of every run is printed (139 = SIGSEGV). The
# world_loop_maps variant saves its own /proc/self/maps so the crash frames can be symbolised.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/profexit; rm -rf $O; mkdir -p $O
v() {  # v <name> <python code>
  timeout -k 10 120 rocprofv3 --kernel-trace -d $O/$1 -o run --output-format csv -- python3 -c "$2" > $O/$1.log 2>&1
  echo "$1 rc=$?"
}
LOOP="import torch, bench, magicsoup_amd as ms; from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY as C; w = ms.World(chemistry=C, map_size=128, device='cuda', seed=0); w.spawn_cells(bench.random_genomes(2000, 500, 'cuda')); [bench.step(w, 2000, 500, C.molname_2_idx['ATP']) for _ in range(5)]; torch.cuda.synchronize(); print(w.n_cells)"
v pinned "import torch; t = torch.zeros(4, dtype=torch.int32, pin_memory=True); x = torch.ones(1000, device='cuda'); t.copy_(x[:4].int(), non_blocking=True); torch.cuda.synchronize(); print(int(t.sum()))"
v prio_stream "import torch; s = torch.cuda.Stream(priority=-1); ev = torch.cuda.Event(); x = torch.ones(1000, device='cuda')
with torch.cuda.stream(s): y = x * 2
ev.record(s); torch.cuda.current_stream().wait_event(ev); print(float(y.sum()))"
v world_loop_maps "$LOOP
open('$O/maps.txt', 'w').write(open('/proc/self/maps').read())"
v world_loop_exit "$LOOP
import os, sys; sys.stdout.flush(); os._exit(0)"
exit 0
