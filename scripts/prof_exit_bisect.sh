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
  local rc=$?
  echo "$1 rc=$rc"
  case $rc in 124|134|137|139) exit 0;; esac  # nothing more on the GPU after a crash
}
LOOP="import torch, bench, magicsoup_amd as ms; from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY as C; w = ms.World(chemistry=C, map_size=128, device='cuda', seed=0); w.spawn_cells(bench.random_genomes(2000, 500, 'cuda')); [bench.step(w, 2000, 500, C.molname_2_idx['ATP']) for _ in range(5)]; torch.cuda.synchronize(); print(w.n_cells)"
DIV="import torch, bench, magicsoup_amd as ms; from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY as C; w = ms.World(chemistry=C, map_size=128, device='cuda', seed=0); w.spawn_cells(bench.random_genomes(2000, 500, 'cuda')); [w.divide_cells(list(range(0, w.n_cells, 3))) for _ in range(3)]; torch.cuda.synchronize(); print(w.n_cells)"
case "${1:-coop}" in
  coop)
    MS_PLACE_MODE=1 v loop_place_rounds "$LOOP"
    MS_PLACE_MODE=1 v divide_place_rounds "$DIV"
    v divide_coop "$DIV" ;;
  release)
    v loop_release "$LOOP"
    MS_RELEASE_AT_EXIT=0 v loop_no_release "$LOOP" ;;
  ops)
    PRE="import torch, bench, magicsoup_amd as ms; from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY as C; w = ms.World(chemistry=C, map_size=128, device='cuda', seed=0); w.spawn_cells(bench.random_genomes(2000, 500, 'cuda')); a = C.molname_2_idx['ATP']"
    v ops_kill "$PRE
for _ in range(5): w.enzymatic_activity(); w.kill_cells(w.cell_molecules[:, a] < 1.0)
torch.cuda.synchronize()"
    v ops_divide "$PRE
for _ in range(5): w.enzymatic_activity(); w.divide_cells_t(w.cell_molecules[:, a] > 5.0)
torch.cuda.synchronize()"
    v ops_mutate "$PRE
for _ in range(5): w.mutate_cells(p=1e-4); w.diffuse_molecules()
torch.cuda.synchronize(); print(w.n_cells)"
    v ops_recombinate "$PRE
for _ in range(5): w.recombinate_cells(p=1e-4); w.diffuse_molecules()
torch.cuda.synchronize(); print(w.n_cells)" ;;
  coop2)
    PRE="import torch, bench, magicsoup_amd as ms; from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY as C; w = ms.World(chemistry=C, map_size=128, device='cuda', seed=0); w.spawn_cells(bench.random_genomes(2000, 500, 'cuda')); a = C.molname_2_idx['ATP']"
    MS_PLACE_MODE=1 v divide_list_rounds "$PRE
for _ in range(5): w.enzymatic_activity(); w.divide_cells(torch.nonzero(w.cell_molecules[:, a] > 5.0).flatten().tolist())
torch.cuda.synchronize()"
    v divide_list_coop "$PRE
for _ in range(5): w.enzymatic_activity(); w.divide_cells(torch.nonzero(w.cell_molecules[:, a] > 5.0).flatten().tolist())
torch.cuda.synchronize()" ;;
  maps)
    v world_loop_maps "$LOOP
open('$O/maps.txt', 'w').write(open('/proc/self/maps').read())" ;;
esac
exit 0
