#!/bin/bash
# AddressSanitizer + UndefinedBehaviorSanitizer run of the OpenMP host core (CPU only).
#
# 1. builds the host core (csrc/host/*.cpp) with -fsanitize=address,undefined into build/asan/;
# 2. builds `pyasan`, CPython embedded in an ASan-linked executable (the ASan runtime then comes
#    first in the process without any preloading);
# 3. runs the host-side tests through it, with MS_HOST_SO pointing the loader (ops/native.py) at
#    the instrumented module. Any ASan report or UBSan diagnostic fails the run
#    (halt_on_error, UBSan errors are made fatal).
#
# usage: scripts/sanitize_host.sh [pytest args...]   (default: the host-core test files)
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=build/asan
mkdir -p "$OUT"
PYINC=$(python3 -c "import sysconfig; print(sysconfig.get_paths()['include'])")
PBINC=$(python3 -c "import pybind11; print(pybind11.get_include())")
EXT=$(python3 -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer"
objs=()
for src in magicsoup_amd/csrc/host/*.cpp; do
  o="$OUT/$(basename "${src%.cpp}").o"
  g++ -O1 -g -std=c++17 -fPIC -fopenmp $SAN -Imagicsoup_amd/csrc/include -I"$PBINC" -I"$PYINC" -c "$src" -o "$o" &
  objs+=("$o")
done
wait
g++ -shared -fopenmp $SAN "${objs[@]}" -o "$OUT/_host$EXT"
cat > "$OUT/pyasan.c" <<'EOF'
#include <Python.h>
int main(int argc, char** argv) { return Py_BytesMain(argc, argv); }
EOF
gcc -O1 -g $SAN "$OUT/pyasan.c" $(python3-config --includes) $(python3-config --ldflags --embed) -o "$OUT/pyasan"
export MS_HOST_SO="$PWD/$OUT/_host$EXT" PYTHONHOME="$(python3 -c 'import sys; print(sys.base_prefix)')"
export PYTHONPATH="$PWD:$(python3 -c 'import site; print(":".join(site.getsitepackages()))')"
# CPython and torch are not instrumented: leaks at interpreter exit are theirs, not the core's
export ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=86:protect_shadow_gap=0"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87"
export OMP_NUM_THREADS=4
if [ $# -eq 0 ]; then
  set -- tests/test_lib.py tests/test_genetics.py tests/test_mutations.py tests/test_kinetics_reference_cases.py \
         tests/test_kinetics.py tests/test_kinetics_cases.py tests/test_util_containers.py tests/test_world.py
fi
"$OUT/pyasan" -c "import magicsoup_amd.ops.native as n, os; m = n.host(); assert m.__file__ == os.environ['MS_HOST_SO'], m.__file__; print('instrumented host core:', m.__file__)"
exec "$OUT/pyasan" -m pytest -x -q -p no:cacheprovider -m "not gpu and not slow" "$@"
