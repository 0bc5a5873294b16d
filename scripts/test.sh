#!/bin/bash
# Build the native modules in-tree and run the test suite.
#   scripts/test.sh            CPU tests (no GPU needed)
#   scripts/test.sh gpu        GPU tests (MI355X / gfx950), each with its own time limit
#   scripts/test.sh slow       long-running statistical / invariant checks
#   scripts/test.sh sanitize   host core under ASan + UBSan (scripts/sanitize_host.sh)
set -euo pipefail
cd "$(dirname "$0")/.."
python -m magicsoup_amd.ops.build -j "${MAX_JOBS:-8}"
case "${1:-cpu}" in
  cpu)  python -m pytest tests -x -q -m "not gpu" ;;
  gpu)  python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ;;
  slow) python -m pytest tests -x -q -m slow ;;
  sanitize) exec scripts/sanitize_host.sh ;;
  *)    echo "usage: $0 [cpu|gpu|slow|sanitize]"; exit 2 ;;
esac
