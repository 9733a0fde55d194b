#!/bin/bash
# End-of-round session: full GPU parity suite, smoke, then the final bench
# lines, kernel trace and PMC traffic (scripts/gpurun_final.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 &&
step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
bash scripts/gpurun_final.sh
