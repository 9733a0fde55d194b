#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in 0 1; do PROBE_MIRROR=$m timeout -k 10 120 python tools/reuse_visits.py 1 || exit 1; done
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_grid.py -k "reuse_stays_exact and lane" > gpurun_out/diag_grid2.log 2>&1; grep -E "visits|passed|failed" gpurun_out/diag_grid2.log | head -20
