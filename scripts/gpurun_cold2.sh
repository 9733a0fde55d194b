#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tests/cold_probe.py c3 > gpurun_out/cold_c3.log 2>&1 &&
timeout -k 10 300 python tests/cold_probe.py c2 > gpurun_out/cold_c2.log 2>&1 &&
timeout -k 10 300 env PMX_GRID_REUSE=0 python tests/cold_probe.py c3 > gpurun_out/cold_c3_noreuse.log 2>&1
