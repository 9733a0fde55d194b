#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_icp.py tests/test_gpu_icp_sequence.py tests/test_gpu_grid.py tests/test_gpu_loop.py tests/test_gpu_configs.py tests/test_gpu_normals.py > gpurun_out/setup_tests.log 2>&1 || { tail -30 gpurun_out/setup_tests.log; exit 1; }
tail -1 gpurun_out/setup_tests.log
bash scripts/r5_setup2.sh
