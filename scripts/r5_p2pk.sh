#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_icp.py tests/test_gpu_loop.py tests/test_gpu_kernels.py > gpurun_out/p2pk_tests.log 2>&1 || { tail -30 gpurun_out/p2pk_tests.log; exit 1; }
tail -1 gpurun_out/p2pk_tests.log
CFGS="c4 c3" bash scripts/r5_quick.sh
