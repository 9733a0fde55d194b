#!/bin/bash
# Quantile-window exactness tests only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_loop.py -x -q -m gpu -k "window" --timeout 120 --timeout-method thread > gpurun_out/tests_window.log 2>&1
