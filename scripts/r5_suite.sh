#!/bin/bash
# the GPU suite in two parts (per-part time limits): everything but the
# multi-rank tests, then the multi-rank tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PART=${1:-all}
T="python -u -m pytest -q --timeout 1200 --timeout-method thread -m gpu"
if [ "$PART" = "main" ] || [ "$PART" = all ]; then
  timeout -k 10 1000 $T tests --deselect tests/test_gpu_multirank.py > gpurun_out/suite_main.log 2>&1
  rc=$?; tail -5 gpurun_out/suite_main.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "$PART" = "multi" ] || [ "$PART" = all ]; then
  timeout -k 10 1100 $T tests/test_gpu_multirank.py > gpurun_out/suite_multi.log 2>&1
  rc=$?; tail -5 gpurun_out/suite_multi.log; exit $rc
fi
