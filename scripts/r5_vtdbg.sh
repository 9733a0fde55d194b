#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PMX_VT_TRACE=1 timeout -k 10 300 python tools/vt_debug.py jump f32 > gpurun_out/vtdbg.out 2> gpurun_out/vtdbg.err
echo "exit $?"; cat gpurun_out/vtdbg.out; grep -c vt_trace gpurun_out/vtdbg.err
