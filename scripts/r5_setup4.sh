#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PMX_SETUP_TRACE=2 timeout -k 10 300 python tools/setup_trace.py c3 > gpurun_out/setup4.out 2> gpurun_out/setup4.err || { tail -20 gpurun_out/setup4.err; exit 1; }
tail -36 gpurun_out/setup4.err
