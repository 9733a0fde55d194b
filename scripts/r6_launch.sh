#!/bin/bash
# Round 6: the launch-boundary probe (tools/launch_probe.hip) plain, with the
# kernarg placement toggled, and under the kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out/launch
export TMPDIR=/tmp
timeout -k 10 60 tools/launch_probe 400 > gpurun_out/launch/plain.jsonl || exit 1
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 60 tools/launch_probe 400 > gpurun_out/launch/kernarg0.jsonl || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 60 tools/launch_probe 400 > gpurun_out/launch/kernarg1.jsonl || exit 1
(cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/launch/trace" -o run --output-format csv -- "$R/tools/launch_probe" 400 > "$R/gpurun_out/launch/traced.jsonl" 2> "$R/gpurun_out/launch/traced.err") || exit 1
cat gpurun_out/launch/plain.jsonl
