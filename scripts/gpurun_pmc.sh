#!/bin/bash
# HBM traffic of the C3 bench's kernels: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 --pmc passes (TCC budget: FETCH_SIZE 3 counters, WRITE_SIZE 2),
# plus the kernel-trace summary of the same command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="$R/bench.py --steps 20 --warmup 3 --no-cpu-baseline"
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step trace && (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pmc_trace" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/pmc_trace.log" 2>&1) &&
step fetch && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/pmc_fetch.log" 2>&1) &&
step write && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/pmc_write.log" 2>&1)
rc=$?
step "done rc=$rc"
exit $rc
