#!/bin/bash
# HBM traffic and per-phase kernel times of the C3 driver command: the kernel
# trace, FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (TCC budget:
# FETCH_SIZE 3 counters, WRITE_SIZE 2), then tools/pmc_phases.py over the three
# (the match's timed / roofline / cold phases and every kernel of the timed
# iterations) -> gpurun_out/pmc_c3_driver.json
#   scripts/gpurun_r04_pmc.sh [extra bench args...]   (PMC_TAG=c5 -> pmc_c5_driver.json)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
W=5; K=20
TAG="${PMC_TAG:-c3}"
CMD="$R/bench.py --steps $K --warmup $W --no-cpu-baseline $*"
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
rm -rf gpurun_out/pmc_trace gpurun_out/pmc_fetch gpurun_out/pmc_write
step pmc_trace && (cd /tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pmc_trace" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/pmc_trace.log" 2>&1) &&
step pmc_fetch && (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/pmc_fetch.log" 2>&1) &&
step pmc_write && (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/pmc_write.log" 2>&1) &&
python3 tools/pmc_phases.py gpurun_out/pmc_trace gpurun_out/pmc_fetch gpurun_out/pmc_write $W $K "python3 bench.py --steps $K --warmup $W --no-cpu-baseline $*" > gpurun_out/pmc_${TAG}_driver.json
rc=$?
step "pmc done rc=$rc"
exit $rc
