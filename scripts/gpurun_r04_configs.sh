#!/bin/bash
# Per-config bench lines (C2 / C4 / C5, each with its CPU baseline and
# parity block) plus the rocprofv3 kernel-trace summary of each command.
#   scripts/gpurun_r04_configs.sh [configs...]   (default: c2 c4 c5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFGS="${*:-c2 c4 c5}"
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
for c in $CFGS; do
  cap=100; [ "$c" = c5 ] && cap=30
  step bench_$c && timeout -k 10 420 python bench.py --config $c --steps 20 --warmup 5 --cpu-one-thread-cap $cap \
      > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 1
  step pmc_$c && PMC_TAG=$c bash scripts/gpurun_r04_pmc.sh --config $c || exit 1
  mkdir -p gpurun_out/prof_$c && cp gpurun_out/pmc_trace/run_kernel_stats.csv gpurun_out/prof_$c/ || exit 1
done
step "done"
