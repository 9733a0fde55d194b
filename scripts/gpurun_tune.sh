#!/bin/bash
# First-level sweep (grid level of a new reading's cold match) on the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
for p in 4 8 16 32 64; do
  for r in 1 2; do
    step first_$p.$r && PMX_GRID_FIRST_PPC=$p timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/first_$p.$r.json 2>gpurun_out/first_$p.$r.err || exit 1
  done
done
step "done"
