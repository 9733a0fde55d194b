#!/bin/bash
# Parameter sweep of the grid matcher on C3 (bench lines only); stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
CFG=${SWEEP_CONFIG:-c3}
step tests_grid && timeout -k 10 600 python -m pytest tests/test_gpu_grid.py -q -x > gpurun_out/tests_grid.log 2>&1 || exit $?
for mode in ${SWEEP_MODES:-tile lane}; do
  for ppc in ${SWEEP_PPC:-2 4 8 16 32}; do
    step "$mode ppc=$ppc"
    PMX_GRID_MODE=$mode PMX_GRID_PPC=$ppc timeout -k 10 300 python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/sweep/${CFG}_${mode}_${ppc}.json 2> gpurun_out/sweep/${CFG}_${mode}_${ppc}.err || exit $?
  done
done
step done
