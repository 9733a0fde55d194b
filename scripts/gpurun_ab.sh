#!/bin/bash
# A/B session: grid + loop GPU tests, then the C3/C4/C5 bench with and without
# an environment knob ($AB_ENV, e.g. "PMX_GRID_HINT=0"), then a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_ENV="${AB_ENV:-PMX_GRID_HINT=0}"
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 &&
for c in c3 c4 c5; do
  step bench_$c && timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err &&
  step bench_${c}_B && timeout -k 10 300 env $AB_ENV python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${c}_B.json 2> gpurun_out/bench_${c}_B.err || exit 1
done &&
step prof_trace && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1)
rc=$?
step "done rc=$rc"
exit $rc
