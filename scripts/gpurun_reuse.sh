#!/bin/bash
# Validation of the grid match's temporal reuse: grid + loop + icp GPU tests,
# probe and bench with reuse on / off, and a kernel trace of the C3 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 900 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_loop.py tests/test_gpu_icp.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 &&
step probe && timeout -k 10 300 python tests/perf_probe.py 1000000 1000000 1 5 aligned > gpurun_out/probe/reuse.log 2>&1 &&
timeout -k 10 300 env PMX_GRID_REUSE=0 python tests/perf_probe.py 1000000 1000000 1 5 aligned > gpurun_out/probe/noreuse.log 2>&1 &&
for c in c3 c4 c5 c2; do
  step bench_$c && timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err &&
  step bench_${c}_B && timeout -k 10 300 env PMX_GRID_REUSE=0 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${c}_B.json 2> gpurun_out/bench_${c}_B.err || exit 1
done &&
step prof_trace && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1)
rc=$?
step "done rc=$rc"
exit $rc
