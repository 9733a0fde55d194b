#!/bin/bash
# One GPU session: parity tests, benches, rocprof kernel-trace summary.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/tests_gpu.log 2>&1 &&
step bench_c3 && timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err &&
step bench_c2 && timeout -k 10 300 python bench.py --config c2 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2.json 2>&1 &&
step prof && (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c3_grid" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_c3_grid.log" 2>&1)
rc=$?
step "done rc=$rc"
exit $rc
