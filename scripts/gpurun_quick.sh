#!/bin/bash
# Short GPU session: parity tests, then C3 (tile and per-lane grid kernels) and C4 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/tests_gpu.log 2>&1 &&
step bench_c3 && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err &&
step bench_c3_lane && PMX_GRID_MODE=lane timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3_lane.json 2> gpurun_out/bench_c3_lane.err &&
step bench_c4 && timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err &&
step bench_c5 && timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err &&
step prof_trace && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1)
rc=$?
step "done rc=$rc"
exit $rc
