#!/bin/bash
# GPU session: parity tests (device loop included), C3 bench with CPU baseline,
# C2/C4/C5 bench lines, rocprofv3 kernel-trace summary of the C3 bench.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 &&
step bench_c3 && timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err &&
step bench_c2 && timeout -k 10 300 python bench.py --config c2 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err &&
step bench_c4 && timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err &&
step bench_c5 && timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err &&
step prof_trace && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1)
rc=$?
step "done rc=$rc"
exit $rc
