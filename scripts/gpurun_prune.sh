#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 &&
step bench && timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err &&
step bench_cold && timeout -k 10 600 python bench.py --no-cpu-baseline --warmup 1 --steps 40 > gpurun_out/bench_w1.json 2> gpurun_out/bench_w1.err &&
for c in c2 c4 c5; do
  step bench_$c && timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 1
done &&
step prof && (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1)
rc=$?
step "done rc=$rc"
exit $rc
