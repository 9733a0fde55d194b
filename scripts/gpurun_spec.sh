#!/bin/bash
# Quantile-window session: loop / grid / kernel parity tests, default bench,
# a select-grid variant, and the kernel-trace summary of the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 &&
step bench && timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err &&
step bench_nospec && PMX_SPEC_SELECT=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_nospec.json 2> gpurun_out/bench_nospec.err &&
step prof && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1)
rc=$?
step "done rc=$rc"
exit $rc
