#!/bin/bash
# Round bench session: the default bench line (C3 + CPU baseline), the other
# configs' lines, the kernel-trace summary of the default command, and the
# HBM traffic of the same command (FETCH_SIZE / WRITE_SIZE in separate
# rocprofv3 --pmc passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step bench && timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err &&
for c in c2 c4 c5; do
  step bench_$c && timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 1
done &&
step prof && (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1) &&
step fetch && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/pmc_fetch.log" 2>&1) &&
step write && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/pmc_write.log" 2>&1)
rc=$?
step "done rc=$rc"
exit $rc
