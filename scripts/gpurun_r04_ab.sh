#!/bin/bash
# A/B of the C3 driver command: the in-launch finalize on / off, each with a
# rocprofv3 kernel-trace summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
for v in 1 0 1 0; do
  step bench_tail$v && PMX_RED_TAIL=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
      >> gpurun_out/ab_tail$v.jsonl 2>> gpurun_out/ab.err || exit 1
done
for v in 1 0; do
  step prof_tail$v && (cd /tmp && PMX_RED_TAIL=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_tail$v" \
      -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline \
      > "$R/gpurun_out/prof_tail$v.log" 2>&1) || exit 1
done
step done
