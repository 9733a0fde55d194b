#!/bin/bash
# Reduction-grid sweep: kernel trace of the default bench for builds with
# 512 (default), 1024 and 2048 p2plane blocks (lib/r<N>/ variants).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
for v in "" r256 r128; do
  n=${v:-r512}
  step $n && (cd /tmp && PMX_LIB_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$n" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/prof_$n.log" 2>&1) || exit 1
done
step done
