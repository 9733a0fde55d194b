#!/bin/bash
# Round 6: kernel traces of the driver command (C3) with options A / B
# (PMX_OPTS), per-iteration anatomy by tools/trace_iter.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
export TMPDIR=/tmp
if [ -n "$DIST" ]; then export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29519; fi
mkdir -p gpurun_out/trace
i=0
for opt in "$@"; do
  i=$((i+1))
  rm -rf gpurun_out/trace/t$i
  (cd /tmp && PMX_OPTS="$opt" timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/trace/t$i" -o run --output-format csv -- python3 "$R/bench.py" --config ${CFG:-c3} --steps 20 --warmup 5 --no-cpu-baseline $EXTRA > "$R/gpurun_out/trace/t$i.log" 2>&1) || exit 1
  echo "== $opt"
  TRACE_ALL=1 python3 tools/trace_iter.py gpurun_out/trace/t$i/run_kernel_trace.csv > gpurun_out/trace/iter$i.txt 2>&1 || true
  head -24 gpurun_out/trace/iter$i.txt
done
