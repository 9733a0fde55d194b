#!/bin/bash
# VarTrimmed (c3v): bench line, kernel stats of the driver command, the walk's timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c3v --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/vt_bench.json 2> gpurun_out/vt_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/vt_bench.json')); print('c3v ms/step', d['ms_per_step'], 'whole', d['whole_icp']['ms_per_iteration'])"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/vt_prof" -o run --output-format csv -- \
    python3 "$R/bench.py" --config c3v --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/vt_prof.log" 2>&1) || exit 1
PMX_VT_TRACE=1 timeout -k 10 300 python tools/vt_trace.py 10 > gpurun_out/vt_trace.out 2> gpurun_out/vt_trace.err || exit 1
tail -5 gpurun_out/vt_trace.out
