#!/bin/bash
# VarTrimmed after the walk rework: bit-identity tests, then the c3v bench and walk timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_loop.py \
    -k "vartrim or VarTrim or vt" > gpurun_out/vt2_tests.log 2>&1 || { tail -30 gpurun_out/vt2_tests.log; exit 1; }
tail -2 gpurun_out/vt2_tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --config c3v --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/vt2_bench.json 2> gpurun_out/vt2_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/vt2_bench.json')); print('c3v ms/step', d['ms_per_step'], 'whole', d['whole_icp']['ms_per_iteration'])"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/vt2_prof" -o run --output-format csv -- \
    python3 "$R/bench.py" --config c3v --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/vt2_prof.log" 2>&1) || exit 1
PMX_VT_TRACE=1 timeout -k 10 300 python tools/vt_trace.py 10 > gpurun_out/vt2_trace.out 2> gpurun_out/vt2_trace.err || exit 1
