#!/bin/bash
# VarTrimmed with the fill-free radix sort: bit-identity tests (every VarTrimmed
# GPU test), then the c3v bench and its timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "vartrim or VarTrim or vt or c3v" \
    > gpurun_out/vt4_tests.log 2>&1 || { tail -30 gpurun_out/vt4_tests.log; exit 1; }
tail -1 gpurun_out/vt4_tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --config c3v --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/vt4_bench.json 2> gpurun_out/vt4_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/vt4_bench.json')); print('c3v ms/step', d['ms_per_step'], 'whole', d['whole_icp']['ms_per_iteration'])"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/vt4_prof" -o run --output-format csv -- \
    python3 "$R/bench.py" --config c3v --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/vt4_prof.log" 2>&1) || exit 1
