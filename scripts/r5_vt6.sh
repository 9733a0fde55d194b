#!/bin/bash
# VarTrimmed walk with in-wave crossings: parity tests, c3v benches, walk trace, kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "vartrim or VarTrim or vt" \
    > gpurun_out/vt6_tests.log 2>&1 || { tail -30 gpurun_out/vt6_tests.log; exit 1; }
tail -1 gpurun_out/vt6_tests.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c3v --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/vt6_bench.json 2> gpurun_out/vt6_bench.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/vt6_bench.json')); print('c3v ms/step', round(d['ms_per_step'],5), 'whole', round(d['whole_icp']['ms_per_iteration'],5))"
done
PMX_VT_TRACE=1 timeout -k 10 300 python tools/vt_trace.py 10 > gpurun_out/vt6_trace.out 2> gpurun_out/vt6_trace.err || exit 1
grep -c vt_trace gpurun_out/vt6_trace.err; tail -3 gpurun_out/vt6_trace.err
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/vt6_prof" -o run --output-format csv -- \
    python3 "$R/bench.py" --config c3v --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/vt6_prof.log" 2>&1) || exit 1
python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:10]: print(r['Name'].split('(')[0][-40:], r['AverageNs'])" gpurun_out/vt6_prof/run_kernel_stats.csv
