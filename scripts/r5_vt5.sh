#!/bin/bash
# radix tile A/B (16 items product vs 8 items variant): VarTrimmed tests + c3v benches + sort kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ""; do
  PMX_LIB_VARIANT=$v timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "vartrim or VarTrim or vt" \
      > gpurun_out/vt5_tests.log 2>&1 || { tail -30 gpurun_out/vt5_tests.log; exit 1; }
  tail -1 gpurun_out/vt5_tests.log
done
for rep in 1 2; do for v in ""; do
  PMX_LIB_VARIANT=$v timeout -k 10 300 python bench.py --config c3v --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/vt5_bench.json 2> gpurun_out/vt5_bench.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/vt5_bench.json')); print(sys.argv[1] or 'it16', 'c3v ms/step', round(d['ms_per_step'],5), 'whole', round(d['whole_icp']['ms_per_iteration'],5))" "$v"
done; done
for v in ""; do
  (cd /tmp && PMX_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/vt5_prof_$v" -o run --output-format csv -- \
      python3 "$R/bench.py" --config c3v --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/vt5_prof.log" 2>&1) || exit 1
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]: print(sys.argv[2] or 'it16', r['Name'].split('(')[0][-40:], r['AverageNs'])" gpurun_out/vt5_prof_$v/run_kernel_stats.csv "$v"
done
