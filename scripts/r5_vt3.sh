#!/bin/bash
# VarTrimmed head size A/B (8 K product vs 4 K variant): tests, benches, kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" h4k; do
  PMX_LIB_VARIANT=$v timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
      -k "vartrim" > gpurun_out/vt3_tests.log 2>&1 || { tail -30 gpurun_out/vt3_tests.log; exit 1; }
  tail -1 gpurun_out/vt3_tests.log
done
for rep in 1 2; do for v in "" h4k; do
  PMX_LIB_VARIANT=$v timeout -k 10 300 python bench.py --config c3v --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/vt3_bench.json 2> gpurun_out/vt3_bench.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/vt3_bench.json')); print(sys.argv[1] or 'h8k', 'c3v ms/step', round(d['ms_per_step'],5), 'whole', round(d['whole_icp']['ms_per_iteration'],5))" "$v"
done; done
for v in "" h4k; do
  (cd /tmp && PMX_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/vt3_prof_$v" -o run --output-format csv -- \
      python3 "$R/bench.py" --config c3v --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/vt3_prof.log" 2>&1) || exit 1
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:4]: print(sys.argv[2] or 'h8k', r['Name'].split('(')[0][-40:], r['AverageNs'])" gpurun_out/vt3_prof_$v/run_kernel_stats.csv "$v"
done
