#!/bin/bash
# VarTrimmed head size probe: product (4096) vs h1k variant; c3v bench + kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" h1k; do
  PMX_LIB_VARIANT=$v timeout -k 10 300 python bench.py --config c3v --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/vt7_bench.json 2> gpurun_out/vt7_bench.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/vt7_bench.json')); print(sys.argv[1] or 'h4k', 'c3v ms/step', round(d['ms_per_step'],5))" "$v"
  (cd /tmp && PMX_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/vt7_prof_$v" -o run --output-format csv -- \
      python3 "$R/bench.py" --config c3v --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/vt7_prof.log" 2>&1) || exit 1
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if 'vt_' in r['Name']: print(sys.argv[2] or 'h4k', r['Name'].split('(')[0][-40:], r['AverageNs'])" gpurun_out/vt7_prof_$v/run_kernel_stats.csv "$v"
done
