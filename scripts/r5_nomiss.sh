#!/bin/bash
# timing experiment: the converged match without its misses' searches (wrong results; timing only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" nomiss; do
  (cd /tmp && PMX_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/nm_$v" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/nm.log" 2>&1) || exit 1
  python3 tools/pmc_phases.py gpurun_out/nm_$v - - 5 20 x > gpurun_out/nm_$v.json || exit 1
  python3 -c "
import json,sys
p=json.load(open(sys.argv[1])); m=p['match']
print(sys.argv[2] or 'base', 'match timed', m['timed']['avg_ns'], [x for x in m['timed']['launch_ns']][:6])
for k,v in list(p['timed_kernels']['kernels'].items())[:6]: print('   ', k.split('(')[0][-40:], round(v['avg_ns']))" gpurun_out/nm_$v.json "$v"
done
