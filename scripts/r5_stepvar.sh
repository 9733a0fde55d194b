#!/bin/bash
# step kernel timing variants (base / no conditioning bound / no arithmetic): the fused finalize+step launch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" nowc nomath; do
  (cd /tmp && PMX_LIB_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/sv_$v" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/sv.log" 2>&1) || exit 1
  python3 tools/pmc_phases.py gpurun_out/sv_$v - - 5 20 x > gpurun_out/sv_$v.json || exit 1
  python3 -c "
import json,sys
p=json.load(open(sys.argv[1]))
for k,v in p['timed_kernels']['kernels'].items():
    if 'step' in k: print(sys.argv[2] or 'base', k.split('(')[0][-40:], round(v['avg_ns']), 'busy/it', round(p['timed_kernels']['busy_ns_per_iteration']))" gpurun_out/sv_$v.json "$v"
done
