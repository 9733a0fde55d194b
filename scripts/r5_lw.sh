#!/bin/bash
# per-lane kernel waves per SIMD A/B (4 product vs 5 / 6 with spills) at C3 and C4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do for cfg in c3 c4; do for v in "" lw5 lw6; do
  PMX_LIB_VARIANT=$v timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lw_b.json 2> gpurun_out/lw_b.err || { tail -5 gpurun_out/lw_b.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/lw_b.json') if l.startswith('{')][-1]); print(sys.argv[1], sys.argv[2] or 'lw4', 'ms/step', round(d['ms_per_step'],5), 'whole', round(d['whole_icp']['ms_per_iteration'],5))" $cfg "$v"
done; done; done
