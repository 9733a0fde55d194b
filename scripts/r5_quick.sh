#!/bin/bash
# quick C3 / C4 benches (two each)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do for cfg in ${CFGS:-c3 c4}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/q_b.json 2> gpurun_out/q_b.err || { tail -5 gpurun_out/q_b.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/q_b.json') if l.startswith('{')][-1]); print(sys.argv[1], 'ms/step', round(d['ms_per_step'],5), 'whole', round(d['whole_icp']['ms_per_iteration'],5), 'match', round(d['roofline']['avg_launch_ms'],5))" $cfg
done; done
