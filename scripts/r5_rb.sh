#!/bin/bash
# reduction grid A/B (512 product vs 1024 / 256 variants) at C3 and C4, with the neighbour records
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do for cfg in c3 c4; do for v in "" rb1024 rb256; do
  PMX_LIB_VARIANT=$v timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/rb_b.json 2> gpurun_out/rb_b.err || { tail -5 gpurun_out/rb_b.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/rb_b.json') if l.startswith('{')][-1]); print(sys.argv[1], sys.argv[2] or 'rb512', 'ms/step', round(d['ms_per_step'],5), 'whole', round(d['whole_icp']['ms_per_iteration'],5))" $cfg "$v"
done; done; done
