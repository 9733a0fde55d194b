#!/bin/bash
# HIP runtime knobs vs the driver command (C3): kernel-argument placement
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/env_tmp.json 2>> gpurun_out/env.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/env_tmp.json')); print(json.dumps({'env': sys.argv[1:], 'ms_per_step': round(d['ms_per_step'],5), 'whole_ms_it': round(d['whole_icp']['ms_per_iteration'],5), 'match_ms': round(d['roofline']['avg_launch_ms'],5)}))" "$@" | tee -a gpurun_out/env.jsonl
}
for rep in 1 2; do
  run X=0
  run HIP_FORCE_DEV_KERNARG=1
  run HIP_FORCE_DEV_KERNARG=0
done
