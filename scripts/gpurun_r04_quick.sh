#!/bin/bash
# Quick A/B of the C3 driver command over env variants (one bench each, two
# rounds), no profiles:  scripts/gpurun_r04_quick.sh "A=1" "A=1 B=2" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
        > gpurun_out/q_tmp.json 2>> gpurun_out/q.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/q_tmp.json')); print(json.dumps({'variant': sys.argv[1], 'ms_per_step': round(d['ms_per_step'],4), 'whole': round(d['whole_icp']['ms_per_iteration'],4), 'match_ms': round(d['roofline']['avg_launch_ms'],4)}))" "$v" | tee -a gpurun_out/q.jsonl
  done
done
