#!/bin/bash
# the light lane kernel (every miss wave-cooperative, 6 waves per SIMD) vs the
# product build on C3 / C4, then the per-rank cost model for C3 and C4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # cfg, variant
  PMX_LIB_VARIANT=$2 timeout -k 10 300 python bench.py --config $1 --steps 20 --warmup 5 --no-cpu-baseline \
      > gpurun_out/r3_tmp.json 2>> gpurun_out/r3.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/r3_tmp.json')); print(json.dumps({'cfg': sys.argv[1], 'variant': sys.argv[2], 'ms_per_step': round(d['ms_per_step'],5), 'whole_ms_it': round(d['whole_icp']['ms_per_iteration'],5), 'first': d['whole_icp']['first_matches_us'], 'match_ms': round(d['roofline']['avg_launch_ms'],5)}))" $1 "$2" | tee -a gpurun_out/r3.jsonl
}
for rep in 1 2; do run c3 ""; run c3 light; done
run c4 ""; run c4 light
CFGS="c3 c4" bash scripts/r5_costmodel.sh
