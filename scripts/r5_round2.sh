#!/bin/bash
# coop threshold A/B (C3, C4), the steady-iteration anatomy (kernel trace), and
# the per-rank cost model for C3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # cfg, env...
  local cfg=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline \
      > gpurun_out/r2_tmp.json 2>> gpurun_out/r2.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/r2_tmp.json')); t=d['timed_iterations']; print(json.dumps({'cfg': sys.argv[1], 'env': sys.argv[2:], 'ms_per_step': round(d['ms_per_step'],5), 'whole_ms_it': round(d['whole_icp']['ms_per_iteration'],5), 'first': d['whole_icp']['first_matches_us'], 'match_ms': round(d['roofline']['avg_launch_ms'],5), 'setup_ms': round(d['setup_ms'],3), 'setup_parts': d['setup_parts']}))" $cfg "$@" | tee -a gpurun_out/r2.jsonl
}
for rep in 1 2; do
  for c in 0 4 8 16; do run c3 PMX_COOP_MAX=$c; done
done
for c in 0 4 8 16; do run c4 PMX_COOP_MAX=$c; done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/an_base" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/an_base.log" 2>&1) || exit 1
f=$(find gpurun_out/an_base -name '*kernel_trace.csv' | head -1)
python3 tools/trace_iter.py "$f" 20 | tee gpurun_out/an_base_iter.txt
CFGS=c3 bash scripts/r5_costmodel.sh
