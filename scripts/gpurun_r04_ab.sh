#!/bin/bash
# A/B of the C3 driver command over tuning knobs (env assignments as args,
# e.g. "PMX_RED_TAIL=0" "PMX_LANE_OCC=6"), alternated twice, then the
# rocprofv3 kernel-trace summary of the first variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
VARIANTS=("$@")
[ ${#VARIANTS[@]} -eq 0 ] && VARIANTS=("BASE=1")
for rep in 1 2; do
  for v in "${VARIANTS[@]}"; do
    step "bench $v" && env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
        > gpurun_out/ab_tmp.json 2>> gpurun_out/ab.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_tmp.json')); print(json.dumps({'variant': sys.argv[1], 'ms_per_step': d['ms_per_step'], 'whole_ms_it': d['whole_icp']['ms_per_iteration'], 'first': d['whole_icp']['first_matches_us'], 'match_ms': d['roofline']['avg_launch_ms'], 'setup_ms': d['setup_ms'], 'seq_ms': d.get('sequence_scan_ms')}))" "$v" >> gpurun_out/ab.jsonl
  done
done
for v in "${VARIANTS[@]}"; do
  tag=$(echo "$v" | tr '=' '_')
  step "prof $v" && (cd /tmp && env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$tag" \
      -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
      > "$R/gpurun_out/prof_$tag.log" 2>&1) || exit 1
done
step done
