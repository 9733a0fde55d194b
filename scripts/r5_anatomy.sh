#!/bin/bash
# Steady-iteration anatomy per library variant (PMX_LIB_VARIANT; "" = the
# product build): two driver benches each (alternated), then a rocprofv3
# kernel trace of the driver command and tools/trace_iter.py over it.
#   scripts/r5_anatomy.sh base wt nomath     (extra bench args in BENCH_ARGS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "$@"; do
    vv=$v; [ "$v" = base ] && vv=""
    PMX_LIB_VARIANT=$vv timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
        > gpurun_out/an_tmp.json 2>> gpurun_out/an.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/an_tmp.json')); print(json.dumps({'variant': sys.argv[1], 'ms_per_step': round(d['ms_per_step'],5), 'whole_ms_it': round(d['whole_icp']['ms_per_iteration'],5), 'first': d['whole_icp']['first_matches_us'][:3], 'match_ms': round(d['roofline']['avg_launch_ms'],5), 'setup_ms': round(d['setup_ms'],3)}))" "$v" | tee -a gpurun_out/an.jsonl
  done
done
for v in "$@"; do
  vv=$v; [ "$v" = base ] && vv=""
  (cd /tmp && PMX_LIB_VARIANT=$vv timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/an_$v" \
      -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
      > "$R/gpurun_out/an_$v.log" 2>&1) || exit 1
  f=$(find gpurun_out/an_$v -name '*kernel_trace.csv' | head -1)
  echo "== $v"; python3 tools/trace_iter.py "$f" 20
done
