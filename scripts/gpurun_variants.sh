#!/bin/bash
# A/B runs of the driver's bench command under knob settings (development):
#   scripts/gpurun_variants.sh "PMX_FUSE_FINAL=0" "PMX_SELECT_ALL=0,PMX_FUSE_FINAL=0" ...
# Each argument is one comma-separated env setting ("" = defaults); one JSON
# summary line per run into gpurun_out/variants.jsonl.  With EXTRA set, its
# commands run afterwards (e.g. the per-iteration probe).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/variants.jsonl
for v in "$@"; do
  env_args=()
  IFS=',' read -ra kvs <<< "$v"
  for kv in "${kvs[@]}"; do [ -n "$kv" ] && env_args+=("$kv"); done
  echo "== $(date +%T) variant [$v]" >> gpurun_out/steps.log
  out=$(timeout -k 10 300 env "${env_args[@]}" python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
        2> gpurun_out/variant_err.log) || { echo "variant [$v] failed" >> gpurun_out/steps.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads(sys.argv[2]); print(json.dumps({'variant': sys.argv[1], 'ms_per_step': d['ms_per_step'],
 'match_ms': d['roofline']['avg_launch_ms'], 'setup_ms': d.get('setup_ms')}))" "$v" "$out" >> gpurun_out/variants.jsonl
done
if [ -n "$EXTRA" ]; then
  echo "== $(date +%T) extra" >> gpurun_out/steps.log
  timeout -k 10 600 bash -c "$EXTRA" > gpurun_out/extra.log 2>&1 || exit 1
fi
echo "== $(date +%T) done" >> gpurun_out/steps.log
