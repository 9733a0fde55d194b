#!/bin/bash
# Per-iteration match times of one C3 ICP (tools/iter_profile.py) under env
# variants, each in its own process.  scripts/gpurun_iters.sh variant...
# (a variant: comma-separated env settings, "default" = none)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/iters.jsonl
for v in "$@"; do
  env_args=()
  if [ "$v" != default ]; then IFS=',' read -ra kvs <<< "$v"; env_args=("${kvs[@]}"); fi
  echo "== $(date +%T) $v" | tee -a gpurun_out/steps.log
  env "${env_args[@]}" PROF_ITERS=${PROF_ITERS:-12} timeout -k 10 240 python3 tools/iter_profile.py > gpurun_out/iter_tmp.jsonl 2> gpurun_out/iter_err.log || { tail -5 gpurun_out/iter_err.log; exit 1; }
  python3 -c "
import json,sys
rows=[json.loads(l) for l in open('gpurun_out/iter_tmp.jsonl')]
print(json.dumps({'variant': sys.argv[1], 'match_us': [round(r['match_ms']*1e3,1) for r in rows],
  'full': [round(r['full_search_frac'],3) for r in rows], 'ppq': [round(r['pairs_per_query'],1) for r in rows]}))" "$v" | tee -a gpurun_out/iters.jsonl
done
