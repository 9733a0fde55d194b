#!/bin/bash
# A/B of variants on the driver's bench command and on the whole ICP from the
# initial pose (development).  A variant is comma-separated env settings
# ("default" = none), e.g. PMX_COLD_TILE=0 or PMX_LIB_VARIANT=vX (lib/vX/).
#   scripts/gpurun_ab.sh [tests] -- variant...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
if [ "$1" = tests ]; then
  shift
  step tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_loop.py tests/test_gpu_icp.py \
      tests/test_gpu_vardist.py tests/test_gpu_kernels.py -m gpu -q --maxfail 10 --timeout 180 --timeout-method thread > gpurun_out/tests_ab.log 2>&1 || exit $?
fi
[ "$1" = -- ] && shift
for rep in 1 2; do
  for v in "$@"; do
    env_args=()
    if [ "$v" != default ]; then IFS=',' read -ra kvs <<< "$v"; env_args=("${kvs[@]}"); fi
    for w in 5 0; do
      step "$v warmup $w rep $rep"
      out=$(env "${env_args[@]}" timeout -k 10 300 python3 bench.py --gpus 1 --steps $([ $w = 5 ] && echo 20 || echo 40) \
            --warmup $w --no-cpu-baseline 2> gpurun_out/ab_err.log) || { step "failed $v"; exit 1; }
      python3 -c "
import json,sys
d=json.loads(sys.argv[3]); r=d['roofline']
print(json.dumps({'variant': sys.argv[1], 'warmup': int(sys.argv[2]), 'ms_per_step': d['ms_per_step'],
 'match_ms': r['avg_launch_ms'], 'cold_ms': r.get('cold_launch_ms'), 'parity': d.get('parity', {}).get('pass')}))" \
        "$v" "$w" "$out" >> gpurun_out/ab.jsonl
    done
  done
done
step done
