#!/bin/bash
# Round-5 experiment: parity of the wave-cooperative miss search (default on)
# and of the reuse candidates (PMX_REUSE_CAND=4), then A/B benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_grid.py tests/test_gpu_loop.py tests/test_gpu_configs.py \
    tests/test_gpu_robust.py -k "not equals_modules or second" > gpurun_out/exp_tests_coop.log 2>&1 || { tail -30 gpurun_out/exp_tests_coop.log; exit 1; }
tail -2 gpurun_out/exp_tests_coop.log
PMX_REUSE_CAND=4 timeout -k 10 600 $T tests/test_gpu_grid.py tests/test_gpu_loop.py tests/test_gpu_configs.py \
    > gpurun_out/exp_tests_cand.log 2>&1 || { tail -30 gpurun_out/exp_tests_cand.log; exit 1; }
tail -2 gpurun_out/exp_tests_cand.log
run() {  # cfg, env...
  local cfg=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline \
      > gpurun_out/exp_tmp.json 2>> gpurun_out/exp.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/exp_tmp.json')); t=d['timed_iterations']; print(json.dumps({'cfg': sys.argv[1], 'env': sys.argv[2:], 'ms_per_step': round(d['ms_per_step'],5), 'whole_ms_it': round(d['whole_icp']['ms_per_iteration'],5), 'first': d['whole_icp']['first_matches_us'], 'match_ms': round(d['roofline']['avg_launch_ms'],5), 'full': t['full_searches'][:8], 'levels': t['levels'][:8]}))" $cfg "$@" | tee -a gpurun_out/exp.jsonl
}
for rep in 1 2; do
  run c3 PMX_COOP_MAX=0
  run c3 PMX_COOP_MAX=16
  run c3 PMX_COOP_MAX=64
done
run c3 PMX_REUSE_CAND=2
run c5 PMX_REUSE_CAND=0 PMX_COOP_MAX=0
run c5 PMX_REUSE_CAND=0
run c5 PMX_REUSE_CAND=4
run c5 PMX_REUSE_CAND=2
run c4 PMX_COOP_MAX=0
run c4 PMX_COOP_MAX=16
