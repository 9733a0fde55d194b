#!/bin/bash
# fused finalize + step and the tile dispatch's certificate estimate: parity
# (loop / configs / icp / robust / multirank-free suites), then A/B benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_loop.py tests/test_gpu_configs.py tests/test_gpu_icp.py tests/test_gpu_robust.py \
    tests/test_gpu_icp_sequence.py > gpurun_out/r6_tests.log 2>&1 || { tail -30 gpurun_out/r6_tests.log; exit 1; }
tail -1 gpurun_out/r6_tests.log
run() {  # cfg, env...
  local cfg=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline \
      > gpurun_out/r6_tmp.json 2>> gpurun_out/r6.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/r6_tmp.json')); t=d['timed_iterations']; print(json.dumps({'cfg': sys.argv[1], 'env': sys.argv[2:], 'ms_per_step': round(d['ms_per_step'],5), 'whole_ms_it': round(d['whole_icp']['ms_per_iteration'],5), 'first': d['whole_icp']['first_matches_us'], 'match_ms': round(d['roofline']['avg_launch_ms'],5), 'full': t['full_searches'][:6]}))" $cfg "$@" | tee -a gpurun_out/r6.jsonl
}
for rep in 1 2; do run c3 PMX_FUSE_STEP=0; run c3 PMX_FUSE_STEP=1; done
run c5 PMX_TILE_DISPATCH=0
run c5 PMX_TILE_DISPATCH=-1
run c4 PMX_FUSE_STEP=0
run c4 PMX_FUSE_STEP=1
