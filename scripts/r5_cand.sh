#!/bin/bash
# Reuse-candidate experiment: parity first (grid / loop GPU tests with
# PMX_REUSE_CAND=4), then C5 and C3 driver benches with K = k (off) vs K.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PMX_REUSE_CAND=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_grid.py tests/test_gpu_loop.py tests/test_gpu_configs.py -k "not c4 and not c3_full" \
    > gpurun_out/cand_tests.log 2>&1 || { tail -30 gpurun_out/cand_tests.log; exit 1; }
tail -3 gpurun_out/cand_tests.log
for cfg in c5 c3; do
  for K in 0 4 2; do
    [ $cfg = c5 ] && [ $K = 2 ] && continue
    PMX_REUSE_CAND=$K timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/cand_tmp.json 2>> gpurun_out/cand.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/cand_tmp.json')); t=d['timed_iterations']; print(json.dumps({'cfg': sys.argv[1], 'K': sys.argv[2], 'ms_per_step': round(d['ms_per_step'],5), 'whole_ms_it': round(d['whole_icp']['ms_per_iteration'],5), 'first': d['whole_icp']['first_matches_us'], 'match_ms': round(d['roofline']['avg_launch_ms'],5), 'full': t['full_searches'][:6], 'levels': t['levels'][:6]}))" $cfg $K | tee -a gpurun_out/cand.jsonl
  done
done
