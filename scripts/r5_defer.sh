#!/bin/bash
# deferred tile-fallback lanes: GPU tests with PMX_TILE_DEFER=1, then C3 / C5 A/B (cold match, whole ICP)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PMX_TILE_DEFER=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_grid.py tests/test_gpu_loop.py tests/test_gpu_icp.py tests/test_gpu_configs.py > gpurun_out/defer_tests.log 2>&1 || { tail -30 gpurun_out/defer_tests.log; exit 1; }
tail -1 gpurun_out/defer_tests.log
for rep in 1 2; do for cfg in c3 c5; do for on in 1 0; do
  PMX_TILE_DEFER=$on timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/defer_b.json 2> gpurun_out/defer_b.err || { tail -5 gpurun_out/defer_b.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/defer_b.json') if l.startswith('{')][-1]); w=d['whole_icp']; print(sys.argv[1], 'defer', sys.argv[2], 'ms/step', round(d['ms_per_step'],5), 'whole', round(w['ms_per_iteration'],5), 'cold', w.get('cold_match_ms'), 'first', w.get('first_matches_us', [])[:4])" $cfg $on
done; done; done
