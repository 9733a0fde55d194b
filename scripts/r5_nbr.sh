#!/bin/bash
# neighbour-record cache: GPU tests touching the match, then C3 / C4 / C5 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_grid.py tests/test_gpu_loop.py tests/test_gpu_icp.py tests/test_gpu_configs.py tests/test_gpu_icp_sequence.py tests/test_gpu_robust.py tests/test_gpu_kernels.py > gpurun_out/nbr_tests.log 2>&1 || { tail -30 gpurun_out/nbr_tests.log; exit 1; }
tail -1 gpurun_out/nbr_tests.log
for rep in 1 2; do for cfg in c3 c4; do for on in 1 0; do
  PMX_NBR_CACHE=$on timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/nbr_b.json 2> gpurun_out/nbr_b.err || { tail -5 gpurun_out/nbr_b.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/nbr_b.json') if l.startswith('{')][-1]); print(sys.argv[1], 'nbr', sys.argv[2], 'ms/step', round(d['ms_per_step'],5), 'whole', round(d['whole_icp']['ms_per_iteration'],5), 'match', round(d['roofline']['avg_launch_ms'],5))" $cfg $on
done; done; done
