#!/bin/bash
# counter phase folded into the fused finalize + step (no quantile window):
# the loop / config tests, then C4 / C5 / C2 A/B against PMX_STEP_COUNTER=0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_loop.py tests/test_gpu_configs.py tests/test_gpu_icp.py tests/test_gpu_robust.py \
  > gpurun_out/sc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sc_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for cfg in c4 c5 c3; do for sc in 1 0; do
  PMX_STEP_COUNTER=$sc timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sc_b.json 2> gpurun_out/sc_b.err || { tail -5 gpurun_out/sc_b.err; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sc_b.json') if l.startswith('{')][-1]); print(sys.argv[1], 'sc', sys.argv[2], 'ms/step', round(d['ms_per_step'],5), 'whole', round(d['whole_icp']['ms_per_iteration'],5), 'parity', d.get('parity'))" $cfg $sc | tee -a gpurun_out/sc_ab.txt
done; done; done
