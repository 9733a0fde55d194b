#!/bin/bash
# Round 6: A/B of the current tree against a variant library build
# (libpointmatcher_amd/lib/<variant>, PMX_LIB_VARIANT), alternating, after
# the grid / loop / config tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_grid.py tests/test_gpu_loop.py tests/test_gpu_configs.py tests/test_gpu_options.py} > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -2 gpurun_out/ab/pytest.log
fi
for rep in 1 2; do for v in "" $VARIANTS; do for cfg in ${CFGS:-c3 c4}; do
  PMX_LIB_VARIANT=$v timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -5 gpurun_out/ab/b.err; exit 1; }
  python -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); w=d['whole_icp']
print(sys.argv[2], sys.argv[3] or 'head', 'ms/step', round(d['ms_per_step'],5), 'whole', round(w['ms_per_iteration'],5), 'cold', round(w.get('cold_match_ms') or 0,4), 'match_us', round(d['roofline']['avg_launch_ms']*1e3,2), 'setup', round(d.get('setup_ms',0),3))" gpurun_out/ab/b.json $cfg "$v"
done; done; done
