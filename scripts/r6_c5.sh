#!/bin/bash
# Round 6: point-to-point in one pass — loop / config / robust tests, then C5
# (and C2 as a quick check) with it on and off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c5
timeout -k 10 800 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
   tests/test_gpu_loop.py tests/test_gpu_options.py tests/test_gpu_configs.py tests/test_gpu_robust.py > gpurun_out/c5/pytest.log 2>&1 || { tail -30 gpurun_out/c5/pytest.log; exit 1; }
tail -2 gpurun_out/c5/pytest.log
for opt in p2p_onepass=1 p2p_onepass=0; do for cfg in ${CFGS:-c5}; do
  PMX_OPTS=$opt timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c5/b.json 2> gpurun_out/c5/b.err || { tail -5 gpurun_out/c5/b.err; exit 1; }
  python -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); w=d['whole_icp']
print(sys.argv[2], sys.argv[3], 'ms/step', round(d['ms_per_step'],5), 'whole', round(w['ms_per_iteration'],5), 'cold', round(w.get('cold_match_ms') or 0,4), 'match_us', round(d['roofline']['avg_launch_ms']*1e3,2))" gpurun_out/c5/b.json $cfg $opt
done; done
