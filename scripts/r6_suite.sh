#!/bin/bash
# Round 6: the GPU suite (single-process tests, then the multi-rank file), then
# quick C3 / C4 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/suite
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    --ignore=tests/test_gpu_multirank.py > gpurun_out/suite/suite_main.log 2>&1 || { tail -40 gpurun_out/suite/suite_main.log; exit 1; }
tail -2 gpurun_out/suite/suite_main.log
if [ -z "$NO_MULTI" ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu tests/test_gpu_multirank.py \
    > gpurun_out/suite/suite_multi.log 2>&1 || { tail -40 gpurun_out/suite/suite_multi.log; exit 1; }
tail -2 gpurun_out/suite/suite_multi.log
fi
for cfg in ${CFGS:-c3 c4}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/suite/b_$cfg.json 2> gpurun_out/suite/b_$cfg.err || { tail -5 gpurun_out/suite/b_$cfg.err; exit 1; }
  python -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); w=d['whole_icp']
print(sys.argv[2], 'ms/step', round(d['ms_per_step'],5), 'whole', round(w['ms_per_iteration'],5), 'cold', w.get('cold_match_ms'), 'setup', round(d.get('setup_ms',0),3), 'match_us', round(d['roofline']['avg_launch_ms']*1e3,2))" gpurun_out/suite/b_$cfg.json $cfg
done
