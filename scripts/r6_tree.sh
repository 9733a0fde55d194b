#!/bin/bash
# Round 6: the cold match over the box tree — grid / config parity tests, then
# C3 / C4 / C5 benches with the tree and with the tile form (PMX_COLD_TREE=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tree
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
   tests/test_gpu_grid.py tests/test_gpu_icp.py tests/test_gpu_loop.py > gpurun_out/tree/pytest.log 2>&1 || { tail -30 gpurun_out/tree/pytest.log; exit 1; }
tail -3 gpurun_out/tree/pytest.log
for cfg in ${CFGS:-c3 c4}; do for tree in 1 0; do
  PMX_COLD_TREE=$tree timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/tree/b_${cfg}_$tree.json 2> gpurun_out/tree/b_${cfg}_$tree.err || { tail -5 gpurun_out/tree/b_${cfg}_$tree.err; exit 1; }
  python -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); w=d['whole_icp']
print(sys.argv[2], 'tree', sys.argv[3], 'ms/step', round(d['ms_per_step'],5), 'whole', round(w['ms_per_iteration'],5), 'cold', w.get('cold_match_ms'), 'first', w.get('first_matches_us'), 'setup', round(d.get('setup_ms',0),3), 'parity', (d.get('parity') or {}).get('pass'))" gpurun_out/tree/b_${cfg}_$tree.json $cfg $tree
done; done
