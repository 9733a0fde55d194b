#!/bin/bash
# Round 6: reuse candidates (the pre-prune tree in wt_cand/, PMX_REUSE_CAND=K)
# on C4 / C3, alternating with K = 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}/wt_cand"
mkdir -p ../gpurun_out/cand
for rep in 1 2; do for K in ${KS:-0 5 7}; do for cfg in ${CFGS:-c4}; do
  PMX_REUSE_CAND=$K timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > ../gpurun_out/cand/b.json 2> ../gpurun_out/cand/b.err || { tail -5 ../gpurun_out/cand/b.err; exit 1; }
  python -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); w=d['whole_icp']
print(sys.argv[2], 'K', sys.argv[3], 'ms/step', round(d['ms_per_step'],5), 'whole', round(w['ms_per_iteration'],5), 'first', [round(x) for x in w.get('first_matches_us',[])], 'fs', d['timed_iterations']['full_searches'][:6])" ../gpurun_out/cand/b.json $cfg $K
done; done; done
