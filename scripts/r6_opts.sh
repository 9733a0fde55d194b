#!/bin/bash
# Round 6: A/B of context options (PMX_OPTS) on bench configs, alternating.
# Usage: CFGS="c4" bash scripts/r6_opts.sh "" "tile_dispatch=1" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/opts
for rep in 1 2; do for o in "$@"; do for cfg in ${CFGS:-c3 c4}; do
  PMX_OPTS="$o" timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/opts/b.json 2> gpurun_out/opts/b.err || { tail -5 gpurun_out/opts/b.err; exit 1; }
  python -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); w=d['whole_icp']
print(sys.argv[2], repr(sys.argv[3]), 'ms/step', round(d['ms_per_step'],5), 'whole', round(w['ms_per_iteration'],5), 'cold', round(w.get('cold_match_ms') or 0,4), 'first', [round(x) for x in w.get('first_matches_us',[])], 'fs', d['timed_iterations']['full_searches'][:5])" gpurun_out/opts/b.json $cfg "$o"
done; done; done
