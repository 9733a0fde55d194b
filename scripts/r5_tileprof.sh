#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c3 c5; do
PMX_TILE_PROF=1 timeout -k 10 300 python tools/tile_prof.py $c 3 > gpurun_out/tileprof.out 2> gpurun_out/tileprof_$c.err || { tail -20 gpurun_out/tileprof_$c.err; exit 1; }
echo "== $c"; grep tile_prof gpurun_out/tileprof_$c.err | tail -12 | head -2
done
