#!/bin/bash
# setup timing without the trace's stream syncs (A/B: side-stream levels on / off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c3 c5; do
  for side in 1 0; do
    PMX_SIDE_LEVELS=$side timeout -k 10 300 python tools/setup_trace.py $c > gpurun_out/setup2_$c.out 2> gpurun_out/setup2_$c.err || { tail -20 gpurun_out/setup2_$c.err; exit 1; }
    echo "== $c side=$side"; grep "prepare [123]:" gpurun_out/setup2_$c.err
  done
done
