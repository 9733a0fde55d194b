#!/bin/bash
# warm setup A/B: reading upload on the copy stream (1/0) x side-stream levels (1/0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rc in 1 0; do for side in 1 0; do
  PMX_READING_COPY=$rc PMX_SIDE_LEVELS=$side timeout -k 10 300 python tools/setup_trace.py c3 > gpurun_out/setup5.out 2> gpurun_out/setup5.err || { tail -20 gpurun_out/setup5.err; exit 1; }
  echo "copy=$rc side=$side"; grep "prepare [123]:" gpurun_out/setup5.err
done; done
PMX_SETUP_TRACE=2 timeout -k 10 300 python tools/setup_trace.py c3 > gpurun_out/setup5.out 2> gpurun_out/setup5t.err || exit 1
tail -13 gpurun_out/setup5t.err
