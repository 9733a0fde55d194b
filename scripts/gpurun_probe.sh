#!/bin/bash
# perf_probe.py under environment variants (no profiler).  Usage:
#   gpurun_probe.sh "NAME:ENV=V,ENV=V" ...   (PROBE_ARGS overrides the probe args)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/probe
PROBE_ARGS=${PROBE_ARGS:-"1000000 1000000 1 5 aligned"}
for spec in "$@"; do
  name=${spec%%:*}
  envs=${spec#*:}
  echo "== $(date +%T) $name ($envs)" >> gpurun_out/steps.log
  timeout -k 10 300 env $(echo "$envs" | tr ',' ' ') python tests/perf_probe.py $PROBE_ARGS > gpurun_out/probe/$name.log 2>&1 || exit $?
done
echo "== $(date +%T) done" >> gpurun_out/steps.log
