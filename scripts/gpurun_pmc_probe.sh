#!/bin/bash
# One SQ PMC pass of perf_probe.py per environment variant.
#   gpurun_pmc_probe.sh "NAME:ENV=V,ENV=V" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out/pmcp
export TMPDIR=/tmp
PROBE_ARGS=${PROBE_ARGS:-"1000000 1000000 1 3 aligned"}
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"}
for spec in "$@"; do
  name=${spec%%:*}
  envs=${spec#*:}
  echo "== $(date +%T) $name ($envs)" >> gpurun_out/steps.log
  (cd /tmp && env $(echo "$envs" | tr ',' ' ') timeout -s KILL 120 rocprofv3 --pmc $CTRS -d "$R/gpurun_out/pmcp/$name" -o run --output-format csv \
     -- python3 "$R/tests/perf_probe.py" $PROBE_ARGS > "$R/gpurun_out/pmcp/$name.log" 2>&1) || exit $?
done
echo "== $(date +%T) done" >> gpurun_out/steps.log
