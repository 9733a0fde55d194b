#!/bin/bash
# Kernel traces of the match probe under environment variants (one rocprofv3
# --kernel-trace run each).  Usage: gpurun_variants.sh "NAME:ENV=V,ENV=V" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out/var
export TMPDIR=/tmp
PROBE_ARGS=${PROBE_ARGS:-"1000000 1000000 1 5 aligned"}
for spec in "$@"; do
  name=${spec%%:*}
  envs=${spec#*:}
  echo "== $(date +%T) $name ($envs)" >> gpurun_out/steps.log
  (cd /tmp && env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/var/$name" \
      -o run --output-format csv -- python3 "$R/tests/perf_probe.py" $PROBE_ARGS > "$R/gpurun_out/var/$name.log" 2>&1) || exit $?
done
echo "== $(date +%T) done" >> gpurun_out/steps.log
