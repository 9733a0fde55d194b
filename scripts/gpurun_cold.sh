#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cold
for p in 2 4 8 16 32 64; do
  echo "== $(date +%T) ppc $p" >> gpurun_out/steps.log
  timeout -k 10 300 env PMX_GRID_FIRST_PPC=$p python bench.py --no-cpu-baseline --warmup 1 --steps 40 > gpurun_out/cold/c3_$p.json 2>/dev/null || exit 1
  timeout -k 10 300 env PMX_GRID_FIRST_PPC=$p python bench.py --config c2 --no-cpu-baseline --warmup 1 --steps 40 > gpurun_out/cold/c2_$p.json 2>/dev/null || exit 1
  timeout -k 10 300 env PMX_GRID_FIRST_PPC=$p python bench.py --config c4 --no-cpu-baseline --warmup 1 --steps 40 > gpurun_out/cold/c4_$p.json 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/cold/c3_default.json 2>/dev/null
