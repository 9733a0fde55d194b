#!/bin/bash
# Round-4 batch: the full GPU suite, the VarTrimmed walk trace + c3v bench and
# PMC, the world-size-1 RCCL rehearsal, then A/Bs at C3 and C5 of the seeded
# full search (PMX_SEED=0: without) and the octant-first full search.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/tests_full.log 2>&1 || exit 1
step vt_trace && PMX_VT_TRACE=1 timeout -k 10 300 python tools/vt_trace.py 10 > gpurun_out/vt_trace.out 2> gpurun_out/vt_trace.err || exit 1
BENCH_ARGS="--config c3v" bash scripts/gpurun_r04_ab.sh BASE=1 && mv gpurun_out/ab.jsonl gpurun_out/ab_c3v.jsonl || exit 1
step dist1 && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --dist --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err || exit 1
bash scripts/gpurun_r04_ab.sh BASE=1 PMX_SEED=0 PMX_GRID_MODE=octant && mv gpurun_out/ab.jsonl gpurun_out/ab_c3.jsonl || exit 1
BENCH_ARGS="--config c5" bash scripts/gpurun_r04_ab.sh BASE=1 PMX_SEED=0 PMX_GRID_MODE=octant && mv gpurun_out/ab.jsonl gpurun_out/ab_c5.jsonl
