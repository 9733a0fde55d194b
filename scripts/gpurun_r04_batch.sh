#!/bin/bash
# Round-4 batch: VarTrimmed tests + walk trace + c3v bench and PMC, the
# world-size-1 RCCL rehearsal, then the octant-first A/B at C3 and C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step vt_tests && timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_kernels.py tests/test_gpu_icp.py tests/test_gpu_loop.py tests/test_gpu_grid.py -k "artrim or VarTrim or octant or grid" \
    > gpurun_out/vt_tests.log 2>&1 || exit 1
step vt_trace && PMX_VT_TRACE=1 timeout -k 10 300 python tools/vt_trace.py 10 > gpurun_out/vt_trace.out 2> gpurun_out/vt_trace.err || exit 1
BENCH_ARGS="--config c3v" bash scripts/gpurun_r04_ab.sh BASE=1 && mv gpurun_out/ab.jsonl gpurun_out/ab_c3v.jsonl || exit 1
PMC_TAG=c3v bash scripts/gpurun_r04_pmc.sh --config c3v || exit 1
step dist1 && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --dist --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err || exit 1
bash scripts/gpurun_r04_ab.sh BASE=1 PMX_GRID_MODE=octant && mv gpurun_out/ab.jsonl gpurun_out/ab_oct_c3.jsonl || exit 1
BENCH_ARGS="--config c5" bash scripts/gpurun_r04_ab.sh BASE=1 PMX_GRID_MODE=octant && mv gpurun_out/ab.jsonl gpurun_out/ab_oct_c5.jsonl
