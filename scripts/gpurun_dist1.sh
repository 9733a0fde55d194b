#!/bin/bash
# torchrun / RCCL rehearsal of the multi-rank bench path on one GPU (world 1, --dist).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --dist --no-cpu-baseline > gpurun_out/bench_c3_dist1.json 2> gpurun_out/bench_c3_dist1.err
