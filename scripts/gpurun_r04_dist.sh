#!/bin/bash
# Sharded-path checks on one GPU: the two-rank (gloo) GPU tests incl. the
# forced-miss replay, the ICPSequence tests, and the RCCL world-size-1
# rehearsal of the bench (stall-and-replay timing).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 1000 python -u -m pytest -v --timeout 900 --timeout-method thread \
    tests/test_gpu_multirank.py tests/test_gpu_icp_sequence.py tests/test_gpu_loop.py tests/test_gpu_knn_wide.py tests/test_gpu_normals.py tests/test_gpu_robust.py "tests/test_gpu_kernels.py::test_vartrimmed_parallel_partial_sum" > gpurun_out/tests_dist.log 2>&1 &&
step dist1 && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --dist --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err &&
step single && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_single.json 2> gpurun_out/bench_single.err
rc=$?
step "done rc=$rc"
exit $rc
