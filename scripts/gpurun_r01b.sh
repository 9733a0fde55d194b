#!/bin/bash
# GPU session: parity tests, C3 bench, 1-rank RCCL rehearsal, c4/c5 bench lines,
# HBM traffic PMC passes (FETCH_SIZE and WRITE_SIZE in separate passes).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
prof() {  # name, extra rocprofv3 args...
    local name=$1; shift
    (cd /tmp && timeout -k 10 600 rocprofv3 "$@" -d "$R/gpurun_out/$name" -o run --output-format csv \
        -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/$name.log" 2>&1)
}
step tests && timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/tests_gpu.log 2>&1 &&
step bench_c3 && timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err &&
step dist1 && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --dist --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3_dist1.json 2> gpurun_out/bench_c3_dist1.err &&
step bench_c4 && timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err &&
step bench_c5 && timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err &&
step prof_trace && prof prof_c3_trace --kernel-trace --stats &&
step pmc_fetch && prof pmc_fetch --pmc FETCH_SIZE &&
step pmc_write && prof pmc_write --pmc WRITE_SIZE
rc=$?
step "done rc=$rc"
exit $rc
