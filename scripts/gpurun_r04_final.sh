#!/bin/bash
# Round-4 final C3 evidence: the GPU suite, smoke, the driver's default bench
# line (with the CPU baseline and the parity block), the PMC passes of the
# driver command, and the world-size-1 RCCL rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/tests_full.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step smoke && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
step bench && timeout -k 10 500 python bench.py > gpurun_out/bench_default_cpu.json 2> gpurun_out/bench_default_cpu.err || exit 1
PMC_TAG=c3 bash scripts/gpurun_r04_pmc.sh || exit 1
step dist1 && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --dist --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err
rc=$?
step "done rc=$rc"
exit $rc
