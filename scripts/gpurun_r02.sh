#!/bin/bash
# Round-2 GPU session: the GPU test suite, the driver's bench command, its
# kernel trace and its HBM traffic (FETCH_SIZE / WRITE_SIZE, separate
# rocprofv3 --pmc passes).  Usage: scripts/gpurun_r02.sh [tests|bench|trace|prof|all]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
what="${1:-all}"
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
CMD=(python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5)
(grep -m1 "model name" /proc/cpuinfo; nproc; rocm-smi --showproductname 2>/dev/null | grep -i series) > gpurun_out/box.txt 2>&1
rc=0
if [ "$what" = tests ] || [ "$what" = all ]; then
  step tests && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
      > gpurun_out/tests_gpu.log 2>&1 || rc=$?
  [ $rc -ne 0 ] && { step "tests rc=$rc"; exit $rc; }
  step smoke && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
fi
if [ "$what" = bench ] || [ "$what" = all ] || [ "$what" = prof ]; then
  step bench && timeout -k 10 600 "${CMD[@]}" > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || exit $?
fi
if [ "$what" = prof ] || [ "$what" = all ] || [ "$what" = trace ]; then
  step trace && (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run \
      --output-format csv -- "${CMD[@]}" > "$R/gpurun_out/prof.log" 2>&1) || exit $?
fi
if [ "$what" = prof ] || [ "$what" = all ]; then
  step fetch && (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o run \
      --output-format csv -- "${CMD[@]}" > "$R/gpurun_out/pmc_fetch.log" 2>&1) || exit $?
  step write && (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o run \
      --output-format csv -- "${CMD[@]}" > "$R/gpurun_out/pmc_write.log" 2>&1) || exit $?
fi
step "done rc=$rc"
exit $rc
