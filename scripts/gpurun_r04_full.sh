#!/bin/bash
# Full GPU test suite, smoke, then the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
step tests && timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/tests_full.log 2>&1
rc=$?
step "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step smoke && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
step bench && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc2=$?
step "done rc=$rc2"
exit $rc2
