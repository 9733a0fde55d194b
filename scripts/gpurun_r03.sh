#!/bin/bash
# Round-3 measurement session: GPU tests (optional), the default bench line
# (C3 + CPU baseline + whole ICP), and the kernel-trace summary of the same
# command without the CPU baseline.  Usage: scripts/gpurun_r03.sh [tests] [quick] [bench] [configs] [vartrim] [prof] [pmc]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" | tee -a gpurun_out/steps.log; }
want() { [[ " $* " == *" all "* ]] || [[ " $ARGS " == *" $1 "* ]]; }
ARGS=" $* "
rc=0
if [[ "$ARGS" == *" tests "* ]]; then
  step tests && timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 || { tail -30 gpurun_out/tests_gpu.log; exit 1; }
  tail -3 gpurun_out/tests_gpu.log
fi
if [[ "$ARGS" == *" quick "* ]]; then
  step bench_quick && timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
  step bench_driver && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
fi
if [[ "$ARGS" == *" ab "* ]]; then
  for v in ${AB:-PMX_GRID_REUSE=0}; do
    step "bench_ab $v" && env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "gpurun_out/bench_ab_$v.json" 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
  done
fi
if [[ "$ARGS" == *" bench "* ]]; then
  step bench && timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
  step bench_driver && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { tail -20 gpurun_out/bench_driver.err; exit 1; }
fi
if [[ "$ARGS" == *" configs "* ]]; then
  for c in c2 c4 c5; do
    step bench_$c && timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  done
fi
if [[ "$ARGS" == *" vartrim "* ]]; then
  step bench_c3v && timeout -k 10 300 python bench.py --config c3v --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3v.json 2> gpurun_out/bench_c3v.err || { tail -20 gpurun_out/bench_c3v.err; exit 1; }
  step prof_c3v && (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c3v" -o run --output-format csv -- python3 "$R/bench.py" --config c3v --steps 10 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/prof_c3v.log" 2>&1) || { tail -20 gpurun_out/prof_c3v.log; exit 1; }
fi
if [[ "$ARGS" == *" prof "* ]]; then
  step prof && (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1) || { tail -20 gpurun_out/prof.log; exit 1; }
  python tools/kstats_quick.py gpurun_out/prof 24 > gpurun_out/prof_summary.txt 2>&1 || true
fi
if [[ "$ARGS" == *" pmc "* ]]; then
  # the driver command's kernel trace + FETCH_SIZE / WRITE_SIZE in separate passes -> per-phase traffic
  CMD="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --device-warmup 0.05"
  step pmc_trace && (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pmc_trace" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/pmc_trace.log" 2>&1) || exit 1
  step pmc_fetch && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/pmc_fetch.log" 2>&1) || exit 1
  step pmc_write && (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/pmc_write.log" 2>&1) || exit 1
  python tools/pmc_phases.py gpurun_out/pmc_trace gpurun_out/pmc_fetch gpurun_out/pmc_write 5 20 "python bench.py --steps 20 --warmup 5 --no-cpu-baseline" > gpurun_out/pmc_c3_driver.json 2> gpurun_out/pmc_phases.err || true
fi
step "done"
