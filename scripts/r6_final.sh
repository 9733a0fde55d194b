#!/bin/bash
# Final per-config records (round 6): for each config, the PMC passes of its
# driver command first (kernel trace, FETCH_SIZE, WRITE_SIZE in separate
# rocprofv3 runs -> tools/pmc_phases.py -> profiles/r06/pmc_<cfg>_driver.json
# in this tree, which bench.py reads for `traffic`), then the bench line with
# the CPU baseline -> gpurun_out/final/bench_<cfg>.json, and the rocprofv3
# stats summary of the same command.
#   scripts/r6_final.sh c3 c2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out/final profiles/r06
export TMPDIR=/tmp
W=5; K=20
for cfg in "$@"; do
  CMD="$R/bench.py --config $cfg --steps $K --warmup $W --no-cpu-baseline"
  echo "== $(date +%T) $cfg pmc"
  rm -rf gpurun_out/final/t_$cfg gpurun_out/final/f_$cfg gpurun_out/final/w_$cfg
  (cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/final/t_$cfg" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/final/t_$cfg.log" 2>&1) || exit 1
  (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/final/f_$cfg" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/final/f_$cfg.log" 2>&1) || exit 1
  (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/final/w_$cfg" -o run --output-format csv -- python3 $CMD > "$R/gpurun_out/final/w_$cfg.log" 2>&1) || exit 1
  python3 tools/pmc_phases.py gpurun_out/final/t_$cfg gpurun_out/final/f_$cfg gpurun_out/final/w_$cfg $W $K \
      "python3 bench.py --config $cfg --steps $K --warmup $W --no-cpu-baseline" > profiles/r06/pmc_${cfg}_driver.json || exit 1
  cp profiles/r06/pmc_${cfg}_driver.json gpurun_out/final/
  cp gpurun_out/final/t_$cfg/run_kernel_stats.csv gpurun_out/final/kernel_stats_$cfg.csv
  echo "== $(date +%T) $cfg bench"
  timeout -k 10 400 python3 bench.py --config $cfg --steps $K --warmup $W > gpurun_out/final/bench_$cfg.json 2> gpurun_out/final/bench_$cfg.err || { tail -5 gpurun_out/final/bench_$cfg.err; exit 1; }
  python3 - "$cfg" <<'PY'
import json, sys
cfg = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/final/bench_{cfg}.json") if l.startswith("{")][-1])
r = d["roofline"]
print(cfg, "ms/step", round(d["ms_per_step"], 5), "whole", round(d["whole_icp"]["ms_per_iteration"], 5),
      "frac", round(r["frac"], 4), "traffic", r["traffic"], "avg_launch_ms", round(r["avg_launch_ms"], 5),
      "cpu", (d.get("cpu_baseline") or {}).get("value"), "parity", (d.get("parity") or {}).get("pass"),
      "setup", round(d.get("setup_ms", 0), 3))
PY
done
