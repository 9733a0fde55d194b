#!/bin/bash
# Same-box A/B of env variants on the driver command (interleaved, R rounds),
# then an optional kernel trace of one variant.
#   AB="A=1 B=2" R=2 PROF_ENV="PMX_GRID_REUSE=0" scripts/gpurun_ab3.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R0="$(pwd)"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for r in $(seq 1 ${R:-2}); do
  for v in base ${AB}; do
    echo "== $(date +%T) round $r $v"
    ev=""; [ "$v" != base ] && ev="$v"
    env $ev timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup ${WARM:-5} --no-cpu-baseline ${BARGS} > "gpurun_out/ab/${v}_$r.json" 2> gpurun_out/ab/err.log || { tail -20 gpurun_out/ab/err.log; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));w=d['whole_icp'];print(sys.argv[2], 'driver %.4f ms  whole %.4f ms/it  cold %.3f ms  first %s hits %d/%d' % (d['ms_per_step'], w['ms_per_iteration'], w['cold_match_ms'], w['first_matches_us'][:6], w['window_hits'], w['window_misses']))" "gpurun_out/ab/${v}_$r.json" "$v" | tee -a gpurun_out/ab/summary.txt
  done
done
if [ -n "$PROF_ENV" ]; then
  for pe in $PROF_ENV; do
    echo "== $(date +%T) prof $pe"
    ( export $pe; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R0/gpurun_out/prof_$pe" -o run --output-format csv -- python3 "$R0/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --device-warmup 0.05 > "$R0/gpurun_out/prof_$pe.log" 2>&1 ) || { tail -20 "gpurun_out/prof_$pe.log"; exit 1; }
  done
fi
echo "== done"
