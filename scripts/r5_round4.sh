#!/bin/bash
# step-kernel floor (PMX_STEP_NOMATH variant) from the kernel trace, then the
# per-rank cost model with the RCCL path (world size 1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base nomath wt; do
  vv=$v; [ $v = base ] && vv=""
  (cd /tmp && PMX_LIB_VARIANT=$vv timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r4_$v" -o run --output-format csv -- \
      python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/r4_$v.log" 2>&1) || exit 1
  f=$(find gpurun_out/r4_$v -name '*kernel_trace.csv' | head -1)
  echo "== $v"; python3 tools/trace_iter.py "$f" 20
done
CFGS="c3 c4" bash scripts/r5_costmodel.sh
for rep in 1 2; do for v in "" wt; do
  PMX_LIB_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4_tmp.json 2>> gpurun_out/r4.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/r4_tmp.json')); print(json.dumps({'variant': sys.argv[1], 'ms_per_step': round(d['ms_per_step'],5), 'whole_ms_it': round(d['whole_icp']['ms_per_iteration'],5), 'match_ms': round(d['roofline']['avg_launch_ms'],5)}))" "$v" | tee -a gpurun_out/r4.jsonl
done; done
