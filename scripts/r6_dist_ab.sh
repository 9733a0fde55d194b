#!/bin/bash
# Round 6: per-rank cost model (dist, RCCL at world size 1) of the current
# tree against a variant library (PMX_LIB_VARIANT), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dab
for rep in 1 2; do for v in "" $VARIANTS; do for G in ${GS:-1 8}; do
  PMX_LIB_VARIANT=$v timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --config ${CFG:-c3} --steps 20 --warmup 5 --no-cpu-baseline --emulate-ranks $G --dist > gpurun_out/dab/b.json 2> gpurun_out/dab/b.err || { tail -5 gpurun_out/dab/b.err; exit 1; }
  python -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2] or 'head', 'G', sys.argv[3], 'ms/step', round(d['ms_per_step'],5), d.get('comm_timed'))" gpurun_out/dab/b.json "$v" $G
done; done; done
