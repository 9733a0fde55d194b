#!/bin/bash
# Per-rank cost model for G = 1/2/4/8 (strong scaling of the global reading):
# one GPU runs shard 0 of G, without a communicator and with the RCCL path at
# world size 1 (--dist); ms/iteration, whole-ICP ms/iteration and the loop's
# synchronisation counters per configuration.  -> gpurun_out/costmodel.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CFGS:-c3 c4 c5}; do
  for G in 1 2 4 8; do
    for mode in local dist; do
      if [ $mode = dist ]; then
        launch="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --dist"
      else
        launch="python bench.py"
      fi
      timeout -k 10 300 $launch --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --emulate-ranks $G \
          > gpurun_out/cm_tmp.json 2>> gpurun_out/cm.err || exit 1
      python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/cm_tmp.json') if l.startswith('{')][-1]); print(json.dumps({'cfg': sys.argv[1], 'G': int(sys.argv[2]), 'mode': sys.argv[3], 'reading_per_rank': d['config']['reading_per_gpu'], 'ms_per_step': round(d['ms_per_step'],5), 'whole_ms_it': round(d['whole_icp']['ms_per_iteration'],5), 'match_ms': round(d['roofline']['avg_launch_ms'],5), 'comm_timed': d['comm_timed']}))" $cfg $G $mode | tee -a gpurun_out/costmodel.jsonl
    done
  done
done
