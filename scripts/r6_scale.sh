#!/bin/bash
# Round 6: per-rank cost model (bench.py --emulate-ranks G): shard 0 of G of
# the reading on one GPU, without a communicator (local) and with RCCL at
# world size 1 under torchrun (dist).  One JSON line per (config, G, mode).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/scale
out=gpurun_out/scale/costmodel.jsonl
: > $out
for cfg in ${CFGS:-c3 c4 c5}; do for G in ${GS:-1 2 4 8}; do for mode in local dist; do
  if [ $mode = local ]; then
    timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --emulate-ranks $G > gpurun_out/scale/b.json 2> gpurun_out/scale/b.err || { tail -5 gpurun_out/scale/b.err; exit 1; }
  else
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --emulate-ranks $G --dist > gpurun_out/scale/b.json 2> gpurun_out/scale/b.err || { tail -5 gpurun_out/scale/b.err; exit 1; }
  fi
  python - "$cfg" "$G" "$mode" <<'PY' >> $out
import json, sys
d = json.loads([l for l in open("gpurun_out/scale/b.json") if l.startswith("{")][-1])
print(json.dumps({"config": sys.argv[1], "G": int(sys.argv[2]), "mode": sys.argv[3], "ms_per_step": d["ms_per_step"],
                  "whole_ms_per_iteration": d["whole_icp"]["ms_per_iteration"], "comm_timed": d.get("comm_timed"),
                  "timed_iterations": d.get("timed_iterations"), "parallelism": d["config"].get("parallelism")}))
PY
  tail -1 $out | cut -c1-200
done; done; done
