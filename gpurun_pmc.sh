#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group) over the match
# probe, for each grid kernel mode.  Kernel-trace/stats are collected alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
R="$(pwd)"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
step() { echo "== $(date +%T) $*" >> gpurun_out/steps.log; }
PPC=${PMC_PPC:-4}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM"
C="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
for mode in ${PMC_MODES:-tile lane}; do
  n=0
  for grp in "$A" "$B" "$C"; do
    n=$((n + 1))
    step "$mode pass $n"
    (cd /tmp && PMX_GRID_MODE=$mode PMX_GRID_PPC=$PPC timeout -k 10 300 rocprofv3 --pmc $grp -d "$R/gpurun_out/pmc/${mode}_$n" -o run \
        --output-format csv -- python3 "$R/tests/perf_probe.py" 1000000 1000000 1 3 aligned \
        > "$R/gpurun_out/pmc/${mode}_$n.log" 2>&1) || exit $?
  done
done
step done
